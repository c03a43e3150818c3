// Internal types shared by the host library (capi.cpp) and the kernels
// (tg_kernels.hip). Not part of the public ABI.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "../../include/hyg_model.h"

namespace hyg {

constexpr int kDefaultThreads = 256;     // forward workgroup size
constexpr int kDefaultThreadsBwd = 256;  // backward workgroup size (HYG_THREADS[_FWD/_BWD] override)
// forward / backward workgroup size when a launch has at most one chain per CU
// (tg_kernels.hip threads_per_chain; HYG_LOWOCC_THREADS overrides both): the
// backward's list phase keeps 12 waves busy (768: 546 vs 558 ms at 145 chains,
// r03x), the forward is faster at 512 (1327 vs 1377 ms)
constexpr int kLowOccThreads = 512;
constexpr int kLowOccThreadsBwd = 768;
constexpr int kEBlock = 8;     // emission rows staged in LDS per block of steps

// Device-side chain descriptor (lives in the workspace header).
struct ChainDev {
  int64_t site_begin;
  int64_t out_begin;
  int64_t ws_offset;  // byte offset of the chain's history records
  uint64_t seed;
  uint64_t chain_id;
  int32_t T;
  int32_t pad;
  int64_t wg_offset;  // byte offset of the backward's full-N weight scratch (Nmax f64; backward_global_w)
};

// Per-step history record: scalars, then M packed parent states, then M
// parent weights. Written by the forward kernel, read by the backward kernel.
struct StepScalars {
  int32_t mode;   // 0 keep, 1 optimal, 2 unbiased, 3 init
  int32_t n_par;
  float log_c;
  int32_t r_ph;
  double lse;
  double pad;
};
static_assert(sizeof(StepScalars) == 32, "record scalars");
// (the backward kernel reads them as dwords: mode 0, n_par 1, log_c 2, r_ph 3, lse 4-5)
static_assert(offsetof(StepScalars, n_par) == 4 && offsetof(StepScalars, log_c) == 8 &&
                  offsetof(StepScalars, r_ph) == 12 && offsetof(StepScalars, lse) == 16,
              "record scalar dwords");

#if defined(__HIPCC__)
__host__ __device__
#endif
inline size_t record_bytes(int M) { return sizeof(StepScalars) + (size_t)M * 16; }

struct ModelDev {
  const hyg_tg_consts* consts;  // device copy
  const double* hz;             // [2][K][dcap][2]
  int32_t dcap;
  int32_t nmax_reads;
  const double* lf;   // [nmax+1]
  const double* lg;   // [K][3][nmax+1]
  const double* cst;  // [K]
  const double* bbt;  // per-(n, y) terms [(nmax+1)(nmax+2)/2][K] (hyg_bb_term_table), or null when too large
};

struct FwdLayout {  // LDS carve of the forward kernel (byte offsets)
  size_t W, keys, mass, pst, pw, phz, ering, cp, misc, total;
  int npad, nsort;
};

// Launchers (tg_kernels.hip)
int launch_emission(const ModelDev& md, const hyg_tg_consts& c, const uint16_t* meth_c, const uint16_t* tot_c,
                    int s_c, const uint16_t* meth_k, const uint16_t* tot_k, int s_k, int64_t n_sites,
                    double* E, void* stream);
int launch_chains(const ModelDev& md, const hyg_tg_consts& c, const ChainDev* chains_dev, int n_chains,
                  const double* E, uint8_t* ws, const hyg_tg_outputs& out, void* stream);
size_t forward_lds_bytes(const hyg_tg_consts& c, int n_chains);
void set_kernel_timing(bool on);
int last_kernel_ms(float* out3);
size_t backward_lds_bytes(const hyg_tg_consts& c, int n_chains);
int tg_threads_per_chain(const hyg_tg_consts& c, int n_chains);  // forward workgroup size of a launch
int tg_force_threads(int fwd, int bwd);                           // test override (0 = automatic)
int tg_resident_per_cu(const hyg_tg_consts& c, int n_chains);     // forward workgroups per CU
void tg_set_tail_overlap(bool on);                                // hyg_tg_set_tail_overlap
int tg_device_cus(int dev);                                       // CUs of a device as the launcher sees them
int tg_set_device_cus(int dev, int cus);                          // test override (0 = query the device)
size_t tg_layout_bytes(const hyg_tg_consts& c, int threads, bool backward);  // LDS of one chain (0: bad width)
// Whether a model's backward keeps its full-N weights (the general path and the
// final step's draw) in a per-chain global scratch of Nmax f64 instead of LDS,
// so that its LDS holds several chains per CU (the C5 shape); the workspace
// then carries n_chains * backward_scratch_bytes(c) more bytes.
bool backward_global_w(const hyg_tg_consts& c);
inline size_t backward_scratch_bytes(const hyg_tg_consts& c) {
  return backward_global_w(c) ? ((size_t)c.Nmax * sizeof(double) + 255) / 256 * 256 : 0;
}

}  // namespace hyg
