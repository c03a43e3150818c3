// Internal types of the single-group path shared by capi.cpp and
// sg_kernels.hip (not part of the public ABI).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "../../include/hyg_sg_model.h"
#include "../../include/hyg_sg_pe.h"

namespace hyg {

constexpr int kSgThreads = 256;         // one particle per thread: N_max <= 256
constexpr int kSgPsiCapDefault = 4096;  // pending smoothing times per chain
constexpr int kSgRngSystematic = 5;     // Philox stream of the systematic uniform

struct SgModelDev {
  const hyg_sg_consts* consts;  // device copy
  const double* hz;             // [K][dcap][2]: log rho, log(1 - rho) | -inf
  const uint8_t* ex;            // [K][dcap] exit status
  int32_t dcap;
  int32_t nmax_reads;
  const double* lf;             // BB tables as hyg_sg_bb_tables
  const double* lg;
  const double* cst;
  uint64_t key_keep;            // the packed log-weight sort's key bits (~0xff; hyg_sg_force_key_drop)
};

struct SgChainDev {
  int64_t site_begin;
  int64_t out_begin;
  int64_t psi_offset;  // byte offset of the chain's smoothing slots in the workspace
  int64_t ring_offset; // byte offset of the chain's step-record ring (SMC workgroup -> smoothing workgroup)
  int64_t ctl_offset;  // byte offset of the chain's ring control words (zeroed before each launch)
  uint64_t seed;
  uint64_t chain_id;
  int32_t T;
  int32_t rcap;        // parameter estimation: hazard rows per regime
  int64_t pe_offset;   // parameter estimation: byte offset of the chain's region
  int64_t theta_row;   // parameter estimation: first output row of theta
};

// Online parameter estimation (include/hyg_sg_pe.h), model-level inputs
struct SgPeDev {
  hyg_sgpe_consts c;
  const double* theta0;        // [dim] initial theta
  const hyg_sgpe_step* steps;  // [n] step sizes / bias corrections per update
  const double* lgk;           // [K][lgk_stride] theta-free part of the NegBin log-pmf
  const double* dgk;           // [K][lgk_stride] psi(x + kappa) - psi(kappa) (kappa estimated), else null
  int32_t lgk_stride;
  int32_t pad;
  double* theta_out;           // [rows][c.dim]
};

// Per-chain region of the estimation path: phi [2][256][K^2] (the kappa
// coordinates' score is identically 0, include/hyg_sg_pe.h), theta, ADAM
// moments, previous / current score [K (K + 1)] each, hazard rows [K][rcap],
// and the rebuild scratch h, g, gk, bigH[d-1], gradBigH[d-1] [K][rcap] f64 +
// exit [K][rcap] u8.
__host__ __device__ inline size_t sg_pe_region_bytes(int K, int rcap) {
  const size_t dim = (size_t)K * K, dth = (size_t)K * (K + 1);
  const size_t b = 8 * (2 * (size_t)kSgThreads * dim + 5 * dth) + 32 * (size_t)K * rcap + 40 * (size_t)K * rcap +
                   (size_t)K * rcap;
  return (b + 255) / 256 * 256;
}

// The SMC of a chain runs in one workgroup and its online marginal smoothing
// in a second one (sg_kernels.hip): per step the SMC workgroup publishes a
// record {N, N_prev, M, t | ancestor + regime [256] u64 | weights [256] f64 |
// backward kernels [K][256] f64} into a ring of kSgRing slots in the
// workspace, the smoothing workgroup consumes it.
constexpr int kSgRing = 32;
__host__ __device__ inline size_t sg_rec_bytes(int K) {
  return (16 + 8 * 2 * (size_t)kSgThreads + 8 * (size_t)K * kSgThreads + 255) / 256 * 256;
}
constexpr size_t kSgCtlBytes = 16;  // per chain: head (records published), tail (consumed), abort code, and
                                    // (first chain of a launch) the launch's dispatch-ticket counter

// Per-chain workspace: cap psi slots [K][256] f64, then the pending-time lists
// slot[2][cap] / time[2][cap] (double-buffered), keep[cap], free[cap] (int32),
// then the step-record ring.
__host__ __device__ inline size_t sg_psi_region_bytes(int K, int cap) {
  return ((sizeof(double) * (size_t)K * kSgThreads * (size_t)cap) + 255) / 256 * 256;
}
__host__ __device__ inline size_t sg_lists_bytes(int cap) {
  return ((sizeof(int32_t) * 6 * (size_t)cap) + 255) / 256 * 256;
}
__host__ __device__ inline size_t sg_chain_ws_bytes(int K, int cap) {
  return sg_psi_region_bytes(K, cap) + sg_lists_bytes(cap) + (size_t)kSgRing * sg_rec_bytes(K);
}

int sg_launch_emission(const SgModelDev& md, const hyg_sg_consts& c, const uint16_t* meth, const uint16_t* tot,
                       int S, int64_t n_sites, double* E, void* stream);
// ctl: the chains' ring control words (kSgCtlBytes each, contiguous), zeroed here before the launches
int sg_force_key_drop(int bits);  // test override of the packed sort's dropped key bits (0 = 8)
int sg_launch_chains(const SgModelDev& md, const hyg_sg_consts& c, const SgChainDev* chains_dev, int n_chains,
                     const double* E, uint8_t* ws, int psi_cap, double* probs, int32_t* status, void* ctl,
                     void* stream, const SgPeDev* pe = nullptr);
size_t sg_lds_bytes(const hyg_sg_consts& c, int psi_cap, bool pe = false);

}  // namespace hyg
