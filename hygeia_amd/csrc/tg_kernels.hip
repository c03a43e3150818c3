// tg_kernels.hip -- CDNA4 (gfx950) kernels of the two-group change-point path.
//
//   tg_emission_kernel   per-site Beta-Binomial emission table (HBM streaming)
//   tg_forward_kernel    particle filter with optimal finite-state resampling,
//                        one workgroup per chain, persistent over the T sites
//   tg_backward_kernel   backward simulation of B trajectories, one workgroup
//                        per chain, regenerating each step's particles from the
//                        forward's ancestor history (read one step ahead)
//
// Every index decision uses the arithmetic contract of include/hyg_arith.h
// (exact integer mass sums, deterministic exp/log, Philox streams), so the
// results are bit-identical to the CPU oracle (oracle/tg_oracle.c) whatever the
// reduction tree; that freedom is what the kernels use to parallelise.
//
// Latency design (one chain = a sequential recursion of ~110k steps, so the
// per-step critical path is what matters): model constants and hazard rows
// are read from LDS (hazard rows of the next step's ancestors are prefetched
// one step ahead), the resampling sort runs in registers / wave shuffles with
// LDS only for cross-wave stages, the K / log c search runs in one wave with
// 64-way probes, and reductions are fused to two block barriers per step.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <mutex>
#include <vector>

#include "../../include/hyg_arith.h"
#include "tg_common.h"
#include "hyg_dev.h"  // wave / block primitives (DPP, readlane, LDS-only barriers)

namespace hyg {

enum { MODE_KEEP = 0, MODE_OPTIMAL = 1, MODE_UNBIASED = 2, MODE_INIT = 3 };

// Wave priority of the single-wave serial sections (the K loop + systematic
// draws, the backward's one-wave categorical): while one wave of a chain works
// alone, the others wait at a barrier, so its issue slots are the chain's
// critical path; the other chains sharing the CU fill the gaps.
#ifndef HYG_SERIAL_PRIO
#define HYG_SERIAL_PRIO 1
#endif
__device__ __forceinline__ void serial_begin() {
  if constexpr (HYG_SERIAL_PRIO > 0) __builtin_amdgcn_s_setprio(HYG_SERIAL_PRIO);
}
__device__ __forceinline__ void serial_end() {
  if constexpr (HYG_SERIAL_PRIO > 0) __builtin_amdgcn_s_setprio(0);
}


// sort key: ascending key == descending f32 value, ties by ascending index
__device__ __forceinline__ uint64_t sort_key(float x, int idx) {
  uint32_t u = hyg_f32_bits(x);
  if (u == 0x80000000u) u = 0;
  const uint32_t ord = (u >> 31) ? ~u : (u | 0x80000000u);
  return ((uint64_t)(~ord) << 32) | (uint32_t)idx;
}
__device__ __forceinline__ float key_value(uint64_t k) {
  const uint32_t ord = ~(uint32_t)(k >> 32);
  const uint32_t u = (ord & 0x80000000u) ? (ord & 0x7fffffffu) : ~ord;
  return hyg_bits_f32(u);
}
__device__ __forceinline__ int key_index(uint64_t k) { return (int)(uint32_t)k; }

// n / d for 0 <= n < 2^22, 1 <= d <= 2^22, via a float reciprocal + fixup
__device__ __forceinline__ int fdiv(int n, int d, float rd) {
  int q = (int)((float)n * rd);
  if (q * d > n) --q;
  if ((q + 1) * d <= n) ++q;
  return q;
}

// hyg_exp_fix100(x[i]) (= hyg_fix100(hyg_exp(x[i])), include/hyg_arith.h) for R
// values at once, written statement by statement across the values: the same
// operations in the same order per value (so the same bits), but the R
// dependent f64 chains sit side by side in the instruction stream. Written as
// one function per value, the compiler schedules the chains one after another
// and every f64 operation waits for its predecessor's result. The image is
// formed from the polynomial value and the exponent by shifts (no scaling by
// 2^k, no float floors).
template <int R>
__device__ __forceinline__ void exp_fix100_lockstep(const double (&x)[R], hyg_u128 (&out)[R]) {
  double xc[R], kd[R], r[R], r2[R], r4[R], r8[R], p[R];
  int k[R];
#pragma unroll
  for (int i = 0; i < R; ++i) xc[i] = __builtin_fmin(__builtin_fmax(x[i], -746.0), 710.0);
#pragma unroll
  for (int i = 0; i < R; ++i) kd[i] = __builtin_floor(xc[i] * HYG_INV_LN2 + 0.5);
#pragma unroll
  for (int i = 0; i < R; ++i) {
    k[i] = (int)kd[i];
    const double hi = xc[i] - kd[i] * HYG_LN2_HI;
    r[i] = __builtin_fma(-kd[i], HYG_LN2_LO, hi);
  }
#pragma unroll
  for (int i = 0; i < R; ++i) r2[i] = r[i] * r[i];
#pragma unroll
  for (int i = 0; i < R; ++i) r4[i] = r2[i] * r2[i];
#pragma unroll
  for (int i = 0; i < R; ++i) r8[i] = r4[i] * r4[i];
#pragma unroll
  for (int i = 0; i < R; ++i) {  // hyg__exp_poly, statement by statement
    const double q0 = __builtin_fma(1.0, r[i], 1.0);
    const double q1 = __builtin_fma(1.6666666666666665741e-01, r[i], 0.5);
    const double q2 = __builtin_fma(8.3333333333333332177e-03, r[i], 4.1666666666666664354e-02);
    const double q3 = __builtin_fma(1.9841269841269841253e-04, r[i], 1.3888888888888888889e-03);
    const double q4 = __builtin_fma(2.7557319223985890653e-06, r[i], 2.4801587301587301566e-05);
    const double q5 = __builtin_fma(2.5052108385441718775e-08, r[i], 2.7557319223985890653e-07);
    const double q6 = __builtin_fma(1.6059043836821614599e-10, r[i], 2.0876756987868098979e-09);
    const double s0 = __builtin_fma(q1, r2[i], q0);
    const double s1 = __builtin_fma(q3, r2[i], q2);
    const double s2 = __builtin_fma(q5, r2[i], q4);
    const double u0 = __builtin_fma(s1, r4[i], s0);
    const double u1 = __builtin_fma(q6, r4[i], s2);
    p[i] = __builtin_fma(u1, r8[i], u0);
  }
#pragma unroll
  for (int i = 0; i < R; ++i) out[i] = hyg_exp_fix100_pk(p[i], k[i], x[i]);
}

// --------------------------------------------------------------- model
struct Hz4 {
  double lrc, l1c, lrk, l1k;  // log rho / log(1-rho) of control (d_c, r_c) and case (d_k, r_k)
};

struct ConstLds {  // model constants staged in LDS
  double lPm[4];
  double lU1, lU2, log_M;
  double2 hz1[2][HYG_KMAX];  // hazard rows at d = 1
  float logMa[64];           // (float)log(M - a) for a < min(M, 64) (resampling_functions.py:13)
  int u, K;
  double lPc[HYG_KMAX * HYG_KMAX];  // last: only K*K entries are allocated (const_lds_bytes)
};
__host__ __device__ inline size_t const_lds_bytes(int K) {
  return sizeof(ConstLds) - sizeof(double) * (size_t)(HYG_KMAX * HYG_KMAX - K * K);
}

__device__ __forceinline__ double2 hz_at(const ModelDev& md, int K, int g, int r, int d) {
  d = d < 0 ? 0 : (d >= md.dcap ? md.dcap - 1 : d);
  return *(const double2*)(md.hz + ((size_t)(g * K + r) * md.dcap + d) * 2);
}

__device__ __forceinline__ void load_consts(ConstLds& cl, const hyg_tg_consts* __restrict__ c, const ModelDev& md) {
  const int K = c->K;
  for (int i = threadIdx.x; i < K * K; i += blockDim.x) cl.lPc[i] = c->lPc[i];
  if (threadIdx.x < 4) cl.lPm[threadIdx.x] = c->lPm[threadIdx.x];
  if (threadIdx.x < 2 * K) {
    const int g = threadIdx.x / K, r = threadIdx.x - g * K;
    cl.hz1[g][r] = hz_at(md, K, g, r, 1);
  }
  if (threadIdx.x < 64 && threadIdx.x < c->M) cl.logMa[threadIdx.x] = hyg_logf((float)(c->M - (int)threadIdx.x));
  if (threadIdx.x == 0) {
    cl.lU1 = c->lU1;
    cl.lU2 = c->lU2;
    cl.log_M = c->log_M;
    cl.u = c->u;
    cl.K = K;
  }
}

// log f_t(next | prev), t >= 1 (case_control_regime_model.py:80-193,
// case_control_distributions.py:138-151, 246-291); h = hazard of prev.
// Same branch structure and addition order as oracle/tg_oracle.c:tg_trans.
__device__ __forceinline__ double tg_trans_sel(double lPm_j, double lpc, double lU1, double lU2, int u, int m,
                                               int dc, int rc, int dk, int rk, uint64_t next, const Hz4& h);
__device__ __forceinline__ double tg_trans(const ConstLds& cl, int K, uint64_t prev, uint64_t next, const Hz4& h) {
  const int m = hyg_st_m(prev), dc = hyg_st_dc(prev), rc = hyg_st_rc(prev), dk = hyg_st_dk(prev),
            rk = hyg_st_rk(prev);
  const int m2 = hyg_st_m(next), rc2 = hyg_st_rc(next);
  return tg_trans_sel(cl.lPm[m * 2 + m2], cl.lPc[rc * K + rc2], cl.lU1, cl.lU2, cl.u, m, dc, rc, dk, rk, next, h);
}

// The case analysis of tg_trans as selects: every operand is loaded and every
// candidate sum formed unconditionally (no divergent branches, no loads under
// a lane condition); the selected value is the same expression, so results
// are bit-identical.
__device__ __forceinline__ double tg_trans_sel(double lPm_j, double lpc, double lU1, double lU2, int u, int m,
                                               int dc, int rc, int dk, int rk, uint64_t next, const Hz4& h) {
  const double NINF = HYG_NINF;
  const int m2 = hyg_st_m(next), dc2 = hyg_st_dc(next), rc2 = hyg_st_rc(next), dk2 = hyg_st_dk(next),
            rk2 = hyg_st_rk(next);
  const double lm = ((dk < dc ? dk : dc) >= u) ? lPm_j : ((m2 == m) ? 0.0 : NINF);
  const double lc_cp = h.lrc + lpc;
  const double lc = (dc2 == 1) ? lc_cp : ((dc2 == dc + 1 && rc2 == rc) ? h.l1c : NINF);
  const double v1 = (rk2 == rc2 && dk2 == dc2) ? 0.0 : NINF;
  const double v23 = (dk2 == 1 && rk2 != rc2) ? lU1 : NINF;
  const double lk_cp = h.lrk + ((rc2 == rk) ? lU1 : lU2);
  const double v4a = (rk2 != rc2 && rk2 != rk) ? lk_cp : NINF;
  const double v4b = (dk2 == dk + 1 && rk2 == rk) ? h.l1k : NINF;
  const double v4 = (dk2 == 1) ? v4a : v4b;
  const double lk = (m2 == 1) ? v1 : ((m == 1 && dc2 != 1) ? v23 : ((rc2 == rk && m == 0) ? v23 : v4));
  return (lm + lc) + lk;
}

// proposal slot s of ancestor a (case_control_proposal_mappings.py:11-134)
__device__ __forceinline__ uint64_t tg_xi(int K, uint64_t a, int s) {
  const int m = hyg_st_m(a), dc = hyg_st_dc(a), rc = hyg_st_rc(a), dk = hyg_st_dk(a), rk = hyg_st_rk(a);
  if (s == 0) return hyg_st_pack(m, dc + 1, rc, dk + 1, rk);
  if (s < K) {
    const int r = (s - 1 < rk) ? s - 1 : s;
    return hyg_st_pack(0, 1, r, dk + 1, rk);
  }
  if (s < 2 * K - 1) {
    const int q = s - K;
    const int r = (q < rc) ? q : q + 1;
    return hyg_st_pack(0, dc + 1, rc, 1, r);
  }
  if (s == 2 * K - 1) {
    const int d = (m == 0) ? dc + 1 : 0;
    return hyg_st_pack(1, d, rc, d, rc);
  }
  const int j = s - 2 * K, i = j / K, jj = j - i * K;
  return hyg_st_pack(i == jj, 1, i, 1, jj);
}
__device__ __forceinline__ uint64_t init_state(int K, int n) {
  const int i = n / K, j = n - (n / K) * K;
  return hyg_st_pack(i == j, 1, i, 1, j);
}

// Hazard rows a child may need, prefetched per ancestor: control at
// (d_c + 1, r_c), case at (d_k + 1, r_k), case at (d_c + 1, r_c) (merge slot).
struct Pf3 {
  double2 c1, k1, kc;
};
__device__ __forceinline__ Pf3 prefetch_rows(const ModelDev& md, int K, uint64_t a) {
  Pf3 p;
  const int dc = hyg_st_dc(a), rc = hyg_st_rc(a);
  p.c1 = hz_at(md, K, 0, rc, dc + 1);
  p.k1 = hz_at(md, K, 1, hyg_st_rk(a), hyg_st_dk(a) + 1);
  p.kc = hz_at(md, K, 1, rc, dc + 1);
  return p;
}
// Hazards of the child in slot s of ancestor a (the rows of the child's own
// durations/regimes), from the ancestor's prefetched rows and the d = 1 rows.
__device__ __forceinline__ Hz4 child_hz(const ConstLds& cl, int K, uint64_t a, int s, const Pf3& p,
                                        const ModelDev& md) {
  Hz4 h;
  const uint64_t x = tg_xi(K, a, s);
  // s == 0: both durations continue; s < K: control changes; s < 2K-1: case
  // changes; s == 2K-1 with m = 0: merge (case continues on the control row);
  // m = 1 there: the merge slot's child (1, 0, r, 0, r) has weight -inf, is
  // never resampled and never becomes an ancestor, so its hazards are unused.
  // Value selects (a select of addresses would put p in scratch memory).
  const double2 h1c = cl.hz1[0][hyg_st_rc(x)], h1k = cl.hz1[1][hyg_st_rk(x)];
  const bool merge = (s == 2 * K - 1) && hyg_st_m(a) == 0;
  const bool c_cont = s == 0 || (s >= K && s < 2 * K - 1) || merge;
  const bool k_cont = s < K;
  h.lrc = c_cont ? p.c1.x : h1c.x;
  h.l1c = c_cont ? p.c1.y : h1c.y;
  h.lrk = merge ? p.kc.x : (k_cont ? p.k1.x : h1k.x);
  h.l1k = merge ? p.kc.y : (k_cont ? p.k1.y : h1k.y);
  return h;
}

// tg_xi + child_hz without divergent branches (slot s varies per lane in
// the gather): every slot type's child is formed and the right one selected.
__device__ __forceinline__ uint64_t tg_xi_hz_sel(const ConstLds& cl, int K, float rK, uint64_t a, int s,
                                                 const Pf3& p, Hz4* hout) {
  const int m = hyg_st_m(a), dc = hyg_st_dc(a), rc = hyg_st_rc(a), dk = hyg_st_dk(a), rk = hyg_st_rk(a);
  const int rB = (s - 1 < rk) ? s - 1 : s;
  const int qq = s - K, rC = (qq < rc) ? qq : qq + 1;
  const int dD = (m == 0) ? dc + 1 : 0;
  const int j = s - 2 * K;
  int i = (int)((float)(j > 0 ? j : 0) * rK);
  if (i * K > j) --i;
  if ((i + 1) * K <= j) ++i;
  const int jj = j - i * K;
  const bool tA = s == 0, tB = s < K, tC = s < 2 * K - 1, tD = s == 2 * K - 1;
  int xm, xdc, xrc, xdk, xrk;
  if (tA) { xm = m; xdc = dc + 1; xrc = rc; xdk = dk + 1; xrk = rk; }
  else if (tB) { xm = 0; xdc = 1; xrc = rB; xdk = dk + 1; xrk = rk; }
  else if (tC) { xm = 0; xdc = dc + 1; xrc = rc; xdk = 1; xrk = rC; }
  else if (tD) { xm = 1; xdc = dD; xrc = rc; xdk = dD; xrk = rc; }
  else { xm = (i == jj); xdc = 1; xrc = i; xdk = 1; xrk = jj; }
  // hazard rows: prefetched rows where the duration continues, d = 1 rows at a change
  const bool c_cont = tA || (!tB && tC) || (tD && m == 0);
  const bool k_cont = tA || (tB && !tA);
  // (value selects: a select of the address would put p in scratch memory)
  const double2 h1c = cl.hz1[0][xrc], h1k = cl.hz1[1][xrk];
  const bool kc = tD && m == 0;
  hout->lrc = c_cont ? p.c1.x : h1c.x;
  hout->l1c = c_cont ? p.c1.y : h1c.y;
  hout->lrk = kc ? p.kc.x : (k_cont ? p.k1.x : h1k.x);
  hout->l1k = kc ? p.kc.y : (k_cont ? p.k1.y : h1k.y);
  return hyg_st_pack(xm, xdc, xrc, xdk, xrk);
}

// ------------------------------------------------------------ LDS layout
constexpr int kPh = 36;  // diagnostic phase timers (last entry: timestamp / step count)

struct Shared {  // broadcast scalars of one workgroup
  double mx, logS;
  float c_new, log_c;
  int cnt, n_sig, Kk, status, r_ph, ng, fast;
  float Unext;  // systematic-resampling uniform of the next step, drawn during the gather
  unsigned sig_ctr;
  hyg_u192 R, preK;
  int segc[16];  // backward: finite logits per reachable slot (segment list)
  unsigned long long ph[kPh];
};

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
__host__ __device__ inline int next_pow2(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

constexpr int kBuckets = 512;  // counting-sort buckets of the resampling sort (sqrt-spaced in -lw)
constexpr int kNCut = 8;       // log-weight cutoffs of the top-set resampling path
// candidate-list entries per lane per chunk (lse / top-set gather): ~900 list
// entries at C3 are ~3.5 per lane at 256 threads, under one at 1024
#ifndef HYG_LR256
#define HYG_LR256 4
#endif
#ifndef HYG_LR512
#define HYG_LR512 2
#endif
template <int NT>
constexpr int kLRof = NT >= 768 ? 2 : (NT >= 512 ? HYG_LR512 : HYG_LR256);
// waves that sort the top set A: at most 256 keys (one per lane of 4 waves)
// whatever the workgroup size, so a 512- or 1024-thread chain sorts no more
// keys than a 256-thread one (HYG_SORT_WAVES overrides, for tuning builds)
#ifndef HYG_SORT_WAVES
#define HYG_SORT_WAVES 4
#endif
// top_set_finish1 (the latency-shaped finish of the top-set path) where its
// scratch fits; 0 selects top_set_finish everywhere (A/B builds)
#ifndef HYG_TSF1
#define HYG_TSF1 1
#endif
template <int NT>
constexpr int kSortWaves = (NT / 64 < HYG_SORT_WAVES) ? NT / 64 : HYG_SORT_WAVES;

struct Lay {  // byte offsets into the dynamic LDS (32-bit: one SGPR each in the kernels)
  uint32_t W, L, keys, bcnt, bpos, pre64, part, cp, pst, pw, phz, pf, ering, cl, parents, X, grp, gst, rb, xo, red,
      sh, uring, total;
  uint32_t bcnt_bytes;
  int npad, nkeys, nt;
  int topset_r;  // keys per lane of the top-set sort: A holds <= 64 * topset_r per wave
  int lcap;      // backward: doubles of the list / logit area at W (Nmax, or the lists alone with gw)
};

// The backward's list area without the full-N weights (gw): the segment lists
// (16 slots x 64 logits, then 64 u128 masses and 64 indices), or an appended
// list of up to 4 (NT + 1) logits (its indices in the cp area), or 64 logits
// and their masses: doubles.
__host__ __device__ constexpr int bwd_list_doubles(int NT) {
  return (64 * 16 + 128 + 32) > 4 * (NT + 1) ? (64 * 16 + 128 + 32) : 4 * (NT + 1);
}

__host__ __device__ inline Lay make_layout(int K, int M, int B, int Nmax, int NT, bool backward, bool gw = false) {
  // Sized for 3 workgroups per CU at K = 6, M = 50, NT = 256 (<= 53 KiB each).
  Lay l{};
  l.nt = NT;
  l.topset_r = 1;
  l.npad = Nmax;
  l.lcap = (backward && gw && bwd_list_doubles(NT) < Nmax) ? bwd_list_doubles(NT) : Nmax;
  size_t o = 0;
  l.W = o; o = align_up(o + sizeof(double) * (backward ? l.lcap : l.npad), 16);
  if (backward) {
    // the backward's list / logit area is the weight area: the list path
    // builds no weights and the general path turns the weights into logits
    // in place
    l.L = l.W;
    l.cp = o; o = align_up(o + sizeof(hyg_u128) * (NT + 1), 16);
  } else {
    // sort keys; the unbiased fallback reuses them as its (NT+1) x u128 prefix array
    size_t kb = sizeof(uint64_t) * (size_t)Nmax;
    if (kb < sizeof(hyg_u128) * (size_t)(NT + 1)) kb = sizeof(hyg_u128) * (size_t)(NT + 1);
    l.nkeys = (int)(kb / sizeof(uint64_t));
    l.keys = o; o = align_up(o + kb, 16);
    // bucket counts / positions; the systematic thresholds (M x u192) reuse them
    size_t bb = sizeof(int) * 2 * kBuckets;
    if (bb < sizeof(hyg_u192) * (size_t)M) bb = sizeof(hyg_u192) * (size_t)M;
    l.bcnt = o;
    l.bpos = o + sizeof(int) * kBuckets;
    l.bcnt_bytes = bb;
    o = align_up(o + bb, 16);
    // the fallback's prefix of the first min(M, 64) sorted positions: written
    // after the counting sort's last use of the bucket area, last read before
    // the systematic thresholds are written there (a barrier apart)
    l.pre64 = l.bcnt;
    // per-wave partials of the top-set resampling path (counts per cutoff, mass)
    l.part = o; o = align_up(o + (sizeof(int) * kNCut + sizeof(hyg_u192)) * (NT / 64), 16);
  }
  // the ancestors of the current step, two buffers: the forward gathers the
  // next step's ancestors into the other buffer while this step's are read;
  // the backward holds record t in buffer t & 1 while record t-1 is stored
  // into the other. (The forward's hazard-row prefetch pf is written after
  // the weights, which do not read it: one buffer.)
  l.pst = o; o = align_up(o + sizeof(uint64_t) * M * 2, 16);
  l.pw = o; o = align_up(o + sizeof(double) * M * 2, 16);
  l.phz = o; o = align_up(o + sizeof(Hz4) * M * 2, 16);
  l.pf = o; o = align_up(o + sizeof(Pf3) * M * (backward ? 2 : 1), 16);
  l.ering = o; o = align_up(o + sizeof(double) * 2 * kEBlock * 2 * K, 16);
  l.cl = o; o = align_up(o + const_lds_bytes(K), 16);
  l.parents = o; o = align_up(o + sizeof(int) * (M > B ? M : B), 16);
  if (backward) {
    l.X = o; o = align_up(o + sizeof(uint64_t) * B, 16);
    l.grp = o; o = align_up(o + sizeof(int) * B, 16);
    l.gst = o; o = align_up(o + sizeof(uint64_t) * B, 16);
    l.rb = o; o = align_up(o + 2 * sizeof(uint64_t) * ((B + 3) / 4) * 4, 16);  // draw bits, two steps
    l.xo = o; o = align_up(o + 2 * sizeof(uint64_t) * B, 16);  // sampled states of two steps (deferred outputs)
  }
  l.red = o; o = align_up(o + 2 * 32 * (NT / 64), 16);  // two slots: the step's log-sum-exp has its own
  l.sh = o; o = align_up(o + sizeof(Shared), 16);
  // the forward's systematic uniforms of the next 64 steps, drawn 64 at a time
  // (NT >= 512: one chain per CU); 32 at 256 threads, whose three chains per CU
  // leave the layout ~240 B of LDS
  l.uring = o;
  if (!backward && NT >= 256) o = align_up(o + sizeof(float) * (NT >= 512 ? 64 : 32), 16);
  l.total = o;
  return l;
}

// ---------------------------------------------------------- shared steps
// Emission rows live in a 2 x kEBlock ring: row t at ring[((t/EB)&1)*EB + t%EB].
__device__ __forceinline__ void load_eblock(double* ering, const double* __restrict__ Ech, int bi, int T, int K2,
                                            int NT) {
  const int t0 = bi * kEBlock;
  if (t0 >= T) return;
  const int rows = (T - t0) < kEBlock ? (T - t0) : kEBlock;
  double* dst = ering + (size_t)(bi & 1) * kEBlock * K2;
  for (int i = threadIdx.x; i < rows * K2; i += NT) dst[i] = Ech[(size_t)t0 * K2 + i];
}
__device__ __forceinline__ const double* erow(const double* ering, int t, int K2) {
  return ering + ((size_t)((t / kEBlock) & 1) * kEBlock + (t % kEBlock)) * K2;
}

// Weight of the child in slot s of ancestor a at a step t >= 1, from the
// ancestors (pst, pw, phz) and the step scalars (_filter_one_step :235-270).
__device__ __forceinline__ double weight_at(const ConstLds& cl, int K, int a, int s, int mode, float log_c,
                                            double lse, const uint64_t* pst, const double* pw, const Hz4* phz,
                                            const double* Et) {
  const uint64_t par = pst[a];
  const uint64_t x = tg_xi(K, par, s);
  const double tr = tg_trans(cl, K, par, x, phz[a]);
  if (!hyg_isfinite(tr)) return HYG_NINF;
  const double lg = tr + (Et[hyg_st_rc(x)] + Et[K + hyg_st_rk(x)]);
  const double pa = pw[a];
  if (mode == MODE_KEEP) return pa + lg;
  if (mode == MODE_UNBIASED) return (-cl.log_M + lse) + lg;
  const double v = (double)log_c + (pa - lse);
  return (pa + lg) - (v < 0.0 ? v : 0.0);
}
// Weight of particle n = s * np + a.
__device__ __forceinline__ double weight_one(const ConstLds& cl, int K, int n, int np, int mode, float log_c,
                                             double lse, const uint64_t* pst, const double* pw, const Hz4* phz,
                                             const double* Et) {
  const int s = fdiv(n, np, 1.0f / (float)np), a = n - s * np;
  return weight_at(cl, K, a, s, mode, log_c, lse, pst, pw, phz, Et);
}

// Scalars of the transition density held in registers by gen_weights.
struct TransRegs {
  double lPm0, lPm1, lPm2, lPm3, lU1, lU2;
  int u;
};

// tg_trans with the ancestor decoded in registers (same operands, same
// addition order, so bit-identical); lPc stays in LDS.
__device__ __forceinline__ double tg_trans_r(const TransRegs& q, const double* __restrict__ lPc, int K, int m,
                                             int dc, int rc, int dk, int rk, uint64_t next, const Hz4& h) {
  const int m2 = hyg_st_m(next), rc2 = hyg_st_rc(next);
  const int j = m * 2 + m2;
  const double lPm_j = j == 0 ? q.lPm0 : (j == 1 ? q.lPm1 : (j == 2 ? q.lPm2 : q.lPm3));
  return tg_trans_sel(lPm_j, lPc[rc * K + rc2], q.lU1, q.lU2, q.u, m, dc, rc, dk, rk, next, h);
}

// All weights of a step t >= 1; returns this thread's max and count of finite weights.
// With np <= 64 every wave keeps one ancestor per lane in registers and walks
// the proposal slots s = wave, wave + NT/64, ... (slot-uniform control flow);
// otherwise one candidate per thread through weight_one.
template <int NT>
__device__ __forceinline__ void gen_weights(const ConstLds& cl, int K, int I, int np, int mode, float log_c,
                                            double lse, const uint64_t* __restrict__ pst,
                                            const double* __restrict__ pw, const Hz4* __restrict__ phz,
                                            const double* __restrict__ Et, double* __restrict__ W, double* m_out,
                                            int* c_out) {
  const int N = I * np;
  double m = HYG_NINF;
  int cnt = 0;
  if (np <= 64) {
    constexpr int NW = NT / 64;
    const int lane = lane_id(), wv = wave_id();
    TransRegs q;
    q.lPm0 = cl.lPm[0]; q.lPm1 = cl.lPm[1]; q.lPm2 = cl.lPm[2]; q.lPm3 = cl.lPm[3];
    q.lU1 = cl.lU1; q.lU2 = cl.lU2; q.u = cl.u;
    const double* __restrict__ lPc = cl.lPc;
    if (lane < np) {
      const uint64_t par = pst[lane];
      const double pa = pw[lane];
      const Hz4 h = phz[lane];
      const int am = hyg_st_m(par), adc = hyg_st_dc(par), arc = hyg_st_rc(par), adk = hyg_st_dk(par),
                ark = hyg_st_rk(par);
      // w = (base + lg) - sub reproduces the three branches of weight_one exactly
      double base = pa, sub = 0.0;
      if (mode == MODE_UNBIASED) base = -cl.log_M + lse;
      if (mode == MODE_OPTIMAL) {
        const double v = (double)log_c + (pa - lse);
        sub = v < 0.0 ? v : 0.0;
      }
      // tg_trans of every proposal slot with the child substituted
      // (case_control_proposal_mappings.py:11-134): the per-ancestor parts
      // once, per slot only what the slot changes. Same operands and the same
      // addition order as tg_trans, so the weights are bit-identical.
      const double NINF = HYG_NINF;
      const bool ok = (adk < adc ? adk : adc) >= q.u;
      const int j00 = am * 2;
      const double lPm_s = j00 == 0 ? q.lPm0 : q.lPm3;  // m' = m
      const double lm0 = ok ? (am ? q.lPm2 : q.lPm0) : (am == 0 ? 0.0 : NINF);
      const double lm1 = ok ? (am ? q.lPm3 : q.lPm1) : (am == 1 ? 0.0 : NINF);
      const double lmA = ok ? lPm_s : 0.0;
      const double* __restrict__ lPcr = lPc + arc * K;  // row r_c of log P_ctrl
      const double lcA = (adc + 1 == 1) ? (h.lrc + lPcr[arc]) : h.l1c;  // d_c' = d_c + 1, r_c' = r_c
      const double lkB = (adk == 0) ? NINF : h.l1k;
      const double lkA = am == 1 ? ((ark == arc && adk == adc) ? 0.0 : NINF) : (arc == ark ? NINF : lkB);
      const bool condC = (am == 1 && adc + 1 != 1) || (arc == ark && am == 0);
      const double lkC_cp = h.lrk + ((arc == ark) ? q.lU1 : q.lU2);
      const int dD = (am == 0) ? adc + 1 : 0;  // merge slot: both groups at d
      const double lcD = (dD == 1) ? (h.lrc + lPcr[arc]) : ((dD == adc + 1) ? h.l1c : NINF);
      const double Ec_rc = Et[arc], Ek_rk = Et[K + ark];
      auto put = [&](int s, double tr, double e) {
        double w = NINF;
        if (hyg_isfinite(tr)) w = (base + (tr + e)) - sub;
        W[s * np + lane] = w;
        m = dmax(m, w);
        cnt += (w > NINF) ? 1 : 0;
      };
      const int K2 = 2 * K;
      // Slot loops with trip counts fixed by K (compile-time in the
      // shape-specialised kernels, so they unroll and the LDS reads of later
      // slots issue ahead of earlier slots' arithmetic); s is wave-uniform.
#pragma unroll
      for (int k = 0; k < (K2 + NW - 1) / NW; ++k) {  // slot types A-D
        const int s = wv + k * NW;
        if (s >= K2) break;
        if (s == 0) {
          put(0, (lmA + lcA) + lkA, Ec_rc + Ek_rk);
        } else if (s < K) {  // control change to r != r_k
          const int r = (s - 1 < ark) ? s - 1 : s;
          put(s, (lm0 + (h.lrc + lPcr[r])) + lkB, Et[r] + Ek_rk);
        } else if (s < K2 - 1) {  // case change to r != r_c
          const int qq = s - K;
          const int r = (qq < arc) ? qq : qq + 1;
          const double lk = condC ? q.lU1 : ((r != ark) ? lkC_cp : NINF);
          put(s, (lm0 + lcA) + lk, Ec_rc + Et[K + r]);
        } else {  // merge
          put(s, (lm1 + lcD) + 0.0, Ec_rc + Et[K + arc]);
        }
      }
      // two change points (i, j): x = (i == j, 1, i, 1, j), from the wave's
      // first slot >= 2K
      const int s0 = wv + NW * ((K2 - wv + NW - 1) / NW);
#pragma unroll
      for (int k = 0; k < (I - K2 + NW - 1) / NW; ++k) {
        const int s = s0 + k * NW;
        if (s >= I) break;
        const int ii = (s - K2) / K, jj = (s - K2) - ii * K;
        const double e = Et[ii] + Et[K + jj];
        const double lc = h.lrc + lPcr[ii];
        double lk;
        if (ii == jj) lk = 0.0;
        else if (ii == ark && am == 0) lk = q.lU1;
        else lk = (jj != ark) ? (h.lrk + ((ii == ark) ? q.lU1 : q.lU2)) : NINF;
        put(s, (((ii == jj) ? lm1 : lm0) + lc) + lk, e);
      }
    }
    *m_out = m;
    *c_out = cnt;
    return;
  }
  for (int n = threadIdx.x; n < N; n += NT) {
    const double w = weight_one(cl, K, n, np, mode, log_c, lse, pst, pw, phz, Et);
    W[n] = w;
    m = dmax(m, w);
    cnt += (w > HYG_NINF) ? 1 : 0;
  }
  *m_out = m;
  *c_out = cnt;
}
template <int NT>
__device__ __forceinline__ void gen_weights_init(const ConstLds& cl, int K, int r_ph, const double* Et, double* W,
                                                 double* m_out, int* c_out) {
  double m = HYG_NINF;
  int cnt = 0;
  for (int n = threadIdx.x; n < K * K; n += NT) {
    const int i = n / K, j = n - (n / K) * K;
    const double obs = Et[i] + Et[K + j];
    const double tr = (i == j) ? cl.lPc[r_ph * K + i] : HYG_NINF;
    const double w = obs + tr;
    W[n] = w;
    m = dmax(m, w);
    cnt += (w > HYG_NINF) ? 1 : 0;
  }
  *m_out = m;
  *c_out = cnt;
}

// log of the exact F=100 mass sum of exp(W - mx) over W[0..N).
template <int NT>
__device__ __forceinline__ double log_mass_sum(const double* W, int N, double mx, unsigned char* red) {
  hyg_u128 s = hyg_u128_zero();
#pragma unroll 4
  for (int n = threadIdx.x; n < N; n += NT) {
    const double x = W[n] - mx;
    s = hyg_u128_add(s, hyg_exp_fix100(x));  // exp(x < -70) < 2^-100 -> 0
  }
  const hyg_u128 S = block_sum128<NT>(s, red);
  return hyg_log(hyg_u128_to_f64(S, 100));
}

// Categorical draws (tfd.Categorical(logits).sample with TF's multinomial CDF
// semantics): for each active draw q with random bits rnd(q), the first n with
// cdf_n > floor(u * total). logit(n) is recomputed on demand.
template <int NT, typename LogitFn, typename ActiveFn, typename RandFn, typename OutFn>
__device__ __forceinline__ void categorical_block(int N, double lmax, LogitFn logit, int n_draw, ActiveFn active,
                                                  RandFn rnd, OutFn out, hyg_u128* cp, unsigned char* red) {
  const int cs = (N + NT - 1) / NT;
  const int p0 = threadIdx.x * cs, p1 = (p0 + cs < N) ? p0 + cs : N;
  hyg_u128 loc = hyg_u128_zero();
  for (int n = p0; n < p1; ++n) {
    const double x = logit(n) - lmax;
    loc = hyg_u128_add(loc, hyg_exp_fix100(x));
  }
  block_scan128<NT>(loc, cp, red);
  lds_barrier();
  const hyg_u128 total = cp[NT];
  for (int q = threadIdx.x; q < n_draw; q += NT) {
    if (!active(q)) continue;
    const hyg_u128 target = hyg_scale_target(rnd(q), total);
    int lo = 0, hi = NT - 1;  // last chunk with cp[ch] <= target
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (hyg_u128_lt(target, cp[mid])) hi = mid - 1; else lo = mid;
    }
    int sel = -1;
    for (int ch = lo; ch < NT && sel < 0; ++ch) {
      hyg_u128 cdf = cp[ch];
      const int a0 = ch * cs, a1 = (a0 + cs < N) ? a0 + cs : N;
      for (int n = a0; n < a1; ++n) {
        const double x = logit(n) - lmax;
        cdf = hyg_u128_add(cdf, hyg_exp_fix100(x));
        if (hyg_u128_lt(target, cdf)) { sel = n; break; }
      }
    }
    out(q, sel < 0 ? N - 1 : sel);
  }
}

// ------------------------------------------------------ optimal resampling
// OptimalFiniteState (resampling_functions.py:7-52) on the significant
// log-weights (weights below sig_thresh have zero f32 mass and can
// never be counted by the K search):
//  1. counting sort: buckets by a monotone map of the f32 value, then each key
//     is ranked inside its bucket; the sorted order is unique (value desc,
//     index asc), so the bucket map only affects speed;
//  2. exact 192-bit mass prefix sums of the sorted masses;
//  3. the K / log c loop (:12-23): log c(a) and the prefix count P(c(a)) are
//     evaluated for every a < M at once (one lane per a), then the loop's
//     iterates a' = max(a, P(c(a))) are followed;
//  4. the systematic residual draw (:32-40, :56-69): target j lands on the
//     first residual position with C >= ceil(T_j R) (exact), found by the
//     thread whose chunk of sorted positions contains it.
// Writes parents[0..M) and sh.Kk / sh.log_c (log_c not finite -> caller
// runs the unbiased fallback). Returns n_sig via sh.n_sig.
template <int NT>
__device__ __forceinline__ void optimal_resample(const double* W, uint64_t* sorted, int N, double mx, double logS, float thr,
                                 uint64_t* keys, int* bcnt, int* bpos, hyg_u192* pre64, hyg_u192* tau, int* parents,
                                 Shared& sh,
                                 const ConstLds& cl, unsigned char* red, int M, int cnt_fin, uint64_t seed,
                                 uint64_t chain_id, int t, float Usys, unsigned long long* ph, bool timed) {
  const int tid = threadIdx.x;
#define SPH(k)                                                     \
  if (timed && tid == 0) {                                         \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    ph[k] += now_ - ph[kPh - 1];                                        \
    ph[kPh - 1] = now_;                                                 \
  }
  // any monotone map works (the order inside a bucket is resolved exactly);
  // sqrt spacing puts narrow buckets where the weights crowd, near the top
  const float scale = 1.0f / (-thr);
  auto bucket_of = [&](float lw) -> int {
    const int q = (int)(__builtin_sqrtf((-lw) * scale) * (float)kBuckets);
    return q < kBuckets - 1 ? q : kBuckets - 1;
  };
  // ---- 1a. bucket histogram
  for (int i = tid; i < kBuckets; i += NT) bcnt[i] = 0;
  lds_barrier();
  #pragma unroll 4
  for (int n = tid; n < N; n += NT) {
    const double w = W[n];
    if (w > HYG_NINF) {
      const float lw = (float)((w - mx) - logS);
      if (lw >= thr) atomicAdd(&bcnt[bucket_of(lw)], 1);
    }
  }
  lds_barrier();
  SPH(17);
  // ---- 1b. bucket starts (exclusive scan), kBuckets / NT buckets per thread
  {
    constexpr int PB = (kBuckets + NT - 1) / NT;
    int loc = 0;
    for (int i = 0; i < PB; ++i) {
      const int q = tid * PB + i;
      if (q < kBuckets) loc += bcnt[q];
    }
    int tot;
    int run = block_excl_int<NT>(loc, red, &tot);
    for (int i = 0; i < PB; ++i) {
      const int q = tid * PB + i;
      if (q < kBuckets) { bpos[q] = run; run += bcnt[q]; }
    }
    if (tid == 0) sh.n_sig = tot;
  }
  lds_barrier();
  SPH(18);
  const int n_sig = sh.n_sig;
  // ---- 1c. scatter into buckets (arbitrary order inside a bucket)
  #pragma unroll 4
  for (int n = tid; n < N; n += NT) {
    const double w = W[n];
    if (w > HYG_NINF) {
      const float lw = (float)((w - mx) - logS);
      if (lw >= thr) keys[atomicAdd(&bpos[bucket_of(lw)], 1)] = sort_key(lw, n);
    }
  }
  lds_barrier();
  SPH(19);
  // ---- 1d. rank every key inside its bucket and place it in `sorted` (the
  //          W area: every read of W is done); bpos now holds the bucket ends
  for (int p = tid; p < n_sig; p += NT) {
    const uint64_t k = keys[p];
    const int q = bucket_of(key_value(k));
    const int end = bpos[q], beg = end - bcnt[q];
    int rank = 0;
#pragma unroll 4
    for (int i = beg; i < end; ++i) rank += (keys[i] < k) ? 1 : 0;
    sorted[beg + rank] = k;
  }
  lds_barrier();
  SPH(13);
  // ---- 2. masses and exact prefix sums over contiguous chunks of sorted positions
  const int cs = (n_sig + NT - 1) / NT;
  const int p0 = tid * cs;
  const int p1 = (p0 + cs < n_sig) ? p0 + cs : n_sig;
  hyg_u192 loc = hyg_u192_zero();
  // the f32 masses of this thread's chunk stay in registers for the prefix,
  // the K search and the systematic walk (chunks longer than kMR recompute)
  constexpr int kMR = 8;
  float mreg[kMR];
  const bool inreg = cs <= kMR;
  if (inreg) {
#pragma unroll
    for (int i = 0; i < kMR; ++i) {
      const int p = p0 + i;
      mreg[i] = 0.0f;
      if (p < p1) mreg[i] = hyg_expf(key_value(sorted[p]));
    }
#pragma unroll
    for (int i = 0; i < kMR; ++i) loc = hyg_u192_add(loc, hyg_fix149f(mreg[i]));
  } else {
    for (int p = p0; p < p1; ++p) loc = hyg_u192_add(loc, hyg_fix149f(hyg_expf(key_value(sorted[p]))));
  }
  auto mass_at = [&](int p) -> float {  // mass of sorted position p of this thread's chunk
    if (inreg) {
      float v = 0.0f;
#pragma unroll
      for (int i = 0; i < kMR; ++i) v = (p - p0 == i) ? mreg[i] : v;
      return v;
    }
    return hyg_expf(key_value(sorted[p]));
  };
  hyg_u192 total;
  const hyg_u192 myex = block_excl192<NT>(loc, red, &total);
  const int npre = M < 64 ? M : 64;  // pre64 holds min(M, 64) entries (make_layout)
  if (p0 < npre) {  // inclusive prefix of the first npre sorted positions
    hyg_u192 run = myex;
    for (int p = p0; p < p1 && p < npre; ++p) {
      run = hyg_u192_add(run, hyg_fix149f(mass_at(p)));
      pre64[p] = run;
    }
  }
  lds_barrier();
  SPH(14);
  // ---- 3. K / log c (loop-variable semantics of :12-31)
  if (wave_id() == 0) {
    const int lane = lane_id();
    if (M <= 64) {
      // lane a: c(a) and the prefix count P(c(a)) = #{p : fl(c(a) + x_p) > 0}
      int Pa = 0;
      float ca = 0.0f;
      hyg_u192 rva = hyg_u192_zero();
      const int a = lane;
      if (a < M && a < N) {
        if (a < n_sig) rva = hyg_u192_sub(total, a == 0 ? hyg_u192_zero() : pre64[a - 1]);
        const double rvd = hyg_u192_to_f64(rva);
        const float l2 = (rvd == 0.0) ? HYG_NINFF : (float)hyg_log(rvd);
        ca = cl.logMa[a] - l2;
        if (hyg_isfinitef(ca)) {
          int lo = 0, hi = n_sig;  // first p with the predicate false
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((float)(ca + key_value(sorted[mid])) > 0.0f) lo = mid + 1; else hi = mid;
          }
          Pa = lo;
        } else if (ca > 0.0f) {
          Pa = cnt_fin;  // +inf: every finite particle
        } else {
          Pa = 0;
        }
      }
      // follow a <- max(a, P(c(a))) from a = 0 (the body runs at least once)
      int aa = 0, bb = -1;
      while (aa != bb && aa < N && aa < M) {
        const int nxt = __builtin_amdgcn_readlane(Pa, aa);
        bb = aa;
        aa = nxt > aa ? nxt : aa;
      }
      const float lc = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ca), bb));
      hyg_u192 R;
      R.w0 = rdlane64(rva.w0, bb);
      R.w1 = rdlane64(rva.w1, bb);
      R.w2 = rdlane64(rva.w2, bb);
      if (lane == 0) {
        sh.Kk = bb;
        sh.log_c = lc;
        sh.R = R;
        sh.preK = hyg_u192_sub(total, R);
      }
    } else {
      // general M: the loop as written, one iteration at a time
      int a = 0, b = -1;
      float lc = -1.0f;
      hyg_u192 rv_last = hyg_u192_zero();
      while (a != b && a < N && a < M) {
        hyg_u192 rv = hyg_u192_zero();
        if (a < n_sig) {
          hyg_u192 pre = hyg_u192_zero();
          if (a > 0 && a <= 64) pre = pre64[a - 1];
          else if (a > 64) {
            pre = pre64[63];
            for (int p = 64; p < a; ++p) pre = hyg_u192_add(pre, hyg_fix149f(hyg_expf(key_value(sorted[p]))));
          }
          rv = hyg_u192_sub(total, pre);
        }
        const double rvd = hyg_u192_to_f64(rv);
        const float l1 = hyg_logf((float)(M - a));
        const float l2 = (rvd == 0.0) ? HYG_NINFF : (float)hyg_log(rvd);
        const float cn = l1 - l2;
        int cnt = 0;
        if (hyg_isfinitef(cn)) {
          int lo = 0, hi = n_sig;
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((float)(cn + key_value(sorted[mid])) > 0.0f) lo = mid + 1; else hi = mid;
          }
          cnt = (lo - a) > 0 ? lo - a : 0;
        } else if (cn > 0.0f) {
          cnt = (cnt_fin - a) > 0 ? cnt_fin - a : 0;
        }
        b = a;
        a = a + cnt;
        lc = cn;
        rv_last = rv;
      }
      if (lane == 0) {
        sh.Kk = b;
        sh.log_c = lc;
        sh.R = rv_last;
        sh.preK = hyg_u192_sub(total, rv_last);
      }
    }
  }
  lds_barrier();
  SPH(15);
  int Kk = sh.Kk;
  const float log_c = sh.log_c;
  if (Kk >= N || !hyg_isfinitef(log_c)) return;  // caller runs the unbiased fallback
  // ---- 4. deterministic top-K, systematic residual with exact thresholds
  const int L = M - Kk;
  const float U = Usys;  // hyg_u01f(hyg_rand64(seed, chain_id, HYG_RNG_SYSTEMATIC, t, 0)), drawn ahead
  const float Lf = (float)L;
  const hyg_u192 R = sh.R, preK = sh.preK;
  for (int j = tid; j < L; j += NT) {
    tau[j] = hyg_u192_add(preK, hyg_ceil_mul_f32_bf(((float)j + U) / Lf, R));
    parents[Kk + j] = key_index(sorted[Kk]);  // unfilled -> residual index 0
  }
  for (int p = tid; p < Kk; p += NT) parents[p] = key_index(sorted[p]);
  lds_barrier();
  if (p0 < n_sig && p0 + cs > Kk && L > 0) {
    // first target not reached before this chunk: #{j : tau_j <= C(p0 - 1)}
    int j = 0;
    if (p0 > Kk) {
      int lo = 0, hi = L;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (hyg_u192_ge(myex, tau[mid])) lo = mid + 1; else hi = mid;
      }
      j = lo;
    }
    hyg_u192 C = myex;
    for (int p = p0; p < p1 && j < L; ++p) {
      C = hyg_u192_add(C, hyg_fix149f(mass_at(p)));
      if (p >= Kk) {
        while (j < L && hyg_u192_ge(C, tau[j])) {
          parents[Kk + j] = key_index(sorted[p]);
          ++j;
        }
      }
    }
  }
  SPH(16);
#undef SPH
}

// ------------------------------------------- resampling: the top-set path
// OptimalFiniteState touches the order of the largest log-weights only: the
// K / log c search reads the prefix masses of the first a < M sorted weights
// and counts #{p : fl(c + x_p) > 0}, and the systematic targets land where
// the cumulative residual mass crosses them (at C3 the deepest draw sits near
// sorted rank 300 of ~900 significant weights). This path sorts exactly only
// the top set A = {lw >= cut} for the most inclusive of kNCut cutoffs whose
// set fits one block bitonic sort (<= 128 keys per wave), takes the total
// mass of every significant weight from an order-free exact sum, and then
// checks with exact quantities that each index decision falls inside A:
//   - every K-loop probe the loop visits has its prefix and its count in A;
//   - the last systematic target lies at or below the mass of A.
// If a check fails the caller runs the full counting-sort path
// (optimal_resample), so the parents are those of the full sort either way.
enum { FAST_DONE = 0, FAST_FALLBACK = 1, FAST_FALLBACK_REGEN = 2 };
#define TPH(k)                                                     \
  if (timed && threadIdx.x == 0) {                                 \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    ph[k] += now_ - ph[kPh - 1];                                   \
    ph[kPh - 1] = now_;                                            \
  }

// cutoffs of the top set in W - mx (nats below the largest weight); the last
// set (k = kNCut - 1) is the whole candidate list (W - mx >= sig_thresh)
__host__ __device__ constexpr double cut_below_top(int k) {
  // selects, not a table: a runtime index into a local array is a memory load
  return k < 4 ? (k < 2 ? (k == 0 ? 14.0 : 17.0) : (k == 2 ? 20.0 : 23.0))
               : (k < 6 ? (k == 4 ? 26.0 : 30.0) : 36.0);
}

// The narrow (u128) images of the top set's outside masses: from cutoff
// kNarrowCut on, every outside mass is below e^-cut, and a lane sums at most
// kNarrowPerLane of them; their images m 2^149 must sum below 2^128, i.e.
// cut > ln(kNarrowPerLane 2^21) = 19.41 nats for 128 entries per lane.
constexpr int kNarrowCut = 2;
constexpr int kNarrowPerLane = 128;
static_assert(kNarrowPerLane <= 128 && cut_below_top(kNarrowCut) >= 19.5,
              "u128 outside-mass images: 128 masses below e^-19.5 sum below 2^128 at scale 2^149");

// Lanes l of a wave whose key keeps the minimum at stage (KK, J) of the
// bitonic sort below, for J in [R, 64R) and the wave bit of i clear
template <int R, int J, int KK>
constexpr uint64_t keep_min_pattern() {
  uint64_t m = 0;
  for (int l = 0; l < 64; ++l) {
    const bool a = (l & (J / R)) == 0;
    const bool b = (KK < 64 * R) ? ((l & (KK / R)) == 0) : true;
    if (a == b) m |= 1ull << l;
  }
  return m;
}

// One compare-exchange stage (k, j) of a bitonic sort of 64*NW*R keys held
// R per lane, key index i = wave*64R + lane*R + r (ascending result).
// j < R: inside the lane; j < 64R: lane xor shuffles; else: LDS + barrier.
template <int NT, int R, int KK, int J>
__device__ __forceinline__ void bitonic_stage(uint64_t (&e)[R], uint64_t* buf, int& ib) {
  constexpr int n = 64 * (NT / 64) * R;
  const int base = (int)(threadIdx.x >> 6) * 64 * R + lane_id() * R;
  if constexpr (J < R) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int pr = r ^ J;
      if (pr > r) {
        const bool up = ((base + r) & KK) == 0;
        const uint64_t a = e[r], b = e[pr];
        const bool sw = up ? (a > b) : (a < b);
        e[r] = sw ? b : a;
        e[pr] = sw ? a : b;
      }
    }
  } else if constexpr (J < 64 * R) {
    // keep_min = ((i & J) == 0) == ((i & KK) == 0) for i = wave 64R + lane R + r
    // is a constant lane pattern (J, and KK < 64R, select lane bits; KK >= 64R a
    // wave bit): the exchange is the compare's lane mask xnor that pattern
    constexpr uint64_t pat = keep_min_pattern<R, J, KK>();
    const bool wflip = (KK >= 64 * R) && (((wave_id() * 64 * R) & KK) != 0);  // wave-uniform
    const uint64_t keep = wflip ? ~pat : pat;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t o = xshfl64<J / R>(e[r]);
      const uint64_t lt = wave_ballot(o < e[r]);
      e[r] = lane_select64(~(keep ^ lt), e[r], o);
    }
  } else {
    uint64_t* b = buf + (ib & 1) * n;  // alternate buffers: one barrier per stage
    ++ib;
#pragma unroll
    for (int r = 0; r < R; ++r) b[base + r] = e[r];
    lds_barrier();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int i = base + r;
      const uint64_t o = b[i ^ J];
      const bool keep_min = ((i & J) == 0) == ((i & KK) == 0);
      const bool lt = o < e[r];
      e[r] = (keep_min == lt) ? o : e[r];
    }
  }
}
template <int NT, int R, int KK, int J>
struct Bitonic {
  __device__ static __forceinline__ void run(uint64_t (&e)[R], uint64_t* buf, int& ib) {
    bitonic_stage<NT, R, KK, J>(e, buf, ib);
    if constexpr (J > 1) Bitonic<NT, R, KK, J / 2>::run(e, buf, ib);
    else if constexpr (KK < 64 * (NT / 64) * R) Bitonic<NT, R, 2 * KK, KK>::run(e, buf, ib);
  }
};
// The order of Bitonic<64 NSW, 1, 2, 1> (ascending) of distinct keys, one per
// lane of the first NSW waves, by ranks: each wave sorts its 64 keys ascending
// (the network's stages KK <= 64, every wave in the final direction), the
// runs meet in buf[0, 64 NSW), and each key's position is its rank, the sum
// over the runs of the keys below it (its lane in its own run; a 7-probe
// binary search in the others, interleaved); buf[64 NSW, 128 NSW) receives the
// sorted keys. Two barriers and 21 in-wave stages in place
// of the network's three cross-wave stages and 33 in-wave stages. The other
// waves of the workgroup pass the same barriers and run `idle` between them.
template <int J, int KK>
__device__ __forceinline__ void rank_sort_stage(uint64_t& e) {
  constexpr uint64_t pat = keep_min_pattern<1, J, KK>();  // KK = 64: every wave as wave 0 (ascending)
  const uint64_t o = xshfl64<J>(e);
  const uint64_t lt = wave_ballot(o < e);
  e = lane_select64(~(pat ^ lt), e, o);
}
template <int J, int KK>
struct RankRuns {
  __device__ static __forceinline__ void run(uint64_t& e) {
    rank_sort_stage<J, KK>(e);
    if constexpr (J > 1) RankRuns<J / 2, KK>::run(e);
    else if constexpr (KK < 64) RankRuns<KK, 2 * KK>::run(e);
  }
};
template <int NSW, class Idle>
__device__ __forceinline__ uint64_t rank_sort_asc(uint64_t e, uint64_t* buf, bool sorter, Idle idle) {
  const int base = (int)(threadIdx.x >> 6) * 64 + lane_id();
  if (sorter) {
    RankRuns<1, 2>::run(e);
    buf[base] = e;
  }
  lds_barrier();
  if (!sorter) {
    idle();
  } else {
    int pos[NSW];
#pragma unroll
    for (int r = 0; r < NSW; ++r) pos[r] = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1) {
#pragma unroll
      for (int r = 0; r < NSW; ++r) pos[r] += (buf[64 * r + pos[r] + step - 1] < e) ? step : 0;
    }
    int rank = 0;
#pragma unroll
    for (int r = 0; r < NSW; ++r) rank += pos[r] + ((buf[64 * r + pos[r]] < e) ? 1 : 0);
    buf[64 * NSW + rank] = e;
  }
  lds_barrier();
  return sorter ? buf[64 * NSW + base] : e;
}

// workgroup barriers of a bitonic sort of n keys held R per lane (one per
// cross-wave stage): the waves of a larger workgroup that take no part in the
// sort pass the same number of barriers
constexpr int bitonic_lds_stages(int n, int R) {
  int c = 0;
  for (int kk = 2; kk <= n; kk *= 2)
    for (int j = kk / 2; j >= 1; j /= 2) c += (j >= 64 * R) ? 1 : 0;
  return c;
}

// Sort A (nA keys in srt[]), exact prefix masses, the K / log c loop and the
// systematic draws. scr: the W + key areas (W is overwritten). The sort runs on
// the first NSW waves (64 NSW R keys); the other waves of the workgroup only
// pass its barriers.
template <int NT, int NSW, int R>
__device__ __forceinline__ int top_set_finish(uint64_t* srt, int nA, bool hasB, int N, int M, int cnt_fin, const hyg_u192& massB,
                              unsigned char* scr, int* parents, Shared& sh, const ConstLds& cl, unsigned char* red,
                              float Usys, unsigned long long* ph, bool timed) {
  static_assert(NSW <= NT / 64, "sorting waves");
  const int lane = lane_id();
  const bool sorter = (NSW == NT / 64) || wave_id() < NSW;  // wave-uniform
  const int base = (int)(threadIdx.x >> 6) * 64 * R + lane * R;
  uint64_t e[R];
  hyg_u192 f[R];
  hyg_u192 loc = hyg_u192_zero();
  if (sorter) {
#pragma unroll
    for (int r = 0; r < R; ++r) e[r] = (base + r < nA) ? srt[base + r] : ~0ull;
    int ib = 0;
    Bitonic<64 * NSW, R, 2, 1>::run(e, (uint64_t*)scr, ib);
    TPH(27);
    // (every wave loaded its keys before the first cross-wave barrier)
#pragma unroll
    for (int r = 0; r < R; ++r) srt[base + r] = e[r];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float m = hyg_expf(key_value(e[r]));
      f[r] = hyg_fix149f((base + r < nA) ? m : 0.0f);
      loc = hyg_u192_add(loc, f[r]);
    }
  } else {
    constexpr int nb = bitonic_lds_stages(64 * NSW * R, R);
#pragma unroll
    for (int i = 0; i < nb; ++i) lds_barrier();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      e[r] = ~0ull;
      f[r] = hyg_u192_zero();
    }
  }
  hyg_u192 massA;
  // red's last readers (the previous step's block max) are behind this step's
  // barriers; its publishing barrier ends every sort-buffer read
  const hyg_u192 ex = block_excl192<NT, false>(loc, red, &massA);
  hyg_u192* pre = (hyg_u192*)scr;                           // inclusive prefix of sorted position p
  const hyg_u192 total = hyg_u192_add(massA, massB);         // every significant weight's mass
  hyg_u192 run = ex;
  if (sorter) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      run = hyg_u192_add(run, f[r]);
      if (base + r < nA) pre[base + r] = run;
    }
  }
  lds_barrier();
  TPH(28);
  if (wave_id() == 0) {
    serial_begin();
    // lane a: c(a) (loop-variable semantics of :12-31); the loop's counts
    // P(c(a)) = #{p : fl(c(a) + x_p) > 0} are taken only at the iterates it
    // visits, by a ballot over the sorted keys x_p of positions p < min(nA, M)
    // (one per lane; M <= 64 on this path): the predicate is monotone in p,
    // so the count of true lanes is the first false position.
    const int a = lane;
    const int cap = nA < M ? nA : M;
    float xk;
    if constexpr (R == 1) xk = key_value(e[0]);  // wave 0 lane p holds sorted position p
    else xk = key_value(srt[lane < nA ? lane : 0]);
    const uint64_t capmask = (cap >= 64) ? ~0ull : ((1ull << cap) - 1ull);
    int flag = 0;
    float ca = 0.0f;
    hyg_u192 rva = hyg_u192_zero();
    if (a < M && a < N) {
      // (positions past the significant weights have zero mass, so R(a) = 0
      // there; outside the list nothing is significant)
      if (a <= nA) rva = hyg_u192_sub(total, a == 0 ? hyg_u192_zero() : pre[a - 1]);
      else if (hasB) flag = 1;  // prefix outside A
      const double rvd = hyg_u192_to_f64(rva);
      const float l2 = (rvd == 0.0) ? HYG_NINFF : (float)hyg_log(rvd);
      ca = cl.logMa[a] - l2;
    }
    TPH(30);
    int aa = 0, bb = -1, ovf = 0;
    while (aa != bb && aa < N && aa < M) {
      const float c = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ca), aa));
      int nxt = 0;
      if (hyg_isfinitef(c)) {  // uniform
        // (no weight below sig_thresh satisfies the predicate: c < log M + 103.3 there)
        nxt = (int)__builtin_popcountll(wave_ballot((float)(c + xk) > 0.0f) & capmask);
        if (nxt == nA && nA < M && hasB) ovf = 1;  // the count may continue below A
      } else if (c > 0.0f) {
        nxt = cnt_fin;  // +inf: every finite particle
      }
      ovf |= __builtin_amdgcn_readlane(flag, aa);
      bb = aa;
      aa = nxt > aa ? nxt : aa;
    }
    TPH(32);
    const float lc = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ca), bb));
    const hyg_u192 Rr = rdlane192(rva, bb);
    int status = FAST_DONE;
    if (ovf) {
      status = FAST_FALLBACK_REGEN;
    } else if (bb < N && hyg_isfinitef(lc)) {
      // systematic residual (:32-40, :56-69): target j lands on the first
      // sorted position p >= K with C(p) >= preK + ceil(T_j R)
      const int L = M - bb;
      const hyg_u192 preK = hyg_u192_sub(total, Rr);
      hyg_u192 tau = hyg_u192_zero();
      if (lane < L) tau = hyg_u192_add(preK, hyg_ceil_mul_f32_bf(((float)lane + Usys) / (float)L, Rr));
      const hyg_u192 tlast = rdlane192(tau, L > 0 ? L - 1 : 0);
      TPH(31);
      if (L > 0 && hasB && !hyg_u192_ge(massA, tlast)) {
        status = FAST_FALLBACK_REGEN;
      } else {
        if (lane < bb) parents[lane] = key_index(srt[lane]);
        if (lane < L) {
          int lo = bb, hi = nA - 1;
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (hyg_u192_ge(pre[mid], tau)) hi = mid; else lo = mid + 1;
          }
          parents[bb + lane] = key_index(srt[lo]);
        }
        TPH(34);
      }
    }
    if (lane == 0) {
      sh.Kk = bb;
      sh.log_c = lc;
      sh.fast = status;
    }
    TPH(33);
    serial_end();
  }
  lds_barrier();
  TPH(29);
  return sh.fast;
}

// u192 -> f64 to within a few ulp (a search estimate only: every decision it
// guides is checked exactly); the scale 2^-149 cancels in the ratios it forms
__device__ __forceinline__ double u192_approx(const hyg_u192& a) {
  auto w = [](uint64_t x) { return fma((double)(uint32_t)(x >> 32), 0x1p32, (double)(uint32_t)x); };
  return fma(w(a.w2), 0x1p128, fma(w(a.w1), 0x1p64, w(a.w0)));
}

// #{j in [0, L) : ceil(T_j R) <= v} for the systematic targets
// T_j = ((float)j + U) / (float)L (f32, as resampling_functions.py:58-67 forms
// them; Ttab[j] holds T_j): T_j R <= v is T_j <= v / R. The estimate
// j ~ (v / R) L - U is within 1e-5 of the exact threshold (T_j carries two f32
// roundings, v / R here a relative error below 2^-49), so every j < j0 counts
// and no j >= j0 + 2 does (j0 = floor of the estimate); the two candidates in
// between are compared in f64 with a 2^-46 guard band and, inside it, exactly
// in integers.
__device__ __forceinline__ int sys_count(const hyg_u192& v, const hyg_u192& R, double invR, int L, float U,
                                         const float* Ttab) {
  const double y = u192_approx(v) * invR;
  double jf = y * (double)L - (double)U;
  jf = jf < -1.0 ? -1.0 : (jf > (double)L ? (double)L : jf);
  const int j0 = (int)floor(jf);
  const double ylo = y * (1.0 - 0x1p-46), yhi = y * (1.0 + 0x1p-46);
  float T[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // loads first (one LDS round trip)
    const int j = j0 + k;
    T[k] = Ttab[j < 0 ? 0 : (j >= L ? L - 1 : j)];
  }
  int c = j0 > 0 ? j0 : 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int j = j0 + k;
    const double t = (double)T[k];
    bool le = t < ylo;
    if (!le && !(t > yhi) && j >= 0 && j < L) le = hyg_u192_ge(v, hyg_ceil_mul_f32_bf(T[k], R));  // exact
    c += (le && j >= 0 && j < L) ? 1 : 0;
  }
  return c;
}

// The value of the lane below (lane 0: `first`), DPP wave_shr:1.
__device__ __forceinline__ int wave_shr1(int v, int first) {
  return __builtin_amdgcn_update_dpp(first, v, 0x138, 0xf, 0xf, false);
}

// LDS bytes of top_set_finish1's scratch: the sort's two exchange buffers,
// then the sorted masses' in-wave inclusive prefixes, then the targets T_j
template <int NSW>
constexpr size_t tsf1_bytes() { return 2 * 64 * NSW * sizeof(uint64_t) + 64 * NSW * sizeof(hyg_u192) + 64 * sizeof(float); }

// top_set_finish for one key per lane (sorter wave w, lane l: sorted position
// 64 w + l), shaped for latency: after the sort each sorting wave scans its
// own masses and publishes its total (one barrier, no block scan); wave 0 then
// runs the K loop on its own prefixes and finds the systematic targets by
// counting them per sorted position (sys_count), 64 positions per pass, from
// the first kept position on, instead of a binary search per target. Same
// parents, Kk, log c and fallback decisions as top_set_finish.
// The outside masses of the lists, for top_set_finish1<.., SPLIT = true>:
// the lists hold the outside log-weights (f32 bits, -inf inside A).
struct ListsB {
  const int* lst;        // wave w's list at lst[w * stride], part_cnt[w * kNCut + kNCut - 1] entries
  int stride;
  const int* part_cnt;
  hyg_u192* part_tot;    // one partial per non-sorting wave
  bool narrow;           // every outside mass below e^-20, <= kNarrowPerLane images per lane: u128 sums
                         // (a lane sums up to 2 ceil(N / NT) images: two lists)
};
// Exact image sum of the f32 masses exp(lw) of list w (lane-strided, two
// entries per lane in flight).
__device__ __forceinline__ void list_mass(const ListsB& lb, int w, hyg_u128& n128, hyg_u192& m192) {
  const int cnt = lb.part_cnt[w * kNCut + kNCut - 1];
  const int* L = lb.lst + w * lb.stride;
  const int lane = lane_id();
  for (int b = 0; b < cnt; b += 128) {  // cnt is wave-uniform
    const int i0 = b + lane, i1 = b + 64 + lane;
    const float x0 = __builtin_bit_cast(float, L[i0 < cnt ? i0 : b]);
    const float x1 = __builtin_bit_cast(float, L[i1 < cnt ? i1 : b]);
    const float m0 = (i0 < cnt) ? hyg_expf(x0) : 0.0f, m1 = (i1 < cnt) ? hyg_expf(x1) : 0.0f;
    if (lb.narrow) {
      n128 = hyg_u128_add(n128, hyg_u128_add(hyg_fix149f_low128(m0), hyg_fix149f_low128(m1)));
    } else {
      m192 = hyg_u192_add(m192, hyg_u192_add(hyg_fix149f(m0), hyg_fix149f(m1)));
    }
  }
}

template <int NT, int NSW, bool SPLIT>
__device__ __forceinline__ int top_set_finish1(uint64_t* srt, int nA, bool hasB, int N, int M, int cnt_fin,
                                               const hyg_u192& massB_in, unsigned char* scr, int* parents,
                                               Shared& sh, const ConstLds& cl, unsigned char* red, float Usys,
                                               const ListsB& lb, unsigned long long* ph, bool timed) {
  static_assert(NSW <= NT / 64 && NSW <= 4, "sorting waves");
  constexpr int NW = NT / 64, NNS = NW - NSW;
  static_assert(!SPLIT || NNS >= NSW, "the outside masses need idle waves");
  const int lane = lane_id();
  const bool sorter = (NSW == NT / 64) || wave_id() < NSW;  // wave-uniform
  const int base = (int)(threadIdx.x >> 6) * 64 + lane;
  hyg_u192* preL = (hyg_u192*)(scr + 2 * 64 * NSW * sizeof(uint64_t));  // past the sort buffers
  hyg_u192* wtot = (hyg_u192*)red;  // red's last readers are behind this step's barriers
  uint64_t e[1];
  hyg_u192 f = hyg_u192_zero(), inc = hyg_u192_zero();
  if (sorter) {
    // (distinct pads above every key past nA: the rank sort needs distinct keys)
    e[0] = (base < nA) ? srt[base] : ~0ull - (uint64_t)base;
    e[0] = rank_sort_asc<NSW>(e[0], (uint64_t*)scr, true, []() {});
    TPH(27);
    // (every wave loaded its keys before the sort's first barrier)
    srt[base] = e[0];
    const float m = hyg_expf(key_value(e[0]));
    f = hyg_fix149f((base < nA) ? m : 0.0f);
    inc = wave_incl192(f);
    preL[base] = inc;
    if (lane == 63) wtot[wave_id()] = inc;
  } else {
    // SPLIT: the waves that do not sort sum the outside masses meanwhile,
    // wave NSW + v the lists v and v + NNS (NW <= 2 NNS): the first while the
    // sorting waves sort their runs, the second while they search the ranks
    // (between the sort's two barriers)
    static_assert(!SPLIT || NW <= 2 * NNS, "two lists per idle wave");
    hyg_u128 n128 = hyg_u128_zero();
    hyg_u192 m192 = hyg_u192_zero();
    const int v = wave_id() - NSW;
    if (SPLIT && hasB) list_mass(lb, v, n128, m192);  // uniform
    (void)rank_sort_asc<NSW>(0, (uint64_t*)scr, false, [&]() {
      if (SPLIT && hasB && v + NNS < NW) list_mass(lb, v + NNS, n128, m192);
    });
    if (SPLIT && hasB) {
      if (lb.narrow) { m192.w0 = n128.lo; m192.w1 = n128.hi; m192.w2 = 0; }
      const hyg_u192 ws = wave_sum192(m192);
      if (lane == 0) lb.part_tot[v] = ws;
    }
    e[0] = ~0ull;
  }
  lds_barrier();
  TPH(28);
  if (wave_id() == 0) {
    serial_begin();
    hyg_u192 massA = hyg_u192_zero();
#pragma unroll
    for (int w = 0; w < NSW; ++w) massA = hyg_u192_add(massA, wtot[w]);
    hyg_u192 massB = massB_in;
    if (SPLIT && hasB) {
#pragma unroll
      for (int w = 0; w < NNS; ++w) massB = hyg_u192_add(massB, lb.part_tot[w]);
    }
    const hyg_u192 total = hyg_u192_add(massA, massB);  // every significant weight's mass
    // lane a: c(a) (loop-variable semantics of :12-31) from the suffix mass
    // total - C(a - 1), C(a - 1) = this lane's exclusive prefix
    const int a = lane;
    const float xk = key_value(e[0]);
    const int cap = nA < M ? nA : M;
    const uint64_t capmask = (cap >= 64) ? ~0ull : ((1ull << cap) - 1ull);
    int flag = 0;
    float ca = 0.0f;
    hyg_u192 rva = hyg_u192_zero();
    if (a < M && a < N) {
      if (a <= nA) rva = hyg_u192_sub(total, hyg_u192_sub(inc, f));
      else if (hasB) flag = 1;  // prefix outside A
      const double rvd = hyg_u192_to_f64(rva);
      const float l2 = (rvd == 0.0) ? HYG_NINFF : (float)hyg_log(rvd);
      ca = cl.logMa[a] - l2;
    }
    TPH(30);
    int aa = 0, bb = -1, ovf = 0;
    while (aa != bb && aa < N && aa < M) {
      const float c = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ca), aa));
      int nxt = 0;
      if (hyg_isfinitef(c)) {  // uniform
        nxt = (int)__builtin_popcountll(wave_ballot((float)(c + xk) > 0.0f) & capmask);
        if (nxt == nA && nA < M && hasB) ovf = 1;  // the count may continue below A
      } else if (c > 0.0f) {
        nxt = cnt_fin;  // +inf: every finite particle
      }
      ovf |= __builtin_amdgcn_readlane(flag, aa);
      bb = aa;
      aa = nxt > aa ? nxt : aa;
    }
    TPH(32);
    const float lc = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ca), bb));
    int status = FAST_DONE;
    if (ovf) {
      status = FAST_FALLBACK_REGEN;
    } else if (bb < N && hyg_isfinitef(lc)) {
      // (bb < nA here: bb > nA sets ovf, and bb = nA leaves a zero residual
      // mass when nothing lies outside A, so log c is infinite)
      if (lane < bb) parents[lane] = key_index(e[0]);
      const int L = M - bb;
      TPH(31);
      if (L > 0) {
        // systematic residual (:32-40, :56-69): target j lands on the first
        // sorted position p >= K with C(p) >= preK + ceil(T_j R); position p
        // takes the targets j in [count(C(p - 1)), count(C(p)))
        const hyg_u192 Rr = rdlane192(rva, bb);
        const double invR = 1.0 / u192_approx(Rr);
        const hyg_u192 preK = hyg_u192_sub(total, Rr);
        float* Ttab = (float*)(scr + tsf1_bytes<NSW>() - 64 * sizeof(float));
        if (lane < L) Ttab[lane] = ((float)lane + Usys) / (float)L;
        wave_lds_sync();
        // C at the start of each sorting wave's positions
        hyg_u192 wb[NSW];
        wb[0] = hyg_u192_zero();
#pragma unroll
        for (int w = 1; w < NSW; ++w) wb[w] = hyg_u192_add(wb[w - 1], wtot[w - 1]);
        int cprev = 0;
        // 64 positions per pass from the first kept one on (the deepest
        // target sits about 60 positions past it at C3: mostly one pass)
#pragma unroll
        for (int i = 0; i < NSW; ++i) {
          const int p0 = bb + 64 * i;
          if (p0 >= nA || cprev >= L) break;  // uniform
          const int p = p0 + lane;
          const int pc = p < nA ? p : nA - 1;  // past A: the count of its last position
          const int wp = pc >> 6;
          hyg_u192 C = preL[pc];
#pragma unroll
          for (int w = 1; w < NSW; ++w)
            if (wp == w) C = hyg_u192_add(C, wb[w]);
          const uint64_t key = srt[pc];
          const int cnt = sys_count(hyg_u192_sub(C, preK), Rr, invR, L, Usys, Ttab);
          const int cex = wave_shr1(cnt, cprev);
          for (int j = cex; j < cnt; ++j) parents[bb + j] = key_index(key);
          cprev = __builtin_amdgcn_readlane(cnt, 63);
        }
        // targets past A: only when weights lie outside it
        if (cprev < L) status = FAST_FALLBACK_REGEN;
      }
      TPH(34);
    }
    if (lane == 0) {
      sh.Kk = bb;
      sh.log_c = lc;
      sh.fast = status;
    }
    TPH(33);
    serial_end();
  }
  lds_barrier();
  TPH(29);
  return sh.fast;
}

// Top-set path of OptimalFiniteState; returns FAST_DONE (parents / Kk /
// log_c written; log_c infinite -> the caller's unbiased fallback),
// FAST_FALLBACK (W intact) or FAST_FALLBACK_REGEN (W overwritten). The
// counts of the cutoff sets per wave (part_cnt) were published with the
// candidate lists before the log-sum-exp reduction.
template <int NT, int NSW>
__device__ __forceinline__ int top_set_resample(const double* W, int N, double mx, double logS, int* lst, int lb, int cw,
                                unsigned char* scr, size_t scr_bytes, uint64_t* srt, size_t srt_bytes,
                                const int* part_cnt, hyg_u192* part_tot, int* parents, Shared& sh,
                                const ConstLds& cl, unsigned char* red, int M, int cnt_fin, float Usys,
                                int rmax, unsigned long long* ph, bool timed) {
  constexpr int NW = NT / 64;
  const int wv = wave_id(), lane = lane_id();
  // ---- 1. the most inclusive cutoff whose set A fits the sort
  // one LDS read per lane per 8 waves (lane w * kNCut + k holds wave w's count
  // at cutoff k, waves 8-15 in a second register), the per-cutoff totals by
  // xor shuffles (every lane l gets cutoff l % 8)
  static_assert(kNCut == 8 && NW * kNCut <= 128, "cutoff counts: one or two per lane");
  const int pc = (lane < NW * kNCut) ? part_cnt[lane] : 0;
  const int pc2 = (NW * kNCut > 64 && lane + 64 < NW * kNCut) ? part_cnt[lane + 64] : 0;
  int c = pc + pc2;
  c += (int)xshfl32<8>((uint32_t)c);
  c += (int)xshfl32<16>((uint32_t)c);
  c += (int)xshfl32<32>((uint32_t)c);
  const int np = (c <= 64 * NSW) ? 64 * NSW : 128 * NSW;
  const bool fits = lane < kNCut && c <= 64 * NSW * rmax && (size_t)np * sizeof(hyg_u192) <= scr_bytes &&
                    (size_t)np * 8 <= srt_bytes;
  const uint64_t fm = wave_ballot(fits);
  const int nL = __builtin_amdgcn_readlane(c, kNCut - 1);
  if (threadIdx.x == 0) sh.n_sig = nL;
  if (fm == 0) return FAST_FALLBACK;  // uniform
  const int ks = 63 - __builtin_clzll(fm);  // the most inclusive cutoff that fits
  const int nA = __builtin_amdgcn_readlane(c, ks);
  const bool hasB = nA < nL;         // list weights outside A (their masses enter the total)
  const double cutx = (ks == kNCut - 1) ? HYG_NINF : -cut_below_top(ks);
  int off = 0;
  for (int w = 0; w < wv; ++w)
    off += __builtin_amdgcn_readlane(w < 8 ? pc : pc2, (w & 7) * kNCut + ks);
  // ---- 2. gather A's keys; exact mass of the list weights outside A. From the
  // third cutoff on (X >= 20 nats below the top: every outside mass is below
  // e^-20 < 2^-28.8, its image m 2^149 below 2^120.2, and a lane sums at most
  // ceil(N / NT) <= 128 of them, below 2^127.2) a lane's images are formed and
  // summed as u128.
  const bool narrow = ks >= kNarrowCut && (N + NT - 1) / NT <= kNarrowPerLane;
  // SPLIT (workgroups with at least as many idle waves as sorting ones): the
  // lists take the outside log-weights back and the idle waves sum their
  // masses during the sort (top_set_finish1)
  constexpr int NNS = NW - NSW;
  constexpr bool kSplitB = HYG_TSF1 && NSW <= 4 && NNS >= NSW;
  const bool split = kSplitB && nA <= 64 * NSW && scr_bytes >= tsf1_bytes<NSW>();
  hyg_u192 mb = hyg_u192_zero(), mb2 = hyg_u192_zero();
  hyg_u128 nb = hyg_u128_zero(), nb2 = hyg_u128_zero();
  constexpr int kLR = kLRof<NT>;
  for (int b = 0; b < cw; b += 64 * kLR) {  // kLR entries per lane, loads first (see the lse loop)
    int nn[kLR];
    float lw[kLR];
    bool inA[kLR], outA[kLR];
#pragma unroll
    for (int r = 0; r < kLR; ++r) {
      const int i = b + r * 64 + lane;
      nn[r] = lst[lb + (i < cw ? i : b)];
    }
#pragma unroll
    for (int r = 0; r < kLR; ++r) {
      const bool v = b + r * 64 + lane < cw;
      const double x = W[nn[r]] - mx;
      lw[r] = (float)(x - logS);
      inA[r] = v && x >= cutx;
      outA[r] = v && !inA[r];
    }
#pragma unroll
    for (int r = 0; r < kLR; ++r) {
      const uint64_t bal = wave_ballot(inA[r]);
      if (inA[r]) srt[off + lanes_below(bal)] = sort_key(lw[r], nn[r]);
      off += (int)__builtin_popcountll(bal);
    }
    if (split) {
      if (hasB) {
#pragma unroll
        for (int r = 0; r < kLR; ++r)
          if (b + r * 64 + lane < cw) lst[lb + b + r * 64 + lane] = __builtin_bit_cast(int, outA[r] ? lw[r] : HYG_NINFF);
      }
    } else if (hasB && narrow) {  // uniform; expf(lw) is 0 below sig_thresh
#pragma unroll
      for (int r = 0; r < kLR; ++r) {
        const float m = hyg_expf(lw[r]);
        const hyg_u128 f = hyg_fix149f_low128(outA[r] ? m : 0.0f);
        if (r & 1) nb2 = hyg_u128_add(nb2, f); else nb = hyg_u128_add(nb, f);
      }
    } else if (hasB) {
#pragma unroll
      for (int r = 0; r < kLR; ++r) {
        const float m = hyg_expf(lw[r]);
        const hyg_u192 f = hyg_fix149f(outA[r] ? m : 0.0f);
        if (r & 1) mb2 = hyg_u192_add(mb2, f); else mb = hyg_u192_add(mb, f);
      }
    }
  }
  if constexpr (kSplitB) {
    if (split) {
      lds_barrier();  // the keys of A and the lists' log-weights
      TPH(26);
      ListsB lbs;
      lbs.lst = lst;
      lbs.stride = ((N + NT - 1) / NT) * 64;
      lbs.part_cnt = part_cnt;
      lbs.part_tot = part_tot;
      lbs.narrow = ks >= kNarrowCut && 2 * ((N + NT - 1) / NT) <= kNarrowPerLane;
      return top_set_finish1<NT, NSW, kSplitB>(srt, nA, hasB, N, M, cnt_fin, hyg_u192_zero(), scr, parents, sh, cl,
                                               red, Usys, lbs, ph, timed);
    }
  }
  if (hasB) {
    if (narrow) {
      const hyg_u128 t = hyg_u128_add(nb, nb2);
      mb.w0 = t.lo; mb.w1 = t.hi; mb.w2 = 0;
    } else {
      mb = hyg_u192_add(mb, mb2);
    }
    const hyg_u192 ws = wave_sum192(mb);
    if (lane == 0) part_tot[wv] = ws;
  }
  lds_barrier();
  hyg_u192 massB = hyg_u192_zero();
  if (hasB) massB = sum_waves192<NW>(part_tot);
  TPH(26);
  if (nA <= 64 * NSW) {
#if HYG_TSF1
    if constexpr (NSW <= 4)
      if (scr_bytes >= tsf1_bytes<NSW>())
        return top_set_finish1<NT, NSW, false>(srt, nA, hasB, N, M, cnt_fin, massB, scr, parents, sh, cl, red, Usys,
                                               ListsB{}, ph, timed);
#endif
    return top_set_finish<NT, NSW, 1>(srt, nA, hasB, N, M, cnt_fin, massB, scr, parents, sh, cl, red, Usys, ph, timed);
  }
  return top_set_finish<NT, NSW, 2>(srt, nA, hasB, N, M, cnt_fin, massB, scr, parents, sh, cl, red, Usys, ph, timed);
}
#undef TPH

// --------------------------------------------------------------- kernels
// One thread per site of a 256-site tile; the tile's rows [256][2K] f64 are
// assembled in LDS and written out as whole 16-byte pieces by consecutive
// lanes (a thread writing its own 96-byte row in 8-byte stores left partial
// lines: 1.36x the algorithmic write bytes at K = 6).
constexpr int kETile = 256;
__global__ void __launch_bounds__(kETile)
tg_emission_kernel(const double* __restrict__ lf, const double* __restrict__ lg, const double* __restrict__ cst,
                   int L, int K, const uint16_t* __restrict__ meth_c, const uint16_t* __restrict__ tot_c, int s_c,
                   const uint16_t* __restrict__ meth_k, const uint16_t* __restrict__ tot_k, int s_k, int64_t T,
                   double* __restrict__ E) {
  extern __shared__ __align__(16) unsigned char smem[];
  double* tile = (double*)smem;  // [kETile][2K]
  const int K2 = 2 * K;
  for (int64_t t0 = (int64_t)blockIdx.x * kETile; t0 < T; t0 += (int64_t)gridDim.x * kETile) {
    const int64_t t = t0 + threadIdx.x;
    if (t < T) {
      for (int g = 0; g < 2; ++g) {
        const int S = g ? s_k : s_c;
        const uint16_t* my = g ? meth_k + t * s_k : meth_c + t * s_c;
        const uint16_t* nt = g ? tot_k + t * s_k : tot_c + t * s_c;
        double e[HYG_KMAX];
        for (int r = 0; r < K; ++r) e[r] = 0.0;
        for (int s = 0; s < S; ++s) {
          const int n = nt[s], y = my[s];
          if (n == 0) continue;
          if (y > n || n >= L) {  // invalid input: poison the row
            for (int r = 0; r < K; ++r) e[r] = HYG_NAN;
            break;
          }
          double base = lf[n] - lf[y];
          base = base - lf[n - y];
          for (int r = 0; r < K; ++r) {
            double term = base + lg[(size_t)(r * 3 + 0) * L + y];
            term = term + lg[(size_t)(r * 3 + 1) * L + (n - y)];
            term = term - lg[(size_t)(r * 3 + 2) * L + n];
            term = term + cst[r];
            e[r] = e[r] + term;
          }
        }
        for (int r = 0; r < K; ++r) tile[threadIdx.x * K2 + g * K + r] = e[r];
      }
    }
    __syncthreads();
    // the tile's rows are contiguous in E: 16-byte pieces, consecutive lanes
    const int64_t rows = (T - t0) < kETile ? (T - t0) : kETile;
    const int n = (int)rows * K2;  // doubles; E rows start 16-byte aligned when K2 is even
    double* dst = E + t0 * K2;
    for (int i = 2 * threadIdx.x; i + 1 < n; i += 2 * kETile)
      *(double2*)(dst + i) = make_double2(tile[i], tile[i + 1]);
    if ((n & 1) && threadIdx.x == 0) dst[n - 1] = tile[n - 1];
    __syncthreads();
  }
}

// The same sums from the per-(n, y) term table (hyg_bb_term_table: every
// regime's term of a sample in one row of K doubles, built with the per-term
// kernel's operations, so each entry has the bits that kernel forms): one row
// load per sample instead of 3 + 3K table gathers. The table is L2-sized at
// the pipeline's coverage (0.7 MB at K = 6), so the kernel streams the counts
// in and the rows out at close to the HBM rate. KT > 0: the regime count at
// compile time (rows as 16-byte loads).
template <int KT>
__global__ void __launch_bounds__(kETile)
tg_emission_tab_kernel(const double* __restrict__ bbt, int L, int Kr, const uint16_t* __restrict__ meth_c,
                       const uint16_t* __restrict__ tot_c, int s_c, const uint16_t* __restrict__ meth_k,
                       const uint16_t* __restrict__ tot_k, int s_k, int64_t T, double* __restrict__ E) {
  extern __shared__ __align__(16) unsigned char smem[];
  double* tile = (double*)smem;  // [kETile][2K]
  const int K = KT ? KT : Kr, K2 = 2 * K;
  for (int64_t t0 = (int64_t)blockIdx.x * kETile; t0 < T; t0 += (int64_t)gridDim.x * kETile) {
    const int64_t t = t0 + threadIdx.x;
    if (t < T) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int S = g ? s_k : s_c;
        const uint16_t* my = g ? meth_k + t * s_k : meth_c + t * s_c;
        const uint16_t* nt = g ? tot_k + t * s_k : tot_c + t * s_c;
        double e[KT ? KT : HYG_KMAX];
#pragma unroll
        for (int r = 0; r < (KT ? KT : HYG_KMAX); ++r) e[r] = 0.0;
        bool bad = false;
        // samples in chunks of kCh: every count load of the chunk issued first,
        // then every row load, then the sums in sample order (a sample with
        // n = 0 adds nothing, as the per-term kernel skips it)
        constexpr int kCh = 4;
        // (an even sample count with 4-byte aligned rows: the counts as pairs)
        const bool pairs = (S % 2 == 0) && ((((uintptr_t)my) | ((uintptr_t)nt)) & 3) == 0;
        for (int s0 = 0; s0 < S; s0 += kCh) {
          int nn[kCh], yy[kCh];
          if (pairs) {
#pragma unroll
            for (int j = 0; j < kCh; j += 2) {
              const int sj = s0 + j < S ? s0 + j : S - 2;
              const uint32_t a = *(const uint32_t*)(nt + sj), b = *(const uint32_t*)(my + sj);
              nn[j] = (int)(a & 0xffffu);
              nn[j + 1] = (int)(a >> 16);
              yy[j] = (int)(b & 0xffffu);
              yy[j + 1] = (int)(b >> 16);
            }
          } else {
#pragma unroll
            for (int j = 0; j < kCh; ++j) {
              const int sj = s0 + j < S ? s0 + j : S - 1;
              nn[j] = nt[sj];
              yy[j] = my[sj];
            }
          }
          size_t off[kCh];
          bool use[kCh];
#pragma unroll
          for (int j = 0; j < kCh; ++j) {
            const int n = nn[j], y = yy[j];
            use[j] = s0 + j < S && n != 0;
            bad = bad || (use[j] && (y > n || n >= L));  // invalid input: poison the row
            use[j] = use[j] && y <= n && n < L;
            off[j] = use[j] ? ((size_t)n * (size_t)(n + 1) / 2 + (size_t)y) * (size_t)K : 0;
          }
          if constexpr (KT > 0 && KT % 2 == 0) {
            double2 v[kCh][KT / 2];
#pragma unroll
            for (int j = 0; j < kCh; ++j)
#pragma unroll
              for (int r = 0; r < KT / 2; ++r) v[j][r] = *(const double2*)(bbt + off[j] + 2 * r);
#pragma unroll
            for (int j = 0; j < kCh; ++j)
#pragma unroll
              for (int r = 0; r < KT / 2; ++r) {
                e[2 * r] = use[j] ? e[2 * r] + v[j][r].x : e[2 * r];
                e[2 * r + 1] = use[j] ? e[2 * r + 1] + v[j][r].y : e[2 * r + 1];
              }
          } else {
#pragma unroll
            for (int j = 0; j < kCh; ++j)
              if (use[j])
                for (int r = 0; r < K; ++r) e[r] = e[r] + bbt[off[j] + r];
          }
        }
        for (int r = 0; r < K; ++r) tile[threadIdx.x * K2 + g * K + r] = bad ? HYG_NAN : e[r];
      }
    }
    __syncthreads();
    const int64_t rows = (T - t0) < kETile ? (T - t0) : kETile;
    const int n = (int)rows * K2;
    double* dst = E + t0 * K2;
    for (int i = 2 * threadIdx.x; i + 1 < n; i += 2 * kETile)
      *(double2*)(dst + i) = make_double2(tile[i], tile[i + 1]);
    if ((n & 1) && threadIdx.x == 0) dst[n - 1] = tile[n - 1];
    __syncthreads();
  }
}

// Three waves per SIMD (<= 168 VGPRs) at 256 and 768 threads: a CU holds three
// chains or one (the second argument is the minimum waves per SIMD); 512
// threads (one chain per CU: C5 by its LDS, or a low-occupancy launch) may use
// up to 256 VGPRs.
template <int NT, int KC = 0, int MC = 0, int BC = 0, bool PHS = false>  // PHS: phase-timer build
__global__ void __launch_bounds__(NT, (NT == 512 ? 1 : 3))
tg_forward_kernel(ModelDev md, const ChainDev* __restrict__ chains, const double* __restrict__ E,
                  uint8_t* __restrict__ ws, int32_t* status_out, double* __restrict__ logz_out,
                  double* __restrict__ finalw_out, Lay lay_arg, unsigned long long* __restrict__ dbg_arg) {
  // the timers only exist in the PHS instantiation: a constant null pointer
  // folds every timer test away (no SGPRs, branches or s_memtime in the step loop)
  unsigned long long* __restrict__ const dbg = PHS ? dbg_arg : nullptr;
  const hyg_tg_consts* __restrict__ c = md.consts;
  const int K = KC ? KC : c->K, M = KC ? MC : c->M, I = KC ? 2 * KC + KC * KC : c->I, K2 = 2 * K,
            tid = threadIdx.x;
  const Lay lay = KC ? make_layout(KC, MC, BC, MC * (2 * KC + KC * KC), NT, false) : lay_arg;
  // in a register for the whole chain: a load of c-> inside the step loop is a
  // global load the compiler cannot hoist past the record stores (it may
  // alias them), followed by a vmcnt(0) wait on every outstanding store
  const float sig_thresh = c->sig_thresh;
  const ChainDev ch = chains[blockIdx.x];
  const int T = ch.T;
  extern __shared__ __align__(16) unsigned char smem[];
  double* W = (double*)(smem + lay.W);
  uint64_t* keys = (uint64_t*)(smem + lay.keys);
  hyg_u128* cp128 = (hyg_u128*)(smem + lay.keys);  // prefix arrays of the keep / fallback paths
  int* bcnt = (int*)(smem + lay.bcnt);
  int* bpos = (int*)(smem + lay.bpos);
  hyg_u192* tau = (hyg_u192*)(smem + lay.bcnt);
  hyg_u192* pre64 = (hyg_u192*)(smem + lay.pre64);
  uint64_t* pst0 = (uint64_t*)(smem + lay.pst);  // [2][M]: buffer `cur` holds the current ancestors
  double* pw0 = (double*)(smem + lay.pw);
  Hz4* phz0 = (Hz4*)(smem + lay.phz);
  int cur = 0;
  Pf3* pf = (Pf3*)(smem + lay.pf);
  double* ering = (double*)(smem + lay.ering);
  ConstLds& cl = *(ConstLds*)(smem + lay.cl);
  int* parents = (int*)(smem + lay.parents);
  unsigned char* red = smem + lay.red;
  Shared& sh = *(Shared*)(smem + lay.sh);
  float* uring = (float*)(smem + lay.uring);  // NT >= 256 only (kURing)
  constexpr bool kURing = NT >= 256;
  constexpr int kUR = NT >= 512 ? 64 : 32;  // ring entries
  int* part_cnt = (int*)(smem + lay.part);
  hyg_u192* part_tot = (hyg_u192*)(smem + lay.part + sizeof(int) * kNCut * (NT / 64));

  // phase timers (diagnostic runs only: dbg != nullptr), kept in LDS
  unsigned long long* ph_acc = sh.ph;
  if (tid < kPh) ph_acc[tid] = 0;
#define PH(k)                                                      \
  if (dbg && tid == 0) {                                           \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    ph_acc[k] += now_ - ph_acc[kPh - 1];                                \
    ph_acc[kPh - 1] = now_;                                             \
  }

  uint8_t* rec0 = ws + ch.ws_offset;
  const size_t rstride = record_bytes(M);
  const double* Ech = E + ch.site_begin * K2;

  // ---- t = 0 (_filter_first_step)
  load_consts(cl, c, md);
  load_eblock(ering, Ech, 0, T, K2, NT);
  load_eblock(ering, Ech, 1, T, K2, NT);
  if (tid == 0) {
    sh.Unext = hyg_u01f(hyg_rand64(ch.seed, ch.chain_id, HYG_RNG_SYSTEMATIC, 1, 0));
    sh.r_ph = (int)hyg_mulhi64(hyg_rand64(ch.seed, ch.chain_id, HYG_RNG_PHANTOM, 0, 0), (uint64_t)K);
    sh.status = HYG_OK;
    StepScalars* s0 = (StepScalars*)rec0;
    s0->mode = MODE_INIT; s0->n_par = 0; s0->log_c = 0.0f; s0->r_ph = sh.r_ph; s0->lse = 0.0; s0->pad = 0.0;
  }
  if (kURing && wave_id() == NT / 64 - 1 && lane_id() < kUR)  // steps 1 .. kUR
    uring[(1 + lane_id()) & (kUR - 1)] =
        hyg_u01f(hyg_rand64(ch.seed, ch.chain_id, HYG_RNG_SYSTEMATIC, (uint64_t)(1 + lane_id()), 0));
  lds_barrier();
  double mloc;
  int cloc;
  gen_weights_init<NT>(cl, K, sh.r_ph, erow(ering, 0, K2), W, &mloc, &cloc);
  int N = K * K, np_prev = 0, prev_mode = MODE_INIT;
  float prev_logc = 0.0f;
  double prev_lse = 0.0;
  double mx;
  int cnt;
  block_max_cnt<NT>(mloc, cloc, red, &mx, &cnt);

  if (dbg && tid == 0) ph_acc[kPh - 1] = __builtin_amdgcn_s_memtime();
  for (int t = 1; t < T; ++t) {
    // the ancestors of step t-1's particles (read by the regenerations and the gather)
    const uint64_t* pst = pst0 + cur * M;
    const double* pw = pw0 + cur * M;
    const Hz4* phz = phz0 + cur * M;
    // emission rows one block ahead: issue at the block start, land in the ring later
    const bool eload = ((t % kEBlock) == 0) && (t + kEBlock < T);
    PH(0);
    if (!(mx > HYG_NINF)) {
      if (tid == 0) sh.status = HYG_ENUMERIC;
      break;  // uniform
    }
    // written during step t-1's gather (or, kURing, a multiple of kUR steps ago), before two barriers
    const float Ucur = kURing ? uring[t & (kUR - 1)] : sh.Unext;
    // ---- log_softmax / reduce_logsumexp of the weights of step t-1
    // ---- per wave, the list of candidates with W - mx >= sig_thresh (keys
    //      area): every nonzero F=100 mass (x >= -70) and every significant
    //      f32 log-weight is on it; candidates interleaved over the waves
    int* lst = (int*)keys;
    const int lst_base = wave_id() * (((N + NT - 1) / NT) * 64);
    int lst_cnt = 0;
    const bool topset = cnt > M && M <= 64;  // this step resamples by the top-set path
    {
      // kCC candidates per lane at a time, their loads issued together (a
      // load / compare / ballot per iteration waits out an LDS round trip each)
      const double cutw = (double)sig_thresh;
      // (the shape-specialised kernel: every candidate in one pass, N <= M I)
      constexpr int kCC = KC ? (MC * (2 * KC + KC * KC) + NT - 1) / NT : 8;
      for (int b0 = wave_id() * 64; b0 < N; b0 += kCC * NT) {
        bool keep[kCC];
#pragma unroll
        for (int j = 0; j < kCC; ++j) {
          const int n = b0 + j * NT + lane_id();
          const double w = W[n < N ? n : 0];
          // `&`, not `&&`: a short-circuit test puts the load under a branch
          // and waits out its round trip before the next candidate's load
          keep[j] = (n < N) & (w - mx >= cutw);
        }
#pragma unroll
        for (int j = 0; j < kCC; ++j) {
          const uint64_t bal = wave_ballot(keep[j]);
          if (keep[j]) lst[lst_base + lst_cnt + lanes_below(bal)] = b0 + j * NT + lane_id();
          lst_cnt += (int)__builtin_popcountll(bal);
        }
      }
      wave_lds_sync();
    }
    PH(22);
    double logS;
    {
      // kLR list entries per lane at a time: every load of the chunk issued
      // first, then kLR independent exp / fixed-point chains in straight-line
      // code (hyg_fix100 is branch-free), so they interleave. fix100(exp(x))
      // is 0 for x < -70; padding lanes take x = -inf (mass 0, no cutoff).
      // Top-set steps also count the list per cutoff (per-lane counters).
      constexpr int kLR = kLRof<NT>;
      hyg_u128 s0 = hyg_u128_zero(), s1 = hyg_u128_zero();
      int ccut[kNCut - 1];
#pragma unroll
      for (int k = 0; k < kNCut - 1; ++k) ccut[k] = 0;
      for (int b = 0; b < lst_cnt; b += 64 * kLR) {  // lst_cnt is wave-uniform
        int nn[kLR];
        double xx[kLR];
#pragma unroll
        for (int r = 0; r < kLR; ++r) {
          const int i = b + r * 64 + lane_id();
          nn[r] = lst[lst_base + (i < lst_cnt ? i : b)];
        }
#pragma unroll
        for (int r = 0; r < kLR; ++r) {
          const double w = W[nn[r]];
          xx[r] = (b + r * 64 + lane_id() < lst_cnt) ? w - mx : HYG_NINF;
        }
        hyg_u128 ff[kLR];
        exp_fix100_lockstep<kLR>(xx, ff);
#pragma unroll
        for (int r = 0; r < kLR; ++r) {
          if (r & 1) s1 = hyg_u128_add(s1, ff[r]); else s0 = hyg_u128_add(s0, ff[r]);
        }
        if (topset) {  // wave counts per cutoff by ballots (scalar sums)
#pragma unroll
          for (int r = 0; r < kLR; ++r)
#pragma unroll
            for (int k = 0; k < kNCut - 1; ++k)
              ccut[k] += (int)__builtin_popcountll(wave_ballot(xx[r] >= -cut_below_top(k)));
        }
      }
      PH(23);
      if (topset) {
        if (lane_id() == 0) {  // read after the reduction's barriers below
#pragma unroll
          for (int k = 0; k < kNCut - 1; ++k) part_cnt[wave_id() * kNCut + k] = ccut[k];
          part_cnt[wave_id() * kNCut + kNCut - 1] = lst_cnt;
        }
      }
      const hyg_u128 sacc = hyg_u128_add(s0, s1);
      PH(12);
      // own slot of `red`, whose last reader (this reduction, a step ago) is
      // behind many barriers: no leading barrier
      const hyg_u128 S = block_sum128<NT, false>(sacc, red + 32 * (NT / 64));
      PH(11);
      logS = hyg_log(hyg_u128_to_f64(S, 100));
    }
    const double lse = logS + mx;
    PH(1);
    int mode, np;
    float log_c = 0.0f;
    bool need_bar = true;  // parents written by many threads, no barrier behind them yet
    if (cnt <= M) {
      // ---- keep every particle with non-zero weight, in index order (:207-209)
      mode = MODE_KEEP;
      np = cnt;
      const int cs = (N + NT - 1) / NT;
      const int p0 = tid * cs, p1 = (p0 + cs < N) ? p0 + cs : N;
      int loc = 0;
      for (int n = p0; n < p1; ++n) loc += (W[n] > HYG_NINF);
      hyg_u128 v;
      v.lo = (uint64_t)loc;
      v.hi = 0;
      block_scan128<NT>(v, cp128, red);
      lds_barrier();
      int o = (int)cp128[tid].lo;
      for (int n = p0; n < p1; ++n)
        if (W[n] > HYG_NINF) parents[o++] = n;
      PH(2);
      if (dbg && tid == 0) ph_acc[10]++;
    } else {
      // ---- OptimalFiniteState (resampling_functions.py:7-52)
      PH(2);
      int fs = FAST_FALLBACK;
      if (topset)
        fs = top_set_resample<NT, kSortWaves<NT>>(W, N, mx, logS, lst, lst_base, lst_cnt, smem + lay.W, lay.bcnt - lay.W,
                                  (uint64_t*)(smem + lay.bcnt), lay.bcnt_bytes, part_cnt, part_tot, parents, sh, cl,
                                  red, M, cnt, Ucur, lay.topset_r, ph_acc, dbg != nullptr);
      PH(20);
      if (fs != FAST_DONE) {
        if (fs == FAST_FALLBACK_REGEN) {  // the top-set path used the W area: rebuild step t-1's weights
          if (prev_mode == MODE_INIT) {
            gen_weights_init<NT>(cl, K, sh.r_ph, erow(ering, t - 1, K2), W, &mloc, &cloc);
          } else {
            gen_weights<NT>(cl, K, I, np_prev, prev_mode, prev_logc, prev_lse, pst, pw, phz,
                            erow(ering, t - 1, K2), W, &mloc, &cloc);
          }
          lds_barrier();
        }
        optimal_resample<NT>(W, (uint64_t*)W, N, mx, logS, sig_thresh, keys, bcnt, bpos, pre64, tau, parents,
                             sh, cl, red, M, cnt, ch.seed, ch.chain_id, t, Ucur, ph_acc, dbg != nullptr);
        if (dbg && tid == 0) ph_acc[21]++;
      }
      if (dbg && tid == 0) ph_acc[9] += sh.n_sig;
      PH(3);
      int Kk = sh.Kk;
      log_c = sh.log_c;
      if (Kk >= N) { Kk = N; log_c = HYG_NINFF; }
      np = M;
      if (!hyg_isfinitef(log_c)) {
        // ---- unbiased fallback: M categorical draws from log_weights (:42-47)
        mode = MODE_UNBIASED;
        log_c = 0.0f;
        const double lmax = (double)(float)((mx - mx) - logS);  // the largest f32 log-weight
        lds_barrier();  // the sorted keys in the W area are replaced by the regenerated weights
        if (prev_mode == MODE_INIT) {
          gen_weights_init<NT>(cl, K, sh.r_ph, erow(ering, t - 1, K2), W, &mloc, &cloc);
        } else {
          gen_weights<NT>(cl, K, I, np_prev, prev_mode, prev_logc, prev_lse, pst, pw, phz, erow(ering, t - 1, K2),
                          W, &mloc, &cloc);
        }
        lds_barrier();
        auto logit = [&](int n) -> double {
          const double w = W[n];
          return (w > HYG_NINF) ? (double)(float)((w - mx) - logS) : HYG_NINF;
        };
        auto rnd = [&](int q) -> uint64_t {
          return hyg_rand64(ch.seed, ch.chain_id, HYG_RNG_MULTINOMIAL, (uint64_t)t, (uint64_t)q);
        };
        auto out = [&](int q, int n) { parents[q] = n; };
        auto all = [](int) { return true; };
        lds_barrier();
        categorical_block<NT>(N, lmax, logit, M, all, rnd, out, cp128, red);
      } else {
        mode = MODE_OPTIMAL;
        // the top-set path's parents (wave 0) and sh.* are behind its last barrier
        need_bar = fs != FAST_DONE;
      }
    }
    if (need_bar) lds_barrier();
    PH(4);
    // (np <= M <= 64 at the pipeline shape: the gather is wave 0's alone)
    if (wave_id() == 0) serial_begin();
    // ---- gather the ancestors (state, weight, own hazards), record them,
    //      and start the hazard-row prefetch for their children
    StepScalars* rs = (StepScalars*)(rec0 + (size_t)t * rstride);
    uint64_t* rst = (uint64_t*)(rs + 1);
    double* rw = (double*)(rst + M);
    Pf3 pfa;
    uint64_t gs = 0;
    double gw = 0.0;
    Hz4 gh{};
    const bool have_pf = tid < np;  // np <= M <= NT: one ancestor per thread
    if (have_pf) {
      const int a = tid;
      const int n = parents[a];
      uint64_t s;
      Hz4 h;
      if (prev_mode == MODE_INIT) {
        s = init_state(K, n);
        const double2 hc = cl.hz1[0][hyg_st_rc(s)], hk = cl.hz1[1][hyg_st_rk(s)];
        h.lrc = hc.x; h.l1c = hc.y; h.lrk = hk.x; h.l1k = hk.y;
      }
      // the weight of candidate n of step t-1, recomputed (the W area may hold
      // the sort): weight_at's arithmetic with the child formed once. (Reading
      // W[n] instead, with the top-set scratch moved out of the W area at 512
      // threads, measured 0.8 % slower: r03r.)
      double w;
      if (prev_mode == MODE_INIT) {
        const int i = n / K, j = n - (n / K) * K;
        const double* E0 = erow(ering, 0, K2);
        w = (E0[i] + E0[K + j]) + ((i == j) ? cl.lPc[sh.r_ph * K + i] : HYG_NINF);
      } else {
        const int sl = fdiv(n, np_prev, 1.0f / (float)np_prev);
        const int ao = n - sl * np_prev;
        const uint64_t anc = pst[ao];
        const Pf3 pfo = pf[ao];
        const Hz4 hzo = phz[ao];
        const double pao = pw[ao];
        s = tg_xi_hz_sel(cl, K, 1.0f / (float)K, anc, sl, pfo, &h);
        const double tr = tg_trans(cl, K, anc, s, hzo);
        const double* Ep = erow(ering, t - 1, K2);
        w = HYG_NINF;
        if (hyg_isfinite(tr)) {
          const double lg = tr + (Ep[hyg_st_rc(s)] + Ep[K + hyg_st_rk(s)]);
          if (prev_mode == MODE_KEEP) w = pao + lg;
          else if (prev_mode == MODE_UNBIASED) w = (-cl.log_M + prev_lse) + lg;
          else {
            const double v = (double)prev_logc + (pao - prev_lse);
            w = (pao + lg) - (v < 0.0 ? v : 0.0);
          }
        }
      }
      gs = s;
      gw = w;
      gh = h;
      rst[a] = s;
      rw[a] = w;
      pfa = prefetch_rows(md, K, s);  // in flight during the weights
    }
    if (tid == 0) {
      rs->mode = mode; rs->n_par = np; rs->log_c = log_c; rs->r_ph = 0; rs->lse = lse; rs->pad = 0.0;
    }
    if (wave_id() == 0) serial_end();
    if (kURing) {  // steps t+1 .. t+kUR, one per lane, every kUR steps (step t's entry was read above)
      if (wave_id() == NT / 64 - 1 && (t & (kUR - 1)) == 0 && lane_id() < kUR)
        uring[(t + 1 + lane_id()) & (kUR - 1)] =
            hyg_u01f(hyg_rand64(ch.seed, ch.chain_id, HYG_RNG_SYSTEMATIC, (uint64_t)(t + 1 + lane_id()), 0));
    } else if (wave_id() == NT / 64 - 1) {  // a wave with no ancestor (when NT > M): next step's uniform
      const float un = hyg_u01f(hyg_rand64(ch.seed, ch.chain_id, HYG_RNG_SYSTEMATIC, (uint64_t)(t + 1), 0));
      if (lane_id() == 0) sh.Unext = un;
    }
    // emission block prefetch (registers), stored into the ring after the weights
    constexpr int EQ = (kEBlock * 2 * HYG_KMAX + NT - 1) / NT;  // rows of one block per thread
    double ebuf[EQ];
    int e_tot = 0;
    if (eload) {
      const int t0 = (t / kEBlock + 1) * kEBlock;
      const int rows = (T - t0) < kEBlock ? (T - t0) : kEBlock;
      e_tot = rows * K2;
#pragma unroll
      for (int q = 0; q < EQ; ++q) {
        const int i = tid + q * NT;
        ebuf[q] = (i < e_tot) ? Ech[(size_t)t0 * K2 + i] : 0.0;
      }
    }
    np_prev = np;
    prev_mode = mode;
    prev_logc = log_c;
    prev_lse = lse;
    // the new ancestors into the other buffer: its last readers (step t-1's
    // weights) are behind this step's barriers
    if (have_pf) {
      const int o = (cur ^ 1) * M + tid;
      pst0[o] = gs;
      pw0[o] = gw;
      phz0[o] = gh;
    }
    lds_barrier();
    cur ^= 1;
    PH(5);
    // ---- propose and weight the particles of step t
    gen_weights<NT>(cl, K, I, np, mode, log_c, lse, pst0 + cur * M, pw0 + cur * M, phz0 + cur * M,
                    erow(ering, t, K2), W, &mloc, &cloc);
    PH(7);
    N = I * np;
    if (have_pf) pf[tid] = pfa;
    if (eload) {
      double* dst = ering + (size_t)((t / kEBlock + 1) & 1) * kEBlock * K2;
#pragma unroll
      for (int q = 0; q < EQ; ++q) {
        const int i = tid + q * NT;
        if (i < e_tot) dst[i] = ebuf[q];
      }
    }
    PH(8);
    // (every read of red by this step's resampling is behind the gather's barriers)
    block_max_cnt<NT, false>(mloc, cloc, red, &mx, &cnt);
    PH(6);
  }
  // ---- final weights: log normalising constant and run()'s second output
  double logS = HYG_NINF;
  if (mx > HYG_NINF) logS = log_mass_sum<NT>(W, N, mx, red);
  if (tid == 0) {
    int st = sh.status;
    if (st == HYG_OK && !(mx > HYG_NINF)) st = HYG_ENUMERIC;
    status_out[blockIdx.x] = st;
    logz_out[blockIdx.x] = logS + mx;
  }
  if (finalw_out) {
    const int Nmax = c->Nmax;
    for (int n = tid; n < Nmax; n += NT) finalw_out[(size_t)blockIdx.x * Nmax + n] = (n < N) ? W[n] : HYG_NINF;
  }
  if (dbg && tid == 0) {
    for (int k = 0; k < kPh - 1; ++k) dbg[(size_t)blockIdx.x * kPh + k] = ph_acc[k];
    dbg[(size_t)blockIdx.x * kPh + kPh - 1] = (unsigned long long)T;
  }
#undef PH
}

// ------------------------------------------------- backward-kernel rows
// Child of an ancestor (registers) in proposal slot s (wave-uniform), with the
// child's own hazard rows, exactly as tg_xi + child_hz produce them.
struct Child {
  int m, dc, rc, dk, rk;
  Hz4 h;
};
__device__ __forceinline__ Child child_of(const ConstLds& cl, int K, int am, int adc, int arc, int adk, int ark,
                                          const Pf3& p, int s) {
  Child x;
  // c_cont / k_cont: the child's duration continues on the ancestor's
  // prefetched row; merge (m = 0): case continues on the control row; every
  // other row is the d = 1 row of the child's own regime
  bool c_cont, k_cont, merge = false;
  if (s == 0) {
    x.m = am; x.dc = adc + 1; x.rc = arc; x.dk = adk + 1; x.rk = ark;
    c_cont = true; k_cont = true;
  } else if (s < K) {
    const int r = (s - 1 < ark) ? s - 1 : s;
    x.m = 0; x.dc = 1; x.rc = r; x.dk = adk + 1; x.rk = ark;
    c_cont = false; k_cont = true;
  } else if (s < 2 * K - 1) {
    const int qq = s - K;
    const int r = (qq < arc) ? qq : qq + 1;
    x.m = 0; x.dc = adc + 1; x.rc = arc; x.dk = 1; x.rk = r;
    c_cont = true; k_cont = false;
  } else if (s == 2 * K - 1) {
    const int d = (am == 0) ? adc + 1 : 0;
    x.m = 1; x.dc = d; x.rc = arc; x.dk = d; x.rk = arc;
    merge = am == 0;
    c_cont = merge; k_cont = false;
  } else {
    const int j = s - 2 * K, i = j / K, jj = j - i * K;
    x.m = (i == jj); x.dc = 1; x.rc = i; x.dk = 1; x.rk = jj;
    c_cont = false; k_cont = false;
  }
  // value selects (a select of addresses would put p in scratch memory)
  const double2 h1c = cl.hz1[0][x.rc], h1k = cl.hz1[1][x.rk];
  x.h.lrc = c_cont ? p.c1.x : h1c.x;
  x.h.l1c = c_cont ? p.c1.y : h1c.y;
  x.h.lrk = merge ? p.kc.x : (k_cont ? p.k1.x : h1k.x);
  x.h.l1k = merge ? p.kc.y : (k_cont ? p.k1.y : h1k.y);
  return x;
}
// false when tg_trans(x -> next) selects a constant -inf branch whatever the
// table values (the selected value is then -inf; true leaves it to the values)
__device__ __forceinline__ bool trans_possible(int u, const Child& x, int mn, int dcn, int rcn, int dkn, int rkn) {
  const bool lm = ((x.dk < x.dc ? x.dk : x.dc) >= u) || (mn == x.m);
  const bool lc = (dcn == 1) || (dcn == x.dc + 1 && rcn == x.rc);
  bool lk;
  if (mn == 1) lk = (rkn == rcn && dkn == dcn);
  else if (x.m == 1 && dcn != 1) lk = (dkn == 1 && rkn != rcn);
  else if (rcn == x.rk && x.m == 0) lk = (dkn == 1 && rkn != rcn);
  else lk = (dkn == 1) ? (rkn != rcn && rkn != x.rk) : (dkn == x.dk + 1 && rkn == x.rk);
  return lm && lc && lk;
}

// The random bits of step t's B backward draws, hyg_rand64(seed, chain,
// BACKWARD, t, b) for b < B (Philox blocks of 4, one lane per block), into
// rb[0..B); run by one otherwise idle wave one step ahead of their use.
__device__ __forceinline__ void backward_bits(uint64_t* rb, int B, int t, uint64_t seed, uint64_t chain_id) {
  const int q = lane_id();
  if (4 * q < B) {
    const hyg_ph4 r = hyg_philox4x64((uint64_t)HYG_RNG_BACKWARD, (uint64_t)t, (uint64_t)q, 0, seed, chain_id);
    rb[4 * q + 0] = r.v[0]; rb[4 * q + 1] = r.v[1]; rb[4 * q + 2] = r.v[2]; rb[4 * q + 3] = r.v[3];
  }
}

// GW: the full-N weights (the final step's draw and the general path) live in
// the chain's global scratch (ChainDev::wg_offset of `wscr`, the same workspace
// as `ws`, disjoint bytes) instead of LDS, whose W area then holds the lists
// alone (make_layout gw): several chains per CU at the C5 shape. Global W is
// handed between threads behind __syncthreads (its vmcnt(0) release), only on
// the steps that build it.
template <int NT, int KC = 0, int MC = 0, int BC = 0, bool PHS = false, bool GW = false>  // KC > 0: one model shape (see tg_forward_kernel)
__global__ void __launch_bounds__(NT, (NT == 512 ? 1 : 3))
tg_backward_kernel(ModelDev md, const ChainDev* __restrict__ chains, const double* __restrict__ E,
                   const uint8_t* __restrict__ ws, const int32_t* status_in, int16_t* __restrict__ o_merged,
                   int16_t* __restrict__ o_control, int16_t* __restrict__ o_case, float* __restrict__ o_split,
                   float* __restrict__ o_regime, int32_t* status_out, Lay lay_arg,
                   unsigned long long* __restrict__ dbg_arg, uint8_t* __restrict__ wscr) {
  unsigned long long* __restrict__ const dbg = PHS ? dbg_arg : nullptr;  // (see tg_forward_kernel)
  const hyg_tg_consts* __restrict__ c = md.consts;
  const int K = KC ? KC : c->K, M = KC ? MC : c->M, B = KC ? BC : c->B, I = KC ? 2 * KC + KC * KC : c->I,
            K2 = 2 * K, tid = threadIdx.x;
  const Lay lay = KC ? make_layout(KC, MC, BC, MC * (2 * KC + KC * KC), NT, true, GW) : lay_arg;
  const int Lcap = lay.lcap;  // doubles of the list area (Nmax without GW)
  const ChainDev ch = chains[blockIdx.x];
  const int T = ch.T;
  if (status_in[blockIdx.x] != HYG_OK) return;  // uniform
  extern __shared__ __align__(16) unsigned char smem[];
  double* W;
  if constexpr (GW) W = (double*)(wscr + ch.wg_offset);
  else W = (double*)(smem + lay.W);
  // a barrier behind which every thread's W writes are visible (LDS: the
  // LDS-only barrier; global W: a workgroup release of the stores)
  auto w_barrier = [&]() {
    if constexpr (GW) __syncthreads();
    else lds_barrier();
  };
  double* Lg = (double*)(smem + lay.L);
  uint64_t* pst = (uint64_t*)(smem + lay.pst);
  double* pw = (double*)(smem + lay.pw);
  Hz4* phz = (Hz4*)(smem + lay.phz);
  Pf3* pf = (Pf3*)(smem + lay.pf);
  double* ering = (double*)(smem + lay.ering);
  ConstLds& cl = *(ConstLds*)(smem + lay.cl);
  hyg_u128* cp128 = (hyg_u128*)(smem + lay.cp);
  int* idx = (int*)(smem + lay.parents);
  uint64_t* X = (uint64_t*)(smem + lay.X);
  int* grp = (int*)(smem + lay.grp);
  uint64_t* gst = (uint64_t*)(smem + lay.gst);
  uint64_t* rb = (uint64_t*)(smem + lay.rb);
  uint64_t* xo = (uint64_t*)(smem + lay.xo);
  unsigned char* red = smem + lay.red;
  Shared& sh = *(Shared*)(smem + lay.sh);
  // Trajectories and test-function means of time tt
  // (run_inference_two_groups.py:233-240, 294-314) from the states wave 0
  // sampled (xo[tt & 1]), one wave, trajectory b on lane b (B <= 64). From 128
  // threads on they are written by wave 1 during the next step's draw, off
  // wave 0's serial path (deferred by one step; the state buffer is double).
  constexpr int kOutWave = NT >= 128 ? 1 : 0;
  auto write_outputs = [&](int tt) {
    const int lane = lane_id();
    const bool v = lane < B;
    uint64_t x = 0;
    if (v) {
      x = xo[(tt & 1) * B + lane];
      const size_t o = (size_t)(ch.out_begin + tt) * B + lane;
      o_merged[o] = (int16_t)hyg_st_m(x);
      o_control[2 * o + 0] = (int16_t)hyg_st_dc(x);
      o_control[2 * o + 1] = (int16_t)hyg_st_rc(x);
      o_case[2 * o + 0] = (int16_t)hyg_st_dk(x);
      o_case[2 * o + 1] = (int16_t)hyg_st_rk(x);
    }
    int myc = __builtin_popcountll(__ballot(v && hyg_st_m(x) == 0));
    for (int r = 0; r < K; ++r) {
      const int cc = __builtin_popcountll(__ballot(v && hyg_st_rc(x) == r));
      const int ck = __builtin_popcountll(__ballot(v && hyg_st_rk(x) == r));
      myc = (lane == 1 + r) ? cc : ((lane == 1 + K + r) ? ck : myc);
    }
    if (lane < 2 * K + 1) {
      const float vv = (float)myc / (float)B;
      if (lane == 0) o_split[ch.out_begin + tt] = vv;
      else o_regime[(size_t)(ch.out_begin + tt) * K2 + (lane - 1)] = vv;
    }
  };
  int pend = -1;  // the time whose outputs are still to be written (B <= 64)

  const uint8_t* rec0 = ws + ch.ws_offset;
  const size_t rstride = record_bytes(M);
  const double* Ech = E + ch.site_begin * K2;
  load_consts(cl, c, md);
  if (tid == 0) sh.status = HYG_OK;
  unsigned long long* ph_acc = sh.ph;
  if (tid < kPh) ph_acc[tid] = 0;
#define BPH(k)                                                     \
  if (dbg && tid == 0) {                                           \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    ph_acc[k] += now_ - ph_acc[kPh - 1];                                \
    ph_acc[kPh - 1] = now_;                                             \
  }
  // Records are read ahead in two stages: step t consumes record t from LDS,
  // stores record t-1 (read during step t+1) with its hazard rows (issued at
  // the top of step t), and issues the read of record t-2.
  auto rec_ptr = [&](int tt) { return rec0 + (size_t)tt * rstride; };
  StepScalars s = *(const StepScalars*)rec_ptr(T - 1);
  if (tid < s.n_par) {
    const int o0 = ((T - 1) & 1) * M + tid;  // record t lives in LDS buffer t & 1
    const uint64_t* rst = (const uint64_t*)(rec_ptr(T - 1) + sizeof(StepScalars));
    const uint64_t st = rst[tid];
    pst[o0] = st;
    pw[o0] = ((const double*)(rst + M))[tid];
    const double2 hc = hz_at(md, K, 0, hyg_st_rc(st), hyg_st_dc(st));
    const double2 hk = hz_at(md, K, 1, hyg_st_rk(st), hyg_st_dk(st));
    Hz4 h;
    h.lrc = hc.x; h.l1c = hc.y; h.lrk = hk.x; h.l1k = hk.y;
    phz[o0] = h;
    pf[o0] = prefetch_rows(md, K, st);
  }
  // The record pipeline of the steps below (the reads of records t-1 / t-2,
  // the hazard rows of record t-1's ancestors and its LDS store) is the last
  // wave's work when M <= 64, ancestor a on its lane a: that wave has no slot
  // of its own in the list phase at 8 waves (d_c >= 3: K + 1 slots), so the
  // loads leave the waves whose list work the draw waits for. Otherwise thread
  // a holds ancestor a.
  const int ra = (M <= 64 && NT >= 128) ? ((wave_id() == NT / 64 - 1) ? lane_id() : M) : tid;
  // stage-1 registers: record t-1
  StepScalars s1{};
  uint64_t st1 = 0;
  double w1 = 0.0;
  if (T >= 2) {
    s1 = *(const StepScalars*)rec_ptr(T - 2);
    if (ra < M) {
      const uint64_t* rst = (const uint64_t*)(rec_ptr(T - 2) + sizeof(StepScalars));
      st1 = rst[ra];
      w1 = ((const double*)(rst + M))[ra];
    }
  }
  {
    const int bi = (T - 1) / kEBlock;
    load_eblock(ering, Ech, bi, T, K2, NT);
    if (bi > 0) load_eblock(ering, Ech, bi - 1, T, K2, NT);
  }
  lds_barrier();
  if (dbg && tid == 0) ph_acc[kPh - 1] = __builtin_amdgcn_s_memtime();

  for (int t = T - 1; t >= 0; --t) {
    // ---- regenerate the particles of step t from its record (LDS buffer t & 1;
    //      record t-1 is stored into the other buffer during this step)
    const int bt = t & 1;
    const double* Et = erow(ering, t, K2);
    const int np = s.n_par;
    const uint64_t* P = pst + bt * M;
    const double* PW = pw + bt * M;
    const Hz4* PHZ = phz + bt * M;
    const Pf3* PF = pf + bt * M;
    const float rnp = (np > 0) ? 1.0f / (float)np : 0.0f;
    const int N = (s.mode == MODE_INIT) ? K * K : I * np;
    double mloc = HYG_NINF;
    int cloc = 0;
    // The rows of the backward kernel need the weights of the few candidates
    // that can reach a trajectory's next state only (the list path); all N
    // weights are built for the final step's draw and for the general path.
    const bool fast = (s.mode != MODE_INIT) && np <= 64 && B <= 64 && Lcap >= 192 && t != T - 1;
    bool w_ready = false;
    auto make_W = [&]() {
      if (s.mode == MODE_INIT) gen_weights_init<NT>(cl, K, s.r_ph, Et, W, &mloc, &cloc);
      else gen_weights<NT>(cl, K, I, np, s.mode, s.log_c, s.lse, P, PW, PHZ, Et, W, &mloc, &cloc);
      w_ready = true;
    };
    if (!fast) make_W();
    BPH(0);
    // ---- hazard rows of record t-1's ancestors (arrived: read during step t+1)
    double2 h1c = make_double2(0.0, 0.0), h1k = make_double2(0.0, 0.0);
    Pf3 pf1;
    const bool have1 = (t > 0) && (ra < s1.n_par);
    if (have1) {
      h1c = hz_at(md, K, 0, hyg_st_rc(st1), hyg_st_dc(st1));
      h1k = hz_at(md, K, 1, hyg_st_rk(st1), hyg_st_dk(st1));
      pf1 = prefetch_rows(md, K, st1);
    }
    // ---- issue the read of record t-2. Its scalars come in as a vector load
    //      (lane i < 8: dword i) and are unpacked at the end of the step: a
    //      scalar load shares lgkmcnt with LDS, so the step's first LDS wait
    //      (or the spill of its SGPRs) waited out its trip to L2 on every wave.
    uint32_t sv2 = 0;
    uint64_t st2 = 0;
    double w2 = 0.0;
    if (t >= 2) {
      const uint8_t* rn = rec_ptr(t - 2);
      if (lane_id() < 8) sv2 = ((const uint32_t*)rn)[lane_id()];
      if (ra < M) {
        const uint64_t* rst = (const uint64_t*)(rn + sizeof(StepScalars));
        st2 = rst[ra];
        w2 = ((const double*)(rst + M))[ra];
      }
    }
    // ---- emission block t/EB - 2 into the half freed after this step's rows
    const bool eload = (t % kEBlock) == 0 && t >= 2 * kEBlock;
    constexpr int EQ = (kEBlock * 2 * HYG_KMAX + NT - 1) / NT;  // rows of one block per thread
    double ebuf[EQ];
    const int e_tot = eload ? kEBlock * K2 : 0;
    if (eload) {
      const int t0 = (t / kEBlock - 2) * kEBlock;
#pragma unroll
      for (int q = 0; q < EQ; ++q) {
        const int i = tid + q * NT;
        ebuf[q] = (i < e_tot) ? Ech[(size_t)t0 * K2 + i] : 0.0;
      }
    }
    if (!fast) w_barrier();  // W written by every thread (the list path reads only LDS written behind barriers)
    BPH(1);
    auto state_of = [&](int n) -> uint64_t {
      if (s.mode == MODE_INIT) return init_state(K, n);
      const int sl = fdiv(n, np, rnp);
      return tg_xi(K, P[n - sl * np], sl);
    };
    auto hz_of_n = [&](int n) -> Hz4 {
      if (s.mode == MODE_INIT) {
        const int i = n / K, j = n - (n / K) * K;
        Hz4 h;
        h.lrc = cl.hz1[0][i].x; h.l1c = cl.hz1[0][i].y; h.lrk = cl.hz1[1][j].x; h.l1k = cl.hz1[1][j].y;
        return h;
      }
      const int sl = fdiv(n, np, rnp), a = n - sl * np;
      return child_hz(cl, K, P[a], sl, PF[a], md);
    };
    const int rbs = ((B + 3) / 4) * 4;  // stride of the two draw-bit buffers
    const bool pre_bits = B <= 64 && NT >= 128;
    if (pre_bits && t == T - 1 && t >= 1 && wave_id() == NT / 64 - 1)
      backward_bits(rb + ((t - 1) & 1) * rbs, B, t - 1, ch.seed, ch.chain_id);
    auto rnd = [&](int b) -> uint64_t {
      return hyg_rand64(ch.seed, ch.chain_id, HYG_RNG_BACKWARD, (uint64_t)t, (uint64_t)b);
    };
    bool fail = false;
    if (t == T - 1) {
      // ---- B draws from the final weights (:383-385)
      const double lmax = block_max<NT>(mloc, red);
      if (!(lmax > HYG_NINF)) { if (tid == 0) sh.status = HYG_ENUMERIC; lds_barrier(); break; }
      auto logit = [&](int n) -> double { return W[n]; };
      auto out = [&](int q, int n) { idx[q] = n; };
      auto all = [](int) { return true; };
      lds_barrier();
      categorical_block<NT>(N, lmax, logit, B, all, rnd, out, cp128, red);
      lds_barrier();  // idx for the trajectory tail
    } else {
      // ---- backward-kernel rows (:400-435), one per distinct next state.
      // B <= 64: the groups (distinct next states, in order of first
      // occurrence) were formed by wave 0 at the end of step t+1.
      if (B > 64) {
        if (tid == 0) {
          int ng = 0;
          for (int b = 0; b < B; ++b) {
            int g = 0;
            while (g < ng && gst[g] != X[b]) ++g;
            if (g == ng) gst[ng++] = X[b];
            grp[b] = g;
          }
          sh.ng = ng;
        }
        lds_barrier();
      }
      const int ng = sh.ng;
      if (dbg && tid == 0) ph_acc[10] += ng;
      BPH(2);
      for (int g = 0; g < ng; ++g) {
        const uint64_t xn = gst[g];
        const int mn = hyg_st_m(xn), dcn = hyg_st_dc(xn), rcn = hyg_st_rc(xn), dkn = hyg_st_dk(xn),
                  rkn = hyg_st_rk(xn);
        bool one_wave = false;
        int L = 0, seg_incl = 0, nseg = 0;
        constexpr int kSeg = 16;
        bool segp = false;
        int* lst_n = (int*)cp128;  // list indices (cp area, NT+1 u128 = 4(NT+1) ints)
        double* lst_l = Lg;        // list logits (the W area: W is not built on the list path)
        if (fast) {
          // ---- finite logits l_n = log f(xn | x_n) + W_n, gathered into a short
          //      list (n, l_n): only a few dozen of the N candidates can reach xn.
          // Only slots whose child can have d_c = dcn - 1 (or a control change
          // point when dcn = 1) can reach xn: lc of tg_trans is a constant -inf
          // otherwise (ancestors always have d_c >= 1).
          int r0a, r0b, r1a, r1b;
          if (dcn >= 3) {  // A, C, D; the case side of trans_possible leaves fewer:
            r0a = 0; r0b = 1; r1a = K; r1b = 2 * K;
            if (mn == 1 && cl.u > 1) {
              r1a = 2 * K - 1;  // D: a C child (m = 0, d_k = 1 < u) cannot merge
            } else if (mn == 0 && dkn >= 2) {
              // unmerged xn continuing its case segment: x.m = 0 (no D), x.d_k =
              // d_k' - 1 and x.r_k = r_k' (a C child has d_k = 1, r_k = its slot's
              // regime; candidates have r_c = r_c' as lc requires)
              if (dkn == 2 && rkn != rcn) {
                r1a = K + (rkn < rcn ? rkn : rkn - 1);
                r1b = r1a + 1;
              } else {
                r1a = r1b = 2 * K;
              }
            }
          }
          else if (dcn == 2) { r0a = 1; r0b = K; r1a = 2 * K + rcn * K; r1b = r1a + K; }   // B, E(i = rcn)
          else { r0a = 0; r0b = I; r1a = I; r1b = I; }
          const int nseg0 = r0b - r0a;
          nseg = nseg0 + (r1b - r1a);
          // Segment list (at most kSeg reachable slots): slot v's finite logits
          // at [64 v, 64 v + c_v) in lane order, so the list is in n order by
          // construction: no shared counter, no atomics, no rank sort
          segp = nseg <= kSeg && Lcap >= 64 * kSeg + 160 && 4 * (NT + 1) >= 64 * kSeg;
          if (!segp) {
            if (tid == 0) sh.cnt = 0;
            lds_barrier();  // (the segment path: every reader of the areas is behind the last group's barrier)
          }
          const int cap = (4 * (NT + 1) < Lcap) ? 4 * (NT + 1) : Lcap;
          constexpr int NW = NT / 64;
          const int lane = lane_id(), wv = wave_id();
          const bool act = lane < np;
          const uint64_t par = act ? P[lane] : 0;
          const int am = hyg_st_m(par), adc = hyg_st_dc(par), arc = hyg_st_rc(par), adk = hyg_st_dk(par),
                    ark = hyg_st_rk(par);
          Pf3 pa{};
          Hz4 hanc{};
          double pwa = 0.0;
          if (act) {  // the ancestor's rows, once per group (not per slot)
            pa = PF[lane];
            hanc = PHZ[lane];
            pwa = PW[lane];
          }
          // the reachable slots, both ranges, round-robin over the waves (one
          // slot per wave from 8 waves on at d_c >= 3)
          {
            for (int sgv = wv; sgv < nseg; sgv += NW) {  // sgv: segment of slot sl
              const int sl = (sgv < nseg0) ? r0a + sgv : r1a + (sgv - nseg0);
              const Child x = child_of(cl, K, am, adc, arc, adk, ark, pa, sl);
              const bool poss = act && trans_possible(cl.u, x, mn, dcn, rcn, dkn, rkn);
              if (__ballot(poss) == 0) {  // nothing in this slot reaches xn
                if (segp && lane == 0) sh.segc[sgv] = 0;
                continue;
              }
              double l = HYG_NINF;
              if (poss) {
                // weight_at with the ancestor in registers and the child from
                // child_of (the same state as tg_xi): same operands, same order
                const uint64_t xs = hyg_st_pack(x.m, x.dc, x.rc, x.dk, x.rk);
                const double tr = tg_trans_sel(cl.lPm[am * 2 + x.m], cl.lPc[arc * K + x.rc], cl.lU1, cl.lU2, cl.u,
                                               am, adc, arc, adk, ark, xs, hanc);
                double w = HYG_NINF;
                if (hyg_isfinite(tr)) {
                  const double lg = tr + (Et[x.rc] + Et[K + x.rk]);
                  if (s.mode == MODE_KEEP) w = pwa + lg;
                  else if (s.mode == MODE_UNBIASED) w = (-cl.log_M + s.lse) + lg;
                  else {
                    const double vv = (double)s.log_c + (pwa - s.lse);
                    w = (pwa + lg) - (vv < 0.0 ? vv : 0.0);
                  }
                }
                if (w > HYG_NINF) {
                  const double f = tg_trans_sel(cl.lPm[x.m * 2 + mn], cl.lPc[x.rc * K + rcn], cl.lU1, cl.lU2,
                                                cl.u, x.m, x.dc, x.rc, x.dk, x.rk, xn, x.h);
                  if (hyg_isfinite(f)) l = f + w;
                }
              }
              const unsigned long long mask = __ballot(l > HYG_NINF);
              if (segp) {
                if (lane == 0) sh.segc[sgv] = (int)__popcll(mask);
                if (l > HYG_NINF) {
                  const int pos = 64 * sgv + lanes_below(mask);
                  lst_n[pos] = sl * np + lane;
                  lst_l[pos] = l;
                }
              } else if (mask) {
                int base = 0;
                if (lane == 0) base = atomicAdd(&sh.cnt, __popcll(mask));
                base = __builtin_amdgcn_readfirstlane(base);
                if (l > HYG_NINF) {
                  const int pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
                  if (pos < cap) { lst_n[pos] = sl * np + lane; lst_l[pos] = l; }
                }
              }
            }
          }
          lds_barrier();
          BPH(3);
          // segment path: inclusive prefix of the segment counts in every wave
          seg_incl = segp ? wave_incl_int(lane_id() < nseg ? sh.segc[lane_id()] : 0) : 0;
          L = segp ? __builtin_amdgcn_readlane(seg_incl, 63) : sh.cnt;
          if (dbg && tid == 0) ph_acc[11] += L;
          if (L == 0) { fail = true; break; }  // uniform: every logit -inf
          one_wave = L <= 64 && Lcap >= 192;
        }
        if (pre_bits && g == 0 && t >= 1 && wave_id() == NT / 64 - 1)  // next step's bits, while wave 0 draws
          backward_bits(rb + ((t - 1) & 1) * rbs, B, t - 1, ch.seed, ch.chain_id);
        if (one_wave) {
          // ---- one wave: order the list by n, exact masses, scan, draws
          if (wave_id() == 0) {
            serial_begin();
            const int lane = lane_id();
            const bool v = lane < L;
            double sv;
            hyg_u128* cdfa;
            int* cn;
            if (segp) {
              // list position `lane` lies in the segment whose inclusive end
              // is the first one above it (lanes q >= nseg hold the total L:
              // every valid lane is below it, so all kSeg ends are read, each
              // from a constant lane)
              int seg = 0, base = 0;
#pragma unroll
              for (int q = 0; q < kSeg; ++q) {
                const int iv = __builtin_amdgcn_readlane(seg_incl, q);
                seg += (iv <= lane) ? 1 : 0;
                base = (iv <= lane) ? iv : base;
              }
              const int at = 64 * seg + (lane - base);
              const int myn = v ? lst_n[at] : 0;
              sv = v ? lst_l[at] : HYG_NINF;
              cdfa = (hyg_u128*)(Lg + 64 * kSeg);       // behind the segments
              cn = (int*)(Lg + 64 * kSeg + 128);        // the list's indices in n order
              if (v) cn[lane] = myn;
            } else {
              const int myn = v ? lst_n[lane] : 0x7fffffff;
              const double myl = v ? lst_l[lane] : HYG_NINF;
              int rank = 0;
#pragma unroll 4
              for (int j = 0; j < L; ++j) rank += (lst_n[j] < myn) ? 1 : 0;  // broadcast reads
              __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront", "local");
              if (v) { lst_n[rank] = myn; lst_l[rank] = myl; }
              __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront", "local");
              sv = v ? lst_l[lane] : HYG_NINF;
              cdfa = (hyg_u128*)(Lg + 64);  // behind the 64 list logits
              cn = lst_n;
            }
            BPH(12);
            const double lmax = wave_max(sv);
            BPH(13);
            hyg_u128 ms = hyg_u128_zero();
            if (v) ms = hyg_exp_fix100(sv - lmax);
            BPH(14);
            const hyg_u128 cdf = wave_incl128(ms);
            BPH(15);
            hyg_u128 total;
            total.lo = rdlane64(cdf.lo, L - 1);
            total.hi = rdlane64(cdf.hi, L - 1);
            if (v) cdfa[lane] = cdf;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront", "local");
            BPH(16);
            // lane b draws for trajectory b: first list entry with cdf > target
            if (lane < B && grp[lane] == g) {
              const uint64_t bits = pre_bits ? rb[(t & 1) * rbs + lane] : rnd(lane);  // = hyg_rand64(.., t, lane)
              const hyg_u128 tb = hyg_scale_target(bits, total);
              int lo = 0, hi = L - 1;
              while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (hyg_u128_lt(tb, cdfa[mid])) hi = mid; else lo = mid + 1;
              }
              idx[lane] = cn[lo];
            }
            serial_end();
          } else if (kOutWave > 0 && g == 0 && pend >= 0 && wave_id() == kOutWave) {
            write_outputs(pend);
          }
          if (kOutWave > 0 && g == 0) pend = -1;
          BPH(4);
          if (g + 1 < ng) lds_barrier();  // the next group's list reuses the areas wave 0 read
        } else {
          // ---- general case: logits of all N in index order (built in place of
          //      the weights), block categorical
          if (kOutWave > 0 && g == 0 && pend >= 0) {
            if (wave_id() == kOutWave) write_outputs(pend);
            pend = -1;
          }
          if (!w_ready) {
            w_barrier();  // the list areas (= the W area) are reused below
            make_W();
            w_barrier();
          }
          double m = HYG_NINF;
          for (int n = tid; n < N; n += NT) {
            const double w = W[n];
            double l = HYG_NINF;
            if (w > HYG_NINF) {
              const double f = tg_trans(cl, K, state_of(n), xn, hz_of_n(n));
              if (hyg_isfinite(f)) l = f + w;
            }
            W[n] = l;  // each n read and rewritten by one thread
            m = dmax(m, l);
          }
          if constexpr (GW) __syncthreads();  // the categorical reads other threads' logits
          w_ready = false;  // W holds this group's logits now
          const double lmax = block_max<NT>(m, red);
          if (!(lmax > HYG_NINF)) { fail = true; break; }  // uniform: every logit -inf
          auto logit = [&](int n) -> double { return W[n]; };
          auto in_g = [&](int b) { return grp[b] == g; };
          auto out = [&](int b, int n) { idx[b] = n; };
          categorical_block<NT>(N, lmax, logit, B, in_g, rnd, out, cp128, red);
          lds_barrier();
        }
        BPH(5);
      }
      if (fail) { if (tid == 0) sh.status = HYG_ENUMERIC; lds_barrier(); break; }
    }
    // ---- trajectories and test-function means at t (run_inference_two_groups.py:233-240, 294-314)
    if (B <= 64) {
      // wave 0 alone: trajectory b on lane b (idx written by this wave's draws,
      // or behind a barrier), then the groups of step t-1's next states
      if (wave_id() == 0) {
        serial_begin();
        wave_lds_sync();
        const int lane = lane_id();
        const bool v = lane < B;
        uint64_t x = 0;
        if (v) {
          x = state_of(idx[lane]);
          xo[(t & 1) * B + lane] = x;
        }
        if constexpr (kOutWave == 0) {
          wave_lds_sync();
          write_outputs(t);
        }
        BPH(6);
        if (t > 0) {
          // distinct states in order of first occurrence, by ballots: one
          // iteration per group (about one per step)
          uint64_t rem = __ballot(v);
          int gi = 0, mg = 0;
          while (rem) {  // uniform
            const int ld = (int)__builtin_ctzll(rem);
            const uint64_t xv = rdlane64(x, ld);
            const uint64_t eq = __ballot(v && x == xv);
            if (lane == 0) gst[gi] = xv;
            mg = ((eq >> lane) & 1) ? gi : mg;
            rem &= ~eq;
            ++gi;
          }
          if (v) grp[lane] = mg;
          if (lane == 0) sh.ng = gi;
        }
        serial_end();
      }
    } else {
      for (int b = tid; b < B; b += NT) {
        const uint64_t x = state_of(idx[b]);
        X[b] = x;
        const size_t o = (size_t)(ch.out_begin + t) * B + b;
        o_merged[o] = (int16_t)hyg_st_m(x);
        o_control[2 * o + 0] = (int16_t)hyg_st_dc(x);
        o_control[2 * o + 1] = (int16_t)hyg_st_rc(x);
        o_case[2 * o + 0] = (int16_t)hyg_st_dk(x);
        o_case[2 * o + 1] = (int16_t)hyg_st_rk(x);
      }
      lds_barrier();
      if (tid < 2 * K + 1) {
        int cntv = 0;
        for (int b = 0; b < B; ++b) {
          const uint64_t x = X[b];
          if (tid == 0) cntv += (hyg_st_m(x) == 0);
          else if (tid <= K) cntv += (hyg_st_rc(x) == tid - 1);
          else cntv += (hyg_st_rk(x) == tid - 1 - K);
        }
        const float v = (float)cntv / (float)B;
        if (tid == 0) o_split[ch.out_begin + t] = v;
        else o_regime[(size_t)(ch.out_begin + t) * K2 + (tid - 1)] = v;
      }
    }
    // ---- record t-1 (+ hazard rows) into the other buffer: its last readers
    //      (step t+1) are behind this step's barriers; the emission block into
    //      the ring half whose rows this step no longer reads
    if (have1) {
      const int o = (bt ^ 1) * M + ra;
      pst[o] = st1;
      pw[o] = w1;
      Hz4 h;
      h.lrc = h1c.x; h.l1c = h1c.y; h.lrk = h1k.x; h.l1k = h1k.y;
      phz[o] = h;
      pf[o] = pf1;
    }
    if (eload) {
      double* dst = ering + (size_t)((t / kEBlock - 2) & 1) * kEBlock * K2;
#pragma unroll
      for (int q = 0; q < EQ; ++q) {
        const int i = tid + q * NT;
        if (i < e_tot) dst[i] = ebuf[q];
      }
    }
    lds_barrier();
    if (kOutWave > 0 && B <= 64) pend = t;
    s = s1;
    st1 = st2;
    w1 = w2;
    {
      // (StepScalars: mode, n_par, log_c, r_ph, lse; zero before record 0)
      s1.mode = __builtin_amdgcn_readlane((int)sv2, 0);
      s1.n_par = __builtin_amdgcn_readlane((int)sv2, 1);
      s1.log_c = __builtin_bit_cast(float, __builtin_amdgcn_readlane((int)sv2, 2));
      s1.r_ph = __builtin_amdgcn_readlane((int)sv2, 3);
      s1.lse = d_of(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)sv2, 5) << 32) |
                    (uint32_t)__builtin_amdgcn_readlane((int)sv2, 4));
      s1.pad = 0.0;
    }
  }
  lds_barrier();
  if (kOutWave > 0 && B <= 64 && pend >= 0 && wave_id() == kOutWave) write_outputs(pend);
  if (tid == 0 && status_out) status_out[blockIdx.x] = sh.status;
  if (dbg && tid == 0) {
    for (int k = 0; k < kPh - 1; ++k) dbg[(size_t)blockIdx.x * kPh + k] = ph_acc[k];
    dbg[(size_t)blockIdx.x * kPh + kPh - 1] = (unsigned long long)T;
  }
#undef BPH
}

// -------------------------------------------------------------- launchers
// Optional per-kernel timing with HIP events recorded on the launch stream
// (bench.py reads them back with hyg_tg_last_kernel_ms). The events belong to
// the device they were created on and are recreated when the calling thread's
// device changes; one mutex orders every use of them.
namespace {
std::mutex g_ev_mu;
bool g_timing = false;
int g_ev_dev = -1;
hipEvent_t g_ev[6] = {};
bool g_ev_used[3] = {false, false, false};
void ev_record(int k, bool end, hipStream_t s) {
  std::lock_guard<std::mutex> lock(g_ev_mu);
  if (!g_timing) return;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return;
  if (dev != g_ev_dev) {  // new device: the old device's events cannot be recorded here
    for (int i = 0; i < 6; ++i) {
      if (g_ev[i]) (void)hipEventDestroy(g_ev[i]);
      g_ev[i] = nullptr;
    }
    for (int i = 0; i < 3; ++i) g_ev_used[i] = false;
    g_ev_dev = dev;
  }
  hipEvent_t& e = g_ev[2 * k + (end ? 1 : 0)];
  if (!e) (void)hipEventCreate(&e);
  (void)hipEventRecord(e, s);
  g_ev_used[k] = true;
}
// CUs of each device (the launch-width and tail-overlap choices depend on
// them), cached per device: a process that switches devices (hyg_set_device)
// sees each device's own count. hyg_tg_set_device_cus overrides an entry
// (tests fake devices of other sizes); 0 = unknown / query again.
constexpr int kMaxDevices = 64;
std::atomic<int> g_cus[kMaxDevices];
int query_cus(int dev) {
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) return 0;
  return n;
}
int cus_of(int dev) {
  if (dev < 0) return 0;
  if (dev >= kMaxDevices) return query_cus(dev);
  int n = g_cus[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  n = query_cus(dev);
  if (n > 0) g_cus[dev].store(n, std::memory_order_relaxed);
  return n;
}
int device_cus() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  const int n = cus_of(dev);
  return n > 0 ? n : 256;
}
// Threads per chain workgroup. HYG_THREADS (or HYG_THREADS_FWD / _BWD) if set.
// Otherwise by what the launch's chains leave of the GPU:
//  - the forward's LDS at 256 threads already forces one workgroup per CU
//    (K = 12, C5: 145 KB): 512 (forward) / 768 (backward), more waves on the
//    CU's one chain;
//  - at most one chain per CU (e.g. an 8-GPU rank of the C3 job, 73 chains):
//    kLowOccThreads (forward) / kLowOccThreadsBwd (backward), whose extra
//    waves shorten the parallel phases of each step of the sequential chain
//    (HYG_LOWOCC_THREADS: 256, 512 or 768 for both);
//  - else 256, up to three chains per CU (<= 168 VGPRs: C3 on one GPU, 582
//    chains; an 8-GPU rank of C4, 291). A 384-thread workgroup does not buy
//    two chains per CU: its six waves land 2-2-1-1 on the SIMDs, so a second
//    one would need four waves on a SIMD that holds three.
int g_force_threads[2] = {0, 0};  // hyg_tg_force_threads (tests): forward, backward; 0 = automatic
bool valid_width(int x) { return x == 64 || x == 128 || x == 256 || x == 512 || x == 768; }
int threads_per_chain(bool backward, const hyg_tg_consts& c, int n_chains) {
  if (g_force_threads[backward ? 1 : 0]) return g_force_threads[backward ? 1 : 0];
  static int env[2] = {-1, -1};
  static int lowocc = -1;  // 0: the defaults kLowOccThreads / kLowOccThreadsBwd
  const int k = backward ? 1 : 0;
  if (env[k] < 0) {
    const char* v = tuning_env(backward ? "HYG_THREADS_BWD" : "HYG_THREADS_FWD");
    if (!v) v = tuning_env("HYG_THREADS");
    const int x = v ? atoi(v) : 0;
    env[k] = valid_width(x) ? x : 0;
  }
  if (lowocc < 0) {
    const char* v = tuning_env("HYG_LOWOCC_THREADS");
    const int x = v ? atoi(v) : 0;
    lowocc = (x == 256 || x == 512 || x == 768) ? x : 0;
  }
  if (env[k]) return env[k];
  const int def = backward ? kDefaultThreadsBwd : kDefaultThreads;
  if (c.M > 64) return def;  // the wider kernels assume the pipeline's M <= 64 (one ancestor per lane)
  const size_t lds = make_layout(c.K, c.M, c.B, c.Nmax, def, false).total;
  // (C5: the backward's list path keeps its 12 waves busy: 768 threads, 6 %
  // faster than 512 in r03d; the forward is faster at 512). With more chains
  // than CUs the C5 backward runs at 256 threads with its full-N weights in
  // global memory (GW): three chains per CU instead of one.
  if (backward && backward_global_w(c) && n_chains > device_cus()) return 256;
  if (2 * lds > 160 * 1024) return backward ? 768 : 512;
  if (n_chains <= device_cus()) return lowocc ? lowocc : (backward ? kLowOccThreadsBwd : kLowOccThreads);
  return def;
}
}  // namespace

int tg_threads_per_chain(const hyg_tg_consts& c, int n_chains) { return threads_per_chain(false, c, n_chains); }
int tg_force_threads(int fwd, int bwd) {
  if ((fwd && !valid_width(fwd)) || (bwd && !valid_width(bwd))) return HYG_EINVAL;
  g_force_threads[0] = fwd;
  g_force_threads[1] = bwd;
  return HYG_OK;
}

int tg_device_cus(int dev) { return cus_of(dev); }
int tg_set_device_cus(int dev, int cus) {
  if (dev < 0 || dev >= kMaxDevices || cus < 0) return HYG_EINVAL;
  g_cus[dev].store(cus, std::memory_order_relaxed);
  return HYG_OK;
}

void set_kernel_timing(bool on) {
  std::lock_guard<std::mutex> lock(g_ev_mu);
  g_timing = on;
}

int last_kernel_ms(float* out3) {
  std::lock_guard<std::mutex> lock(g_ev_mu);
  for (int k = 0; k < 3; ++k) {
    out3[k] = -1.0f;
    if (!g_ev_used[k] || !g_ev[2 * k] || !g_ev[2 * k + 1]) continue;
    if (hipEventSynchronize(g_ev[2 * k + 1]) != hipSuccess) return HYG_EDEVICE;
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, g_ev[2 * k], g_ev[2 * k + 1]) != hipSuccess) return HYG_EDEVICE;
    out3[k] = ms;
  }
  return HYG_OK;
}

size_t forward_lds_bytes(const hyg_tg_consts& c, int n_chains) {
  return make_layout(c.K, c.M, c.B, c.Nmax, threads_per_chain(false, c, n_chains), false).total;
}
static bool bwd_gw(const hyg_tg_consts& c, int NT);
size_t tg_layout_bytes(const hyg_tg_consts& c, int threads, bool backward) {
  return valid_width(threads)
             ? make_layout(c.K, c.M, c.B, c.Nmax, threads, backward, backward && bwd_gw(c, threads)).total
             : 0;
}
size_t backward_lds_bytes(const hyg_tg_consts& c, int n_chains) {
  const int nt = threads_per_chain(true, c, n_chains);
  return make_layout(c.K, c.M, c.B, c.Nmax, nt, true, bwd_gw(c, nt)).total;
}

int launch_emission(const ModelDev& md, const hyg_tg_consts& c, const uint16_t* meth_c, const uint16_t* tot_c,
                    int s_c, const uint16_t* meth_k, const uint16_t* tot_k, int s_k, int64_t n_sites, double* E,
                    void* stream) {
  if (n_sites <= 0) return HYG_OK;
  int64_t blocks = (n_sites + kETile - 1) / kETile;
  if (blocks > 256 * 16) blocks = 256 * 16;
  ev_record(0, false, (hipStream_t)stream);
  const size_t lds = sizeof(double) * kETile * 2 * c.K;
  const int L = md.nmax_reads + 1;
  if (md.bbt && c.K == 6) {
    hipLaunchKernelGGL(tg_emission_tab_kernel<6>, dim3((unsigned)blocks), dim3(kETile), lds, (hipStream_t)stream,
                       md.bbt, L, c.K, meth_c, tot_c, s_c, meth_k, tot_k, s_k, n_sites, E);
  } else if (md.bbt && c.K == 12) {
    hipLaunchKernelGGL(tg_emission_tab_kernel<12>, dim3((unsigned)blocks), dim3(kETile), lds, (hipStream_t)stream,
                       md.bbt, L, c.K, meth_c, tot_c, s_c, meth_k, tot_k, s_k, n_sites, E);
  } else if (md.bbt) {
    hipLaunchKernelGGL(tg_emission_tab_kernel<0>, dim3((unsigned)blocks), dim3(kETile), lds, (hipStream_t)stream,
                       md.bbt, L, c.K, meth_c, tot_c, s_c, meth_k, tot_k, s_k, n_sites, E);
  } else {
    hipLaunchKernelGGL(tg_emission_kernel, dim3((unsigned)blocks), dim3(kETile), lds, (hipStream_t)stream, md.lf,
                       md.lg, md.cst, L, c.K, meth_c, tot_c, s_c, meth_k, tot_k, s_k, n_sites, E);
  }
  ev_record(0, true, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? HYG_OK : HYG_EDEVICE;
}

// The kernel instantiation for a launch: the pipeline's model shape (K = 6,
// M = 50, B = 25, the C3/C4 configurations) at 256 threads has its own
// compile-time-shaped instantiation (HYG_NO_SHAPE=1: the generic one).
using FwdFn = decltype(&tg_forward_kernel<64>);
using BwdFn = decltype(&tg_backward_kernel<64>);
static bool shape_specialised(const hyg_tg_consts& c) {
  static const bool off = tuning_env("HYG_NO_SHAPE") != nullptr;
  return !off && c.K == 6 && c.M == 50 && c.B == 25 && c.I == 48 && c.Nmax == 2400;
}
// the stress shape (C5: K = 12, M = 50, B = 25): the forward one chain per CU
// at 512 threads, the backward at 768 or, with its full-N weights in global
// memory (GW, more chains than CUs), at 256
static bool shape_c5(const hyg_tg_consts& c) {
  static const bool off = tuning_env("HYG_NO_SHAPE") != nullptr;
  return !off && c.K == 12 && c.M == 50 && c.B == 25 && c.I == 168 && c.Nmax == 8400;
}
bool backward_global_w(const hyg_tg_consts& c) { return shape_c5(c); }
// the backward instantiation of a width keeps its full-N weights in global memory
static bool bwd_gw(const hyg_tg_consts& c, int NT) { return NT == 256 && backward_global_w(c); }
// HYG_DEBUG_PHASES=1 selects the phase-timer instantiations (256 and 512 threads).
static bool want_phases() {
  static const bool on = tuning_env("HYG_DEBUG_PHASES") != nullptr;
  return on;
}
template <int NT>
constexpr bool has_phases() { return NT == 256 || NT == 512 || NT == 768; }
template <int NT>
FwdFn fwd_kernel(const hyg_tg_consts& c) {
  if constexpr (has_phases<NT>()) {
    if (want_phases()) {
      if (shape_specialised(c)) return &tg_forward_kernel<NT, 6, 50, 25, true>;
      if constexpr (NT == 512)
        if (shape_c5(c)) return &tg_forward_kernel<NT, 12, 50, 25, true>;
      return &tg_forward_kernel<NT, 0, 0, 0, true>;
    }
  }
  if constexpr (NT == 256 || NT == 512 || NT == 768)
    if (shape_specialised(c)) return &tg_forward_kernel<NT, 6, 50, 25>;
  if constexpr (NT == 512 || NT == 768)
    if (shape_c5(c)) return &tg_forward_kernel<NT, 12, 50, 25>;
  return &tg_forward_kernel<NT>;
}
template <int NT>
BwdFn bwd_kernel(const hyg_tg_consts& c) {
  if constexpr (NT == 256)
    if (bwd_gw(c, NT)) return want_phases() ? &tg_backward_kernel<NT, 12, 50, 25, true, true>
                                            : &tg_backward_kernel<NT, 12, 50, 25, false, true>;
  if constexpr (has_phases<NT>()) {
    if (want_phases()) {
      if (shape_specialised(c)) return &tg_backward_kernel<NT, 6, 50, 25, true>;
      return &tg_backward_kernel<NT, 0, 0, 0, true>;
    }
  }
  if constexpr (NT == 256 || NT == 512 || NT == 768)
    if (shape_specialised(c)) return &tg_backward_kernel<NT, 6, 50, 25>;
  if constexpr (NT == 512 || NT == 768)
    if (shape_c5(c)) return &tg_backward_kernel<NT, 12, 50, 25>;
  return &tg_backward_kernel<NT>;
}

template <int NT>
static int launch_forward_nt(const ModelDev& md, const hyg_tg_consts& c, const ChainDev* chains_dev, int n_chains,
                            const double* E, uint8_t* ws, const hyg_tg_outputs& out, hipStream_t s, bool timed) {
  Lay lf = make_layout(c.K, c.M, c.B, c.Nmax, NT, false);
  if (lf.total > 160 * 1024) return HYG_EUNSUPPORTED;
  static const char* rv = tuning_env("HYG_TOPSET_R");  // tuning: 1 (A <= 64 per wave) or 2
  if (rv && (atoi(rv) == 1 || atoi(rv) == 2)) lf.topset_r = atoi(rv);
  if (c.M > NT) return HYG_EUNSUPPORTED;  // one ancestor per thread in the record read-ahead
  if (hipFuncSetAttribute((const void*)fwd_kernel<NT>(c), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lf.total) != hipSuccess)
    return HYG_EDEVICE;
  unsigned long long* dbg = nullptr;
  const bool want_dbg = has_phases<NT>() && want_phases();
  if (want_dbg) (void)hipMalloc((void**)&dbg, sizeof(unsigned long long) * kPh * n_chains);
  if (dbg) (void)hipMemsetAsync(dbg, 0, sizeof(unsigned long long) * kPh * n_chains, s);
  if (timed) ev_record(1, false, s);
  hipLaunchKernelGGL(fwd_kernel<NT>(c), dim3(n_chains), dim3(NT), lf.total, s, md, chains_dev, E, ws,
                     out.status, out.log_z, out.final_log_weights, lf, dbg);
  if (timed) ev_record(1, true, s);
  if (hipGetLastError() != hipSuccess) return HYG_EDEVICE;
  if (dbg) {
    std::vector<unsigned long long> h((size_t)kPh * n_chains);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), dbg, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost);
    (void)hipFree(dbg);
    unsigned long long tot[kPh] = {0};
    for (int i = 0; i < n_chains; ++i)
      for (int k = 0; k < kPh; ++k) tot[k] += h[(size_t)i * kPh + k];
    const double steps = (double)tot[kPh - 1];
    fprintf(stderr, "[hyg phases NT=%d] chains=%d steps=%.0f cycles/step:", NT, n_chains, steps);
    const char* nm[9] = {"top", "lse", "compact", "resample", "fallback", "gather", "wmax", "wgen", "wstore"};
    double sum = 0;
    for (int k = 0; k < 9; ++k) {
      fprintf(stderr, " %s=%.0f", nm[k], tot[k] / steps);
      sum += tot[k] / steps;
    }
    fprintf(stderr, " total=%.0f | keep_steps=%.0f mean_nsig=%.1f mean_n2=%.1f", sum, (double)tot[10],
            tot[9] / (steps - tot[10]), 0.0);
    fprintf(stderr, " | list=%.0f lse loop=%.0f cut sums=%.0f lse reduce=%.0f", tot[22] / steps, tot[23] / steps,
            tot[12] / steps, tot[11] / steps);
    const double opt = steps - tot[10];
    fprintf(stderr, " | topset: compact=%.0f mass=%.0f gatherA=%.0f sort=%.0f prefix=%.0f kloop_sys=%.0f",
            tot[24] / opt, tot[25] / opt, tot[26] / opt, tot[27] / opt, tot[28] / opt, tot[29] / opt);
    fprintf(stderr, " | kloop_sys split: c(a)=%.0f loop=%.0f systematic=%.0f (targets=%.0f search=%.0f tail=%.0f)",
            tot[30] / opt, tot[32] / opt, tot[31] / opt + tot[34] / opt + tot[33] / opt, tot[31] / opt, tot[34] / opt,
            tot[33] / opt);
    fprintf(stderr, " | per optimal step: topset=%.0f fallbacks=%.4f | per fallback: hist=%.0f bscan=%.0f scatter=%.0f "
            "bsort=%.0f scan=%.0f kloop=%.0f systematic=%.0f\n", tot[20] / opt, tot[21] / opt,
            tot[17] / (tot[21] + 1e-9), tot[18] / (tot[21] + 1e-9), tot[19] / (tot[21] + 1e-9),
            tot[13] / (tot[21] + 1e-9), tot[14] / (tot[21] + 1e-9), tot[15] / (tot[21] + 1e-9),
            tot[16] / (tot[21] + 1e-9));
  }
  return HYG_OK;
}

template <int NT>
static int launch_backward_nt(const ModelDev& md, const hyg_tg_consts& c, const ChainDev* chains_dev, int n_chains,
                              const double* E, uint8_t* ws, const hyg_tg_outputs& out, hipStream_t s, bool timed) {
  const Lay lb = make_layout(c.K, c.M, c.B, c.Nmax, NT, true, bwd_gw(c, NT));
  if (lb.total > 160 * 1024) return HYG_EUNSUPPORTED;
  if (c.M > NT) return HYG_EUNSUPPORTED;  // one ancestor per thread in the record read-ahead
  if (hipFuncSetAttribute((const void*)bwd_kernel<NT>(c), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lb.total) != hipSuccess)
    return HYG_EDEVICE;
  const bool want_dbg = has_phases<NT>() && want_phases();
  unsigned long long* dbgb = nullptr;
  if (want_dbg) (void)hipMalloc((void**)&dbgb, sizeof(unsigned long long) * kPh * n_chains);
  if (dbgb) (void)hipMemsetAsync(dbgb, 0, sizeof(unsigned long long) * kPh * n_chains, s);
  if (timed) ev_record(2, false, s);
  hipLaunchKernelGGL(bwd_kernel<NT>(c), dim3(n_chains), dim3(NT), lb.total, s, md, chains_dev, E,
                     (const uint8_t*)ws, (const int32_t*)out.status, out.merged, out.control, out.kase,
                     out.split_probs, out.regime_probs, out.status, lb, dbgb, ws);
  if (timed) ev_record(2, true, s);
  if (dbgb) {
    std::vector<unsigned long long> h((size_t)kPh * n_chains);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), dbgb, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost);
    (void)hipFree(dbgb);
    unsigned long long tot[kPh] = {0};
    for (int i = 0; i < n_chains; ++i)
      for (int k = 0; k < kPh; ++k) tot[k] += h[(size_t)i * kPh + k];
    const double steps = (double)tot[kPh - 1];
    const char* nm[7] = {"copy+gen", "issue", "groups", "list", "wave0", "general", "traj"};
    fprintf(stderr, "[hyg backward phases NT=%d] cycles/step:", NT);
    double sum = 0;
    for (int k = 0; k < 7; ++k) {
      fprintf(stderr, " %s=%.0f", nm[k], tot[k] / steps);
      sum += tot[k] / steps;
    }
    fprintf(stderr, " total(+tail)=%.0f | groups/step=%.2f finite logits/group=%.1f", sum, tot[10] / steps,
            (double)(tot[11] & 0xffffffffull) / (tot[10] > 0 ? (double)tot[10] : 1.0));
    fprintf(stderr, " | wave0 split: entries=%.0f max=%.0f exp=%.0f scan=%.0f total=%.0f draw=%.0f\n", tot[12] / steps,
            tot[13] / steps, tot[14] / steps, tot[15] / steps, tot[16] / steps, tot[4] / steps);
  }
  return hipGetLastError() == hipSuccess ? HYG_OK : HYG_EDEVICE;
}

// Forward workgroups one CU holds at the width a launch of n_chains uses
// (the occupancy query on the kernel instantiation and its dynamic LDS).
template <int NT>
static int fwd_resident_nt(const hyg_tg_consts& c) {
  const Lay lf = make_layout(c.K, c.M, c.B, c.Nmax, NT, false);
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)fwd_kernel<NT>(c), NT, lf.total) != hipSuccess)
    return -1;
  return nb;
}
int tg_resident_per_cu(const hyg_tg_consts& c, int n_chains) {
  switch (threads_per_chain(false, c, n_chains)) {
    case 64: return fwd_resident_nt<64>(c);
    case 128: return fwd_resident_nt<128>(c);
    case 256: return fwd_resident_nt<256>(c);
    case 768: return fwd_resident_nt<768>(c);
    default: return fwd_resident_nt<512>(c);
  }
}

static int launch_forward(int nt, const ModelDev& md, const hyg_tg_consts& c, const ChainDev* chains_dev,
                          int n_chains, const double* E, uint8_t* ws, const hyg_tg_outputs& out, hipStream_t s,
                          bool timed) {
  switch (nt) {
    case 64: return launch_forward_nt<64>(md, c, chains_dev, n_chains, E, ws, out, s, timed);
    case 128: return launch_forward_nt<128>(md, c, chains_dev, n_chains, E, ws, out, s, timed);
    case 256: return launch_forward_nt<256>(md, c, chains_dev, n_chains, E, ws, out, s, timed);
    case 768: return launch_forward_nt<768>(md, c, chains_dev, n_chains, E, ws, out, s, timed);
    default: return launch_forward_nt<512>(md, c, chains_dev, n_chains, E, ws, out, s, timed);
  }
}
static int launch_backward(int nt, const ModelDev& md, const hyg_tg_consts& c, const ChainDev* chains_dev,
                           int n_chains, const double* E, uint8_t* ws, const hyg_tg_outputs& out, hipStream_t s,
                           bool timed) {
  switch (nt) {
    case 64: return launch_backward_nt<64>(md, c, chains_dev, n_chains, E, ws, out, s, timed);
    case 128: return launch_backward_nt<128>(md, c, chains_dev, n_chains, E, ws, out, s, timed);
    case 256: return launch_backward_nt<256>(md, c, chains_dev, n_chains, E, ws, out, s, timed);
    case 768: return launch_backward_nt<768>(md, c, chains_dev, n_chains, E, ws, out, s, timed);
    default: return launch_backward_nt<512>(md, c, chains_dev, n_chains, E, ws, out, s, timed);
  }
}

// One wave that sleeps about 0.1 ms (32 x s_sleep 127, ~8 k cycles each). It
// sits between the head's forward and its backward on the second stream so that
// the tail's forward, released by the same event on the launch stream, takes its
// CUs before the backward's workgroups fill them (see launch_chains).
__global__ void tg_dispatch_guard_kernel() {
  for (int i = 0; i < 32; ++i) __builtin_amdgcn_s_sleep(127);
}

namespace {
// The per-chain outputs of chains [c0, ...) of a launch; the per-site outputs
// are addressed through each chain's out_begin and need no offset.
hyg_tg_outputs outputs_from(const hyg_tg_outputs& o, const hyg_tg_consts& c, int c0) {
  hyg_tg_outputs r = o;
  r.status = o.status + c0;
  r.log_z = o.log_z + c0;
  if (o.final_log_weights) r.final_log_weights = o.final_log_weights + (size_t)c0 * c.Nmax;
  return r;
}
// The second stream and two events of a device for the tail overlap
// (created on first use, kept for the process).
struct TailAux {
  std::mutex mu;  // one split launch enqueued at a time (the events are shared)
  hipStream_t s = nullptr;
  hipEvent_t head_done = nullptr, bwd_done = nullptr;
  bool ok = false, tried = false;
};
TailAux* tail_aux() {
  static TailAux aux[32];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 32) return nullptr;
  TailAux& a = aux[dev];
  static std::mutex init_mu;
  std::lock_guard<std::mutex> lock(init_mu);
  if (!a.tried) {
    a.tried = true;
    a.ok = hipStreamCreateWithFlags(&a.s, hipStreamNonBlocking) == hipSuccess &&
           hipEventCreateWithFlags(&a.head_done, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&a.bwd_done, hipEventDisableTiming) == hipSuccess;
  }
  return a.ok ? &a : nullptr;
}
bool g_tail_overlap = true;  // hyg_tg_set_tail_overlap
}  // namespace

void tg_set_tail_overlap(bool on) { g_tail_overlap = on; }

// The whole launch: forward of every chain, then the backward of every chain.
//
// Tail overlap. When the forward's LDS holds one chain per CU (the C5 shape)
// and the chains fill more than one round of CUs with a partial last round, the
// last round leaves most CUs idle for a full chain's latency (C5: 1 164 chains
// = four rounds of 256 and a fifth of 140, 52 of them full length). The
// launch is then split: the forward of the full rounds (the head, the first
// chains in launch order) and of the rest (the tail) run back to back on the
// launch stream, and the head's backward runs on a second stream as soon as
// the head's forward is done, on the CUs the tail's forward leaves free; the
// tail's backward follows its forward. Each chain's forward still precedes its
// backward, no chain's buffers are shared, and the widths are those of the
// whole launch, so the outputs are those of the unsplit launch (GPU test).
int launch_chains(const ModelDev& md, const hyg_tg_consts& c, const ChainDev* chains_dev, int n_chains,
                  const double* E, uint8_t* ws, const hyg_tg_outputs& out, void* stream) {
  if (n_chains <= 0) return HYG_OK;
  hipStream_t s = (hipStream_t)stream;
  const int ntf = threads_per_chain(false, c, n_chains), ntb = threads_per_chain(true, c, n_chains);
  int head = n_chains;
  TailAux* aux = nullptr;
  if (g_tail_overlap && n_chains > device_cus() && n_chains % device_cus() != 0 &&
      tg_resident_per_cu(c, n_chains) == 1 && (aux = tail_aux()) != nullptr)
    head = n_chains - n_chains % device_cus();
  if (head == n_chains) {
    const int rc = launch_forward(ntf, md, c, chains_dev, n_chains, E, ws, out, s, true);
    if (rc != HYG_OK) return rc;
    return launch_backward(ntb, md, c, chains_dev, n_chains, E, ws, out, s, true);
  }
  const int tail = n_chains - head;
  const hyg_tg_outputs out_t = outputs_from(out, c, head);
  std::lock_guard<std::mutex> lock(aux->mu);
  ev_record(1, false, s);
  int rc = launch_forward(ntf, md, c, chains_dev, head, E, ws, out, s, false);
  if (rc != HYG_OK) return rc;
  if (hipEventRecord(aux->head_done, s) != hipSuccess) return HYG_EDEVICE;
  rc = launch_forward(ntf, md, c, chains_dev + head, tail, E, ws, out_t, s, false);
  if (rc != HYG_OK) return rc;
  ev_record(1, true, s);
  // From here the second stream holds work: every return path below makes the
  // launch stream wait for it, so the call's stream covers the whole launch
  // whatever fails.
  auto join = [&](int code) {
    const bool ok = hipEventRecord(aux->bwd_done, aux->s) == hipSuccess &&
                    hipStreamWaitEvent(s, aux->bwd_done, 0) == hipSuccess;
    if (code == HYG_OK && !ok) return (int)HYG_EDEVICE;
    if (!ok) (void)hipStreamSynchronize(aux->s);  // the events failed: drain the second stream instead
    return code;
  };
  if (hipStreamWaitEvent(aux->s, aux->head_done, 0) != hipSuccess) return join(HYG_EDEVICE);
  // The guard kernel is a scheduling heuristic, not a dependency: it only makes
  // the tail's forward (released by head_done on the launch stream) likely to
  // take its CUs before the head's backward fills them. The outputs do not
  // depend on which dispatch wins.
  hipLaunchKernelGGL(tg_dispatch_guard_kernel, dim3(1), dim3(64), 0, aux->s);
  ev_record(2, false, aux->s);
  rc = launch_backward(ntb, md, c, chains_dev, head, E, ws, out, aux->s, false);
  if (rc != HYG_OK) return join(rc);
  rc = launch_backward(ntb, md, c, chains_dev + head, tail, E, ws, out_t, s, false);
  rc = join(rc);
  if (rc != HYG_OK) return rc;
  ev_record(2, true, s);
  return hipGetLastError() == hipSuccess ? HYG_OK : HYG_EDEVICE;
}
}  // namespace hyg
