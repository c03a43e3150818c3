// sg_kernels.hip -- CDNA4 (gfx950) kernels of the single-group path.
//
//   sg_emission_kernel  per-site Beta-Binomial table E[t][r] (HBM streaming)
//   sg_chain_kernel     SMC for the change-point model + online marginal
//                       smoothing, one 256-thread workgroup per chain, one
//                       particle per thread (N_max <= 256), persistent over T.
//                       Template flag PE: with online parameter estimation
//                       (include/hyg_sg_pe.h): the score
//                       recursion phi, an ADAM / gradient step every `every`
//                       steps and the rebuild of P, omega and the hazard rows
//                       from the new theta, all inside the persistent workgroup.
//
// Same computations as oracle/sg_oracle.c (the arithmetic contract of
// include/hyg_arith.h: exact fixed-point sums, hyg_exp / hyg_log, Philox), so
// the smoothed regime probabilities are bit-identical to the oracle's.
// Reference: src/single_group/src/cpp/algorithms/Smc.h:114-579,
// misc/resample.h:85-117,289-409, algorithms/OnlineMarginalSmoothing.h:52-255,
// algorithms/OnlineCombinedInference.h:48-118, singleGroup.h:556-627.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/hyg_arith.h"
#include "hyg_dev.h"
#include "sg_common.h"

namespace hyg {

__device__ __forceinline__ uint32_t sg_pack(int d, int r) { return (uint32_t)d | ((uint32_t)r << 24); }
__device__ __forceinline__ int sg_d(uint32_t s) { return (int)(s & 0xffffffu); }
__device__ __forceinline__ int sg_r(uint32_t s) { return (int)(s >> 24); }

// Model::evaluateLogTransitionDensity (singleGroup.h:569-608) split per
// previous particle (d, r): the density of a fresh particle (1, q) is
// base + log P[r][q] with base = log rho(d, r) (0 after the hazard's exit, -inf
// for d < u), and of the continuing particle (d + 1, r) it is cont =
// log(1 - rho(d, r)). Both equal the oracle's sg_trans bit for bit (the
// diagonal log P[r][r] = -inf covers q == r).
// the hazard row and exit flag of state s (sg_trans_parts in two halves: the
// loads, and the parts formed from them where they are used)
__device__ __forceinline__ void sg_trans_load(const SgModelDev& md, uint32_t s, double2& h, uint8_t& ex) {
  const int d = sg_d(s), r = sg_r(s);
  int di = d - 1;
  if (di >= md.dcap) di = md.dcap - 1;
  h = *(const double2*)(md.hz + ((size_t)r * md.dcap + di) * 2);
  ex = md.ex[(size_t)r * md.dcap + di];
}
__device__ __forceinline__ void sg_trans_form(int u, uint32_t s, const double2& h, uint8_t ex, double& base,
                                              double& cont) {
  base = (sg_d(s) >= u) ? (ex ? 0.0 : h.x) : HYG_NINF;
  cont = h.y;
}
__device__ __forceinline__ void sg_trans_parts(const SgModelDev& md, int u, uint32_t s, double& base,
                                               double& cont) {
  double2 h;
  uint8_t ex;
  sg_trans_load(md, s, h, ex);
  sg_trans_form(u, s, h, ex, base, cont);
}

// ceil(T * R) for a double T in [0, 1] and R < 2^127 (oracle/sg_oracle.c:ceil_mul_f64)
__device__ __forceinline__ hyg_u128 sg_ceil_mul_f64(double T, hyg_u128 R);
// #{j in [0, L) : ceil(T_j R) <= v} for the systematic targets T_j = ((double)j
// + uu) / (double)L (non-decreasing in j, as systematicBase forms them,
// resample.h:85-117). The estimate jf = (v / R) L - uu lies within 2^-40 of the
// crossing (the conversions and the division round at 2^-53, T_j at 2^-45 in
// j units), so every j <= floor(jf) - 2 counts and no j >= floor(jf) + 2 does;
// the three between are compared in f64 outside a 2^-40 relative guard band and
// exactly (ceil(T_j R) <= v in integers) inside it.
__device__ __forceinline__ int sg_sys_count(const hyg_u128& v, const hyg_u128& R, double invR, int L, double uu) {
  const double y = hyg_u128_to_f64(v, 100) * invR;
  double jf = y * (double)L - uu;
  jf = jf < -2.0 ? -2.0 : (jf > (double)L + 2.0 ? (double)L + 2.0 : jf);
  const int j0 = (int)floor(jf);
  int c = j0 - 1;
  c = c < 0 ? 0 : (c > L ? L : c);
  const double ylo = y * (1.0 - 0x1p-40), yhi = y * (1.0 + 0x1p-40);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int j = j0 - 1 + k;
    if (j >= 0 && j < L) {
      const double T = ((double)j + uu) / (double)L;
      bool le = T < ylo;
      if (!le && !(T > yhi)) le = !hyg_u128_lt(v, sg_ceil_mul_f64(T, R));  // exact
      c += le ? 1 : 0;
    }
  }
  return c;
}
__device__ __forceinline__ hyg_u128 sg_ceil_mul_f64(double T, hyg_u128 R) {
  hyg_u128 z = hyg_u128_zero();
  if (!(T > 0.0)) return z;
  const uint64_t b = hyg_f64_bits(T);
  const int E = (int)((b >> 52) & 0x7ff);
  const uint64_t m = (E == 0) ? (b & 0x000fffffffffffffull) : ((b & 0x000fffffffffffffull) | 0x0010000000000000ull);
  const int s = (E == 0) ? 1074 : 1075 - E;
  const uint64_t l0 = m * R.lo, h0 = hyg_mulhi64(m, R.lo);
  const uint64_t l1 = m * R.hi, h1 = hyg_mulhi64(m, R.hi);
  uint64_t w0 = l0, w1 = h0 + l1, w2 = h1 + (w1 < h0 ? 1u : 0u);
  if (s >= 192) { hyg_u128 o; o.lo = (w0 | w1 | w2) ? 1u : 0u; o.hi = 0; return o; }
  uint64_t b0 = 0, b1 = 0, b2 = 0;
  if (s < 64) b0 = (1ull << s) - 1;
  else if (s < 128) { b0 = ~0ull; b1 = (s == 64) ? 0 : (1ull << (s - 64)) - 1; }
  else { b0 = ~0ull; b1 = ~0ull; b2 = (s == 128) ? 0 : (1ull << (s - 128)) - 1; }
  const uint64_t q0 = w0 + b0, c0 = q0 < w0;
  const uint64_t t1 = w1 + b1, c1a = t1 < w1;
  const uint64_t q1 = t1 + c0, c1b = q1 < t1;
  const uint64_t q2 = w2 + b2 + c1a + c1b;
  hyg_u128 r;
  if (s < 64) { r.lo = (q0 >> s) | (s ? q1 << (64 - s) : 0); r.hi = (q1 >> s) | (s ? q2 << (64 - s) : 0); }
  else if (s == 64) { r.lo = q1; r.hi = q2; }
  else if (s < 128) { r.lo = (q1 >> (s - 64)) | (q2 << (128 - s)); r.hi = q2 >> (s - 64); }
  else if (s == 128) { r.lo = q2; r.hi = 0; }
  else { r.lo = q2 >> (s - 128); r.hi = 0; }
  return r;
}



// ------------------------------------------------------------ LDS layout
constexpr int kSgChunk = 32;  // pending entries finalised per smoothing round
constexpr int kSgPh = 24;     // phase-timer slots (HYG_SG_PHASES builds; the last holds the latest stamp)

struct SgShared {
  int npend, nfree, cur, status;
  int Kk, pad0;
  unsigned int lmask;  // free psi slots resident in LDS
  int pad1;
  double logC;
  // the systematic uniforms of steps 64 j .. 64 j + 63, drawn one block ahead
  // by an idle wave, one step per lane (512 threads)
  double uring[64];
  // keep-top steps: each key wave's first and last full log-weight key and index
  // after the packed sort, and whether an in-wave pair is out of order
  unsigned long long kfirst[4], klast[4];
  int ifirst[4], ilast[4], kbad[4];
  unsigned long long ph[kSgPh];  // phase timers (diagnostic runs only)
};

struct SgLay {
  size_t st, lw, w, base, cont;  // [2][NT]: current / previous particle sets, alternating per step
  size_t anc, lwres, logq, sidx, cum, xk, xi, BK, logP, red, scr, meanb, okb, logm, logQ, psil, sh, total;
  size_t pm, gfr, gct, pei, rpu;  // parameter estimation: model, per-particle gradient entries [2][NT], ints,
                                  // regime if d >= u else -1 [2][NT] (int8)
  int nl;  // psi slots resident in LDS (slot ids 0 .. nl-1; the rest live in the workspace)
};

__host__ __device__ inline size_t sg_align(size_t x) { return (x + 15) / 16 * 16; }

// The SMC workgroup's reduction area: block reductions use its first 32 B per
// wave; the weights' arrays (continuing-particle partials, A_r, E_r limbs,
// G[r][q], m_q) live behind them (sg_chain_kernel)
__host__ __device__ inline size_t sg_red_w(int NW) { return 32 * (size_t)NW; }
__host__ __device__ inline size_t sg_red_bytes(int K, int NW) {
  const size_t a = 24 * (size_t)NW * K + 16 * NW + 64;
  const size_t b = sg_red_w(NW) + 12 * (size_t)NW + 8 + 8 * (size_t)K + 24 * (size_t)K + 8 * (size_t)K * K + 8 * K;
  return a > b ? a : b;
}

// NB = threads of the workgroup (particles live on threads < 256, the other
// waves join the block reductions, sorts (on dummy keys) and the smoothing tasks)
__host__ __device__ inline int sg_block_threads(int K) { return K <= 8 ? 512 : 256; }

__host__ __device__ inline SgLay sg_layout(int K, int cap, bool pe) {
  SgLay l{};
  const int NT = kSgThreads, NB = sg_block_threads(K), NW = NB / 64;
  size_t o = 0;
  l.st = o; o = sg_align(o + 4 * 2 * NT);
  l.lw = o; o = sg_align(o + 8 * 2 * NT);
  l.w = o; o = sg_align(o + 8 * 2 * NT);
  l.base = o; o = sg_align(o + 8 * 2 * NT);
  l.cont = o; o = sg_align(o + 8 * 2 * NT);
  l.anc = o; o = sg_align(o + 4 * NT);
  l.lwres = o; o = sg_align(o + 8 * NT);
  l.logq = o; o = sg_align(o + 8 * NT);
  l.sidx = o; o = sg_align(o + 4 * NT);
  l.cum = o; o = sg_align(o + 16 * (NB + 1));
  l.xk = o; o = sg_align(o + 8 * 2 * NB);
  l.xi = o; o = sg_align(o + 4 * 2 * NB);
  l.BK = o; o = sg_align(o + 8 * (size_t)K * NT);
  l.logP = o; o = sg_align(o + 8 * (size_t)K * K);
  l.red = o; o = sg_align(o + sg_red_bytes(K, NW));
  l.scr = o; o = sg_align(o + 8 * (size_t)NW * NT);
  l.meanb = o; o = sg_align(o + 8 * (size_t)kSgChunk * K);
  l.okb = o; o = sg_align(o + (size_t)kSgChunk * K);
  l.logm = o; o = sg_align(o + 8 * (NT + 1));
  l.logQ = o; o = sg_align(o + 8 * (NT + 1));
  l.sh = o; o = sg_align(o + sizeof(SgShared));
  if (pe) {
    l.pm = o; o = sg_align(o + sizeof(hyg_sgpe_model));
    l.gfr = o; o = sg_align(o + 8 * 2 * NT);
    l.gct = o; o = sg_align(o + 8 * 2 * NT);
    l.pei = o; o = sg_align(o + 4 * (2 * HYG_KMAX + 8));
    l.rpu = o; o = sg_align(o + 2 * NT);
  }
  (void)cap;
  l.nl = 0;  // the psi slots live in the smoothing workgroup (SgCLay)
  l.psil = o;
  l.total = o;
  return l;
}

// LDS of the smoothing workgroup: the step record (ancestors, regimes, weights,
// backward kernels), per-wave scratch, the finalisation buffers, and as many
// psi slots [K][256] f64 as fit (up to 32; the rest live in the workspace).
struct SgCLay {
  size_t anc, rgn, w, BK, scr, meanb, okb, red, sh, psil, total;
  int nl;
};
struct SgCShared {
  int npend, nfree, cur, status;
  int avail, abort_code, pad0, pad1;
  unsigned int lmask;
  int pad2;
};
constexpr size_t kSgLdsBudget = 160 * 1024 - 2048;  // headroom below the 160 KiB of a CU (launches at 163808 B fail)
__host__ __device__ inline SgCLay sg_clayout(int K, int cap) {
  SgCLay l{};
  const int NT = kSgThreads, NB = sg_block_threads(K), NW = NB / 64;
  size_t o = 0;
  l.anc = o; o = sg_align(o + 4 * NT);
  l.rgn = o; o = sg_align(o + NT);
  l.w = o; o = sg_align(o + 8 * NT);
  l.BK = o; o = sg_align(o + 8 * (size_t)K * NT);
  l.scr = o; o = sg_align(o + 8 * (size_t)NW * NT);
  l.meanb = o; o = sg_align(o + 8 * (size_t)kSgChunk * K);
  l.okb = o; o = sg_align(o + (size_t)kSgChunk * K);
  l.red = o; o = sg_align(o + 24 * (size_t)NW * K + 16 * NW + 64);
  l.sh = o; o = sg_align(o + sizeof(SgCShared));
  const size_t slot = 8 * (size_t)K * NT;
  int nl = o < kSgLdsBudget ? (int)((kSgLdsBudget - o) / slot) : 0;
  if (nl > 32) nl = 32;
  if (nl > cap) nl = cap;
  l.nl = nl;
  l.psil = o; o = sg_align(o + slot * nl);
  l.total = o;
  return l;
}

// one launch's dynamic LDS: the larger of the two workgroup roles
size_t sg_lds_bytes(const hyg_sg_consts& c, int psi_cap, bool pe) {
  const size_t a = sg_layout(c.K, psi_cap, pe).total, b = sg_clayout(c.K, psi_cap).total;
  return a > b ? a : b;
}

// ------------------------------------------------ inter-workgroup hand-off
// Ring of step records from the SMC workgroup to the smoothing workgroup
// (cdna_hip_programming.md Guideline 16, recipe R1): every payload word is
// stored write-through (agent-scope relaxed atomic store = global_store sc1),
// each storing wave drains its stores (s_waitcnt vmcnt(0)) before a workgroup
// barrier, then ONE lane stores the head counter; the consumer polls head
// relaxed, ONE agent-scope acquire, then plain loads. Control words
// (ctl[0] head = records published, ctl[1] tail = records consumed, ctl[2]
// abort code) are zeroed by the launch function.
typedef __attribute__((address_space(1))) unsigned int sg_gu32;
typedef __attribute__((address_space(1))) unsigned long long sg_gu64;
constexpr unsigned kSgTailAbort = 0x7fffffffu;  // the smoothing workgroup gave up: never wait for ring space
constexpr unsigned kSgSpinMax = 1u << 24;       // bounded spins (~25 s of polling): then HYG_EDEVICE
// the first record may wait for the SMC workgroup to become resident, i.e. for
// another chain of a crowded GPU to finish (a chromosome-1 chain: ~35 s)
constexpr unsigned kSgSpinFirst = 1u << 26;
// ctl word 3 of a launch's first chain: the launch's dispatch-ticket counter
constexpr size_t kSgTicketOffset = 12;
__device__ __forceinline__ void sg_st8(uint8_t* p, uint64_t v) {
  __hip_atomic_store((sg_gu64*)p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sg_st4(uint8_t* p, unsigned v) {
  __hip_atomic_store((sg_gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned sg_ld4(uint8_t* p) {
  return __hip_atomic_load((sg_gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sg_drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ------------------------------------------------------------- emission
// E[t][r] = sum_s log BB(y_ts | n_ts, alpha_r, beta_r) in the oracle's term
// order (oracle_sg_emission); y > n gives -inf as the reference's density,
// a count beyond the model's tables poisons the row with NaN.
__global__ void __launch_bounds__(256)
sg_emission_kernel(const double* __restrict__ lf, const double* __restrict__ lg, const double* __restrict__ cst,
                   int L, int K, const uint16_t* __restrict__ meth, const uint16_t* __restrict__ tot, int S,
                   int64_t T, double* __restrict__ E) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < T; t += (int64_t)gridDim.x * blockDim.x) {
    double e[HYG_KMAX];
#pragma unroll
    for (int r = 0; r < HYG_KMAX; ++r) e[r] = 0.0;
    double poison = 0.0;
    for (int s = 0; s < S; ++s) {
      const int n = tot[t * S + s], y = meth[t * S + s];
      if (n >= L) { poison = HYG_NAN; break; }
      if (y > n) { poison = HYG_NINF; break; }
      const double base = (lf[n] - lf[y]) - lf[n - y];
#pragma unroll
      for (int r = 0; r < HYG_KMAX; ++r) {
        if (r < K) {
          double term = base + lg[(size_t)(r * 3 + 0) * L + y];
          term = term + lg[(size_t)(r * 3 + 1) * L + (n - y)];
          term = term - lg[(size_t)(r * 3 + 2) * L + n];
          term = term + cst[r];
          e[r] = e[r] + term;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < HYG_KMAX; ++r)
      if (r < K) E[t * K + r] = (poison != 0.0) ? poison : e[r];
  }
}


// ------------------------------------------- parameter estimation helpers
// The chain's region of the workspace (sg_pe_region_bytes).
struct SgPeChain {
  double* phi;  // [2][NT][K^2] score recursion, particle-major
  double *th, *am, *av, *gp, *gc;  // [K (K + 1)] (theta rows are c.dim wide)
  hyg_sgpe_row* rows;            // [K][rcap]
  double *h, *g, *gk, *Hm1, *gm1; // rebuild scratch [K][rcap]
  uint8_t* ex;                   // [K][rcap]
  int rcap;
};
__device__ __forceinline__ SgPeChain sg_pe_chain(uint8_t* ws, const SgChainDev& ch, int K) {
  SgPeChain c;
  const size_t dim = (size_t)K * K, dth = (size_t)K * (K + 1), kr = (size_t)K * ch.rcap;
  c.phi = (double*)(ws + ch.pe_offset);
  c.th = c.phi + 2 * (size_t)kSgThreads * dim;
  c.am = c.th + dth;
  c.av = c.am + dth;
  c.gp = c.av + dth;
  c.gc = c.gp + dth;
  c.rows = (hyg_sgpe_row*)(c.gc + dth);
  c.h = (double*)(c.rows + kr);
  c.g = c.h + kr;
  c.gk = c.g + kr;
  c.Hm1 = c.gk + kr;
  c.gm1 = c.Hm1 + kr;
  c.ex = (uint8_t*)(c.gm1 + kr);
  c.rcap = ch.rcap;
  return c;
}

// setUnknownParameters (singleGroup.h:197-270) for the chain's current theta:
// P / log P / omega into LDS, then the hazard rows 0 .. L-1 of every regime
// (include/hyg_sg_pe.h): the NegBin terms in parallel over (r, d), the
// sequential bigH / gradBigH recursion one lane per regime, the finished rows
// in parallel. Called by every thread; ends on a barrier.
template <int NB>
__device__ void sg_pe_rebuild(const SgPeDev& pe, const hyg_sg_consts& c, const SgPeChain& pc, hyg_sgpe_model* pm,
                              int* Lr, int* exr, int K, int u, int L) {
  const int tid = threadIdx.x;
  if (L > pc.rcap) L = pc.rcap;
  if (tid < K) hyg_sgpe_set_regime(pc.th, K, tid, pm);
  __syncthreads();
  const bool kest = pe.dgk != nullptr;  // kappa estimated: the omega coordinate takes d log rho / d theta_kappa
  for (int i = tid; i < K * L; i += NB) {
    const int r = i / L, d = i - r * L;
    double h, g, gk;
    hyg_sgpe_hazard_point(pm, r, d, u, c.kappa[r], pe.lgk + (size_t)r * pe.lgk_stride,
                          kest ? pe.dgk + (size_t)r * pe.lgk_stride : nullptr, &h, &g, &gk);
    const size_t o = (size_t)r * pc.rcap + d;
    pc.h[o] = h;
    pc.g[o] = g;
    if (kest) pc.gk[o] = gk;
  }
  __syncthreads();
  if (tid < K) {
    const size_t o = (size_t)tid * pc.rcap;
    const int l =
        hyg_sgpe_hazard_scan(pc.h + o, pc.g + o, kest ? pc.gk + o : nullptr, u, L, pc.Hm1 + o, pc.gm1 + o, pc.ex + o);
    Lr[tid] = l;
    exr[tid] = pc.ex[o + l - 1];
  }
  __syncthreads();
  const double* gsel = kest ? pc.gk : pc.g;
  for (int i = tid; i < K * L; i += NB) {
    const int r = i / L, d = i - r * L;
    if (d < Lr[r]) {
      const size_t o = (size_t)r * pc.rcap + d;
      pc.rows[o] = hyg_sgpe_hazard_row(pc.h[o], gsel[o], pc.Hm1[o], pc.gm1[o], pc.ex[o], d, u);
    }
  }
  __syncthreads();
}

// sg_trans_parts of the estimation path plus the particle's gradient entries:
// gomg = d log rho / d theta_omega (fresh particles from it), gcont = the
// continuation's entry. `over` is set when a sojourn outruns the rows of a
// regime whose hazard has not exited.
__device__ __forceinline__ void sg_pe_parts(const SgPeChain& pc, const int* Lr, const int* exr, int u, uint32_t s,
                                            double& base, double& cont, double& gomg, double& gcont, int& over) {
  const int d = sg_d(s), r = sg_r(s);
  int di = d - 1;
  if (di >= Lr[r]) {
    if (!exr[r]) over = 1;
    di = Lr[r] - 1;
  }
  const hyg_sgpe_row w = pc.rows[(size_t)r * pc.rcap + di];
  base = (d >= u) ? w.base : HYG_NINF;
  cont = w.cont;
  gomg = w.gomg;
  gcont = w.gcont;
}

// --------------------------------------------------------- chain kernel
// order key of a double: ascending key == ascending value (-0.0 == +0.0)
__device__ __forceinline__ uint64_t sg_okey(double x) {
  uint64_t b = u_of(x);
  if (b == 0x8000000000000000ull) b = 0;
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double sg_okey_value(uint64_t k) {
  return d_of((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k);
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const int lo = __shfl_xor((int)(uint32_t)v, m), hi = __shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
// Bitonic sort of the NT (key, idx) pairs held one per thread into descending
// key, ties by ascending idx (the order of arma::sort_index "descend" /
// oracle sort_desc); afterwards thread q holds the element of sorted position
// q. Distances < 64 exchange within the wave (xshfl: DPP, row rotations,
// permlane swaps), 64 and 128 through LDS
// (xk / xi, two buffers so consecutive cross-wave steps need one barrier each).
template <int NB>
__device__ __forceinline__ void sg_bitonic(uint64_t& key, int& idx, uint64_t* xk, int* xi) {
  constexpr int NT = kSgThreads;  // the keys sorted: threads [0, 256)
  const int tid = threadIdx.x;
  const bool real = (NB == NT) || tid < NT;  // wave-uniform: waves >= 4 hold no keys and only keep the barriers
  int buf = 0;
#pragma unroll
  for (int k = 2; k <= NT; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      uint64_t pk = key;
      int pi = idx;
      if (j >= 64) {
        if (real) {
          xk[buf * NB + tid] = key;
          xi[buf * NB + tid] = idx;
        }
        lds_barrier();
        if (real) {
          pk = xk[buf * NB + (tid ^ j)];
          pi = xi[buf * NB + (tid ^ j)];
        }
        buf ^= 1;
      } else if (real) {  // within a wave: DPP / permlane swaps (no LDS round trip), j constant after unrolling
        switch (j) {
          case 1: pk = xshfl64<1>(key); pi = (int)xshfl32<1>((uint32_t)idx); break;
          case 2: pk = xshfl64<2>(key); pi = (int)xshfl32<2>((uint32_t)idx); break;
          case 4: pk = xshfl64<4>(key); pi = (int)xshfl32<4>((uint32_t)idx); break;
          case 8: pk = xshfl64<8>(key); pi = (int)xshfl32<8>((uint32_t)idx); break;
          case 16: pk = xshfl64<16>(key); pi = (int)xshfl32<16>((uint32_t)idx); break;
          default: pk = xshfl64<32>(key); pi = (int)xshfl32<32>((uint32_t)idx); break;
        }
      }
      if (j < 64) {
        if (real) {
          // (lower == up) is a constant lane pattern (k >= 64: a wave bit), so
          // the exchange is the compare's lane mask xnor that pattern
          const uint64_t lower = lanes_bit_clear(j);
          const uint64_t same = (k < 64) ? ~(lower ^ lanes_bit_clear(k < 64 ? k : 1))
                                         : (((wave_id() * 64) & k) == 0 ? lower : ~lower);
          const uint64_t pf = wave_ballot(pk > key || (pk == key && pi < idx));
          const uint64_t take = ~(same ^ pf);
          key = lane_select64(take, key, pk);
          idx = (int)lane_select32(take, (uint32_t)idx, (uint32_t)pi);
        }
      } else if (real) {
        const bool up = (tid & k) == 0, lower = (tid & j) == 0;
        const bool pfirst = pk > key || (pk == key && pi < idx);
        if ((lower == up) ? pfirst : !pfirst) {
          key = pk;
          idx = pi;
        }
      }
    }
  }
}

// The order of sg_bitonic on one 64-bit word per thread (the log-weight key's
// top 56 bits with 255 - idx in the low byte, so ties of the word order by
// ascending idx; descending words are the pair order except inside a run of
// keys that agree on the top 56 bits and differ below them: the caller checks
// the order it uses, sg_chain_kernel), by ranks: each key wave sorts its 64
// words descending (the network's stages k <= 64, every wave in the final
// direction), the four runs meet in LDS, and each word's position is its
// rank, the sum over the runs of
// the words above it (its lane in its own run; a 7-probe binary search in
// the others, the four searches interleaved). The words are distinct (255 -
// idx in the low byte), so the ranks are a permutation and the result is the
// network's. Two barriers and 21 in-wave stages in place of the three
// cross-wave stages and 33 in-wave stages of the full network (round 6: the
// sort 4.4 k -> 3.6 k cycles per chr1 step, profiles/r06r_phases_sg_c2.log).
template <int NB>
__device__ __forceinline__ void sg_rank_sort_packed(uint64_t& key, uint64_t* xk) {
  constexpr int NT = kSgThreads, NR = NT / 64;
  const int tid = threadIdx.x;
  const bool real = (NB == NT) || tid < NT;
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (real) {
        uint64_t pk;
        switch (j) {
          case 1: pk = xshfl64<1>(key); break;
          case 2: pk = xshfl64<2>(key); break;
          case 4: pk = xshfl64<4>(key); break;
          case 8: pk = xshfl64<8>(key); break;
          case 16: pk = xshfl64<16>(key); break;
          default: pk = xshfl64<32>(key); break;
        }
        const uint64_t lower = lanes_bit_clear(j);
        const uint64_t same = (k < 64) ? ~(lower ^ lanes_bit_clear(k < 64 ? k : 1)) : lower;
        const uint64_t take = ~(same ^ wave_ballot(pk > key));
        key = lane_select64(take, key, pk);
      }
    }
  }
  if (real) xk[tid] = key;
  lds_barrier();
  if (real) {
    int pos[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) pos[r] = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1) {
#pragma unroll
      for (int r = 0; r < NR; ++r) pos[r] += (xk[64 * r + pos[r] + step - 1] > key) ? step : 0;
    }
    int rank = 0;
#pragma unroll
    for (int r = 0; r < NR; ++r) rank += pos[r] + ((xk[64 * r + pos[r]] > key) ? 1 : 0);
    xk[NB + rank] = key;
  }
  lds_barrier();
  if (real) key = xk[NB + tid];
}
__device__ __forceinline__ uint64_t sg_pack_key(uint64_t okey, int idx, uint64_t keep) {
  return (okey & keep) | (uint64_t)(255 - idx);
}
__device__ __forceinline__ int sg_packed_idx(uint64_t key) { return 255 - (int)(key & 0xffull); }
// the value of the lane above (DPP wave_shl:1; lane 63 gets 0)
__device__ __forceinline__ uint32_t sg_lane_next(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);
}

// One workgroup per chain, thread n = particle n (N_max <= 256). Per step the
// critical path is a few dozen barriers: sorts in registers, the K / log c
// fixed point in one wave, batched reductions for the K fresh-particle rows
// and backward kernels, and the smoothing split into (pending time, regime)
// tasks over all waves with the psi rows resident in LDS (up to 32 slots,
// the rest in the chain's workspace region).
template <int KT, int NB>
__device__ __forceinline__ void sg_smoother(const SgModelDev md, const SgChainDev ch, int chain,
                                            uint8_t* __restrict__ ws, int cap, double* __restrict__ probs,
                                            int32_t* __restrict__ status_out, const SgCLay lay);

template <int KT, int NB, bool PE, bool PHS = false>  // PHS: the phase-timer build (HYG_SG_PHASES)
__global__ void __launch_bounds__(NB)
sg_chain_kernel(SgModelDev md, const SgChainDev* __restrict__ chains, int n_chains, const double* __restrict__ E,
                uint8_t* __restrict__ ws, int cap, double* __restrict__ probs, int32_t* __restrict__ status_out,
                SgLay lay, SgCLay clay, unsigned long long* __restrict__ dbg_arg, SgPeDev pe) {
  // a constant null pointer outside the timer build: every timer test folds away
  unsigned long long* __restrict__ const dbg = PHS ? dbg_arg : nullptr;
  // Roles by dispatch ticket, not by block index: the k-th workgroup to start
  // takes ticket k; ticket 2c is the online marginal smoothing of chain c,
  // ticket 2c + 1 its SMC, fed through the ring. A chain's two workgroups wait
  // for each other, so both must be resident at once. With tickets taken in
  // the order workgroups actually become resident, at most one resident
  // workgroup (a smoothing one, which only polls) waits for a partner that is
  // not resident yet, and every other resident pair runs to completion and
  // frees its CUs: the launch finishes whenever two workgroups fit on the GPU,
  // whatever else shares it (other streams, other processes, CU masks).
  __shared__ int role_ticket;
  if (threadIdx.x == 0)
    role_ticket = (int)__hip_atomic_fetch_add((sg_gu32*)(ws + chains[0].ctl_offset + kSgTicketOffset), 1u,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int chain = role_ticket >> 1;
  if ((role_ticket & 1) == 0) {
    sg_smoother<KT, NB>(md, chains[chain], chain, ws, cap, probs, status_out, clay);
    return;
  }
  constexpr int NT = kSgThreads, NW = NB / 64, K = KT;  // NT: particle slots, NB: threads
  const hyg_sg_consts& c = *md.consts;
  const int Nmax = c.Nmax, u = c.u, tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  const SgChainDev ch = chains[chain];
  const int T = ch.T;
  uint8_t* ring = ws + ch.ring_offset;
  uint8_t* ctl = ws + ch.ctl_offset;
  const size_t rec_bytes = sg_rec_bytes(K);
  extern __shared__ __align__(16) unsigned char smem[];
  uint32_t* st_ = (uint32_t*)(smem + lay.st);
  double* lw_ = (double*)(smem + lay.lw);
  double* w_ = (double*)(smem + lay.w);
  double* base_ = (double*)(smem + lay.base);
  double* cont_ = (double*)(smem + lay.cont);
  int* anc = (int*)(smem + lay.anc);
  double* lwres = (double*)(smem + lay.lwres);
  double* logq = (double*)(smem + lay.logq);
  int* sidx = (int*)(smem + lay.sidx);
  hyg_u128* cum = (hyg_u128*)(smem + lay.cum);
  uint64_t* xk = (uint64_t*)(smem + lay.xk);
  int* xi = (int*)(smem + lay.xi);
  double* BK = (double*)(smem + lay.BK);
  hyg_sgpe_model* pm = PE ? (hyg_sgpe_model*)(smem + lay.pm) : nullptr;
  double* logP = PE ? pm->logP : (double*)(smem + lay.logP);
  unsigned char* red = smem + lay.red;
  double* redc = (double*)(red + sg_red_w(NW));   // continuing particles: block max partials
  int* redn = (int*)(redc + NW);                  //   and finite counts (see the normalisation)
  double* Amax = (double*)(redn + NW + (NW & 1)); // [K] A_r (backward kernels)
  unsigned long long* Elimb = (unsigned long long*)(Amax + K);  // [K][2] 51-bit limbs of E_r ([K][3] reserved)
  double* Gq = (double*)(Elimb + 3 * K);          // [K][K] G[r][q]
  double* mqv = Gq + K * K;                       // [K] m_q
  double* logm = (double*)(smem + lay.logm);
  double* logQ = (double*)(smem + lay.logQ);
  SgShared& sh = *(SgShared*)(smem + lay.sh);
  const double* Ech = E + (size_t)ch.site_begin * K;

  if (!PE)
    for (int i = tid; i < K * K; i += NB) logP[i] = c.logP[i];
  // parameter estimation state (OnlineParameterEstimation.h:42-176)
  double* gfr = PE ? (double*)(smem + lay.gfr) : nullptr;  // [2][NT] gomg of each particle
  double* gct = PE ? (double*)(smem + lay.gct) : nullptr;  // [2][NT] continuation entry
  int* peLr = PE ? (int*)(smem + lay.pei) : nullptr;       // [KMAX] rows valid per regime
  int* peEx = PE ? peLr + HYG_KMAX : nullptr;              // [KMAX] exited at the last row
  int8_t* rpu = PE ? (int8_t*)(smem + lay.rpu) : nullptr;  // [2][NT] r if d >= u else -1
  SgPeChain pc{};
  // phi holds the K^2 P / omega coordinates; with kappa estimated theta has
  // K more (dth = K (K + 1)) whose score is identically 0 (include/hyg_sg_pe.h)
  constexpr int dim = K * K, jw = K * (K - 1);
  const int every = PE ? pe.c.every : 1;
  const int dth = PE ? pe.c.dim : dim;
  if constexpr (PE) {
    pc = sg_pe_chain(ws, ch, K);
    for (int j = tid; j < dth; j += NB) {
      const double th0 = pe.theta0[j];
      pc.th[j] = th0;
      pc.am[j] = 0.0;
      pc.av[j] = 0.0;
      pc.gp[j] = 0.0;  // gradientCurr at t = 0: the filtered mean of phi = 0
      pe.theta_out[(size_t)ch.theta_row * dth + j] = th0;
    }
    for (int i = tid; i < K * dim; i += NB) pc.phi[i] = 0.0;  // phi of the K initial particles
    __syncthreads();
    sg_pe_rebuild<NB>(pe, c, pc, pm, peLr, peEx, K, u, 1 + every + 1);
  }
  for (int i = tid; i <= NT; i += NB) logm[i] = hyg_log((double)i);  // log(M - k) of the K loop
  // phase timers: 0 copy, 1 sort, 2 K loop, 3 residual / keep-top, 4 weights,
  // 5 normalise, 6 smoothing, 7 compaction; counters 8 optimal steps, 9
  // keep-top steps, 10 K-loop iterations, 11 pending entries, 12 parameter
  // estimation (phi, updates, rebuilds), 15 = last stamp
  if (tid < kSgPh) sh.ph[tid] = 0;
#define SG_PH(k)                                                   \
  if (dbg && tid == 0) {                                           \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    sh.ph[k] += now_ - sh.ph[kSgPh - 1];                           \
    sh.ph[kSgPh - 1] = now_;                                       \
  }
#define SG_CNT(k, v) \
  if (dbg && tid == 0) sh.ph[k] += (v);
  if (tid == 0) sh.status = HYG_OK;
  // ---- t = 0 (Smc.h:114-188): N = K particles (1, r), log w = -log K + log g_0(r)
  int N = K;
  uint32_t my_st = sg_pack(1, tid < K ? tid : 0);
  double my_lw = (tid < K) ? -c.log_K + Ech[tid] : HYG_NINF;
  double my_base = HYG_NINF, my_cont = HYG_NINF;
  if constexpr (PE) {
    if (tid < K) {
      double gf, gcn;
      int ov = 0;
      sg_pe_parts(pc, peLr, peEx, u, my_st, my_base, my_cont, gf, gcn, ov);
      gfr[tid] = gf;
      gct[tid] = gcn;
      rpu[tid] = (int8_t)(sg_d(my_st) >= u ? sg_r(my_st) : -1);
    }
  } else {
    if (tid < K) sg_trans_parts(md, u, my_st, my_base, my_cont);
  }
  double mx0;
  int fin;
  block_max_cnt<NB>(my_lw, (tid < K && hyg_isfinite(my_lw)) ? 1 : 0, red, &mx0, &fin);
  if (!(mx0 > HYG_NINF)) {
    // no finite initial weight: publish the abort code as the post-loop path
    // does, so the smoothing workgroup stops at once and writes the status
    if (tid == 0) sg_st4(ctl + 8, (unsigned)(-HYG_ENUMERIC));
    return;
  }
  double logZ =
      mx0 + hyg_log(hyg_u128_to_f64(block_sum128<NB>(hyg_exp_fix100(my_lw - mx0), red), 100));
  double my_w = (tid < K) ? hyg_exp(my_lw - logZ) : 0.0;
  if (tid < K) {
    st_[tid] = my_st;
    lw_[tid] = my_lw;
    w_[tid] = my_w;
    base_[tid] = my_base;
    cont_[tid] = my_cont;
  }
  __syncthreads();

  int status = HYG_OK;
  int tail_seen = 0;  // records the smoothing workgroup has consumed, as last read
  constexpr int KHr = (NB == 2 * NT) ? (K + 1) / 2 : K;  // backward-kernel rows per thread (see the weights)
  double BKr[KHr];
#pragma unroll
  for (int j = 0; j < KHr; ++j) BKr[j] = 0.0;
  if (dbg && tid == 0) sh.ph[kSgPh - 1] = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < T; ++t) {
    const int cb = t & 1, pb = cb ^ 1;  // LDS buffers of the current / previous particle sets
    int M = 0, Np = N;
    bool check_top = false;  // a keep-top step: its order is confirmed behind the barrier
    // this thread's ancestor and resampled log-weight (tid < M) when the thread
    // chose them itself (keep-top, no resampling): read from registers, not
    // back from LDS behind the barrier; the optimal branch spreads them over
    // the threads (anc_lds)
    int my_anc = tid;
    double my_lwr = HYG_NINF;
    bool anc_lds = false;
    if (t > 0) {
      // ---- Smc::iterate (:190-286): the current set becomes the previous one
      const uint32_t* stP = st_ + pb * NT;
      const double* lwP = lw_ + pb * NT;
      const double* contP = cont_ + pb * NT;
      const double* Et = Ech + (size_t)t * K;
      double et[K];
#pragma unroll
      for (int q = 0; q < K; ++q) et[q] = Et[q];
      const double logZp = logZ;
      const double pw = my_w, plw = my_lw, pbase = my_base;
      const uint32_t pst = my_st;
      N = (Np + K > Nmax) ? Nmax : Np + K;
      M = N - K;
      // the systematic uniforms (systematicBase, resample.h:85-117) of steps
      // 64 j .. 64 j + 63, at the block's first step, by the last wave, which
      // holds no particle (512 threads): lane l draws step 64 j + l while the
      // key waves sort (read behind the sort's barriers; the previous block's
      // last reader is behind the previous step's barriers)
      if (NB == 2 * NT && wv == NW - 1 && (t == 1 || (t & 63) == 0))
        sh.uring[lane] =
            (double)(hyg_rand64(ch.seed, ch.chain_id, kSgRngSystematic, (uint64_t)((t & ~63) + lane), 0) >> 11) *
            1.1102230246251565404e-16;
      SG_PH(0);
      // ---- resampleCp (:406-450)
      if (N < Np + K) {
        bool keep_top = true;
        // weights with a nonzero F = 100 image (order-free): each wave's count
        // is published before the sort and read behind its cross-wave barriers
        // (red's previous readers are behind the previous step's last barrier)
        int* nzw = (int*)red + 2 * NW;
        if (fin > M) {
          const int wnz0 = __builtin_popcountll(wave_ballot(tid < Np && pw >= 0x1p-100));
          if (lane == 0) nzw[wv] = wnz0;
        }
        // order by log-weight (the keep-top fallback's order, Smc.h:432-441), on
        // packed words: exact wherever the order is used (the optimal branch
        // re-checks it against w below, the keep-top path with the full keys)
        uint64_t lkey = sg_pack_key((tid < Np) ? sg_okey(plw) : 0, tid & (NT - 1), md.key_keep);
        sg_rank_sort_packed<NB>(lkey, xk);
        const int lidx = sg_packed_idx(lkey);
        if (!PE) { SG_PH(12); }
        const double* wP = w_ + pb * NT;
        int nz0 = 0;
        if (fin > M) {
#pragma unroll
          for (int w = 0; w < NW; ++w) nz0 += nzw[w];
        }
        // Fewer than M weights with a nonzero image: the K loop provably ends in
        // the keep-top fallback (see below), so neither the order check nor the
        // loop runs
        if (fin > M && nz0 >= M) {
          // optimalFiniteState (resample.h:289-409) on the weights sorted
          // descending, ties by index. The log-weight order already is that
          // order when every adjacent pair along it has w decreasing, or w
          // equal and the indices ascending (a total order is checked by its
          // adjacent pairs); otherwise the exact sort by w runs. Either way
          // idx is the order the optimal branch assigns: no second sort there.
          // Ties among zero weights may stand in any order: w = exp(lw - log Z)
          // is monotone, so they fill the same tail positions in both orders,
          // and the branch never references a zero-weight entry (K counts
          // log q > -c only, a systematic draw lands on positive mass only).
          double q = (tid < Np) ? wP[lidx] : 0.0;
          if (tid < NT) {
            logq[tid] = q;
            sidx[tid] = lidx;
          }
          // adjacent pairs inside a wave after a wave-level hand-off; the pairs
          // across waves from LDS behind the one barrier of the exchange (the
          // previous users of red are behind the previous step's last barrier)
          auto out_of_order = [](double q1, int i1, double q2, int i2) {
            return !(q1 > q2 || (q1 == q2 && (i1 < i2 || q1 == 0.0)));
          };
          wave_lds_sync();
          bool bad = false;
          if (tid < NT && lane < 63 && tid + 1 < Np) bad = out_of_order(q, lidx, logq[tid + 1], sidx[tid + 1]);
          {
            const int wbad = wave_ballot(bad) != 0 ? 1 : 0;
            const int wnz = __builtin_popcountll(wave_ballot(tid < Np && q >= 0x1p-100));
            if (lane == 0) {
              ((int*)red)[2 * wv] = wbad;
              ((int*)red)[2 * wv + 1] = wnz;
            }
          }
          lds_barrier();
          bool disorder = false;
          int nz = 0;  // weights with a nonzero F = 100 image
#pragma unroll
          for (int w = 0; w < NW; ++w) {
            disorder = disorder || ((int*)red)[2 * w] != 0;
            nz += ((int*)red)[2 * w + 1];
          }
#pragma unroll
          for (int w = 0; w + 1 < NT / 64; ++w) {
            const int p0 = 64 * w + 63;
            if (p0 + 1 < Np) disorder = disorder || out_of_order(logq[p0], sidx[p0], logq[p0 + 1], sidx[p0 + 1]);
          }
          if (!PE) { SG_PH(13); }
          // Fewer than M weights with a nonzero image: the K loop provably ends
          // in the keep-top fallback, so it is not run. At an iterate k < nz,
          // the exact suffix Q(k) <= (nz - k) q_k <= (M - 1 - k) q_k, so
          // log q_k - (log Q(k) - log(M - k)) >= log((M - k) / (M - 1 - k)) >=
          // 1/256, far above the rounding of the logs: q_k is counted and k
          // grows. Once k >= nz, Q(k) = 0 and log c is +inf or NaN, never finite.
          if (nz >= M) {
            int idx = lidx;
            if (disorder) {
              uint64_t key = (tid < Np) ? sg_okey(pw) : 0;
              idx = tid;
              sg_bitonic<NB>(key, idx, xk, xi);
              q = (tid < Np) ? sg_okey_value(key) : 0.0;
            }
            double lq = HYG_NINF;
            hyg_u128 mq = hyg_u128_zero();
            if (tid < Np) {
              lq = hyg_log(q);
              mq = hyg_fix100(q);
            }
            if (tid < NT) {
              logq[tid] = lq;
              sidx[tid] = idx;
            }
            // reverse cumulative sums Q(k) = total - exclusive prefix (exact),
            // the prefix and the total in registers (no LDS round trip, no
            // barriers around one)
            {
              hyg_u128 ex, tot;
              block_scan128_regs<NB>(mq, red, &ex, &tot);
              if (!PE) { SG_PH(14); }
              hyg_u128 suf;
              suf.lo = tot.lo - ex.lo;
              suf.hi = tot.hi - ex.hi - (tot.lo < ex.lo ? 1u : 0u);
              if (tid <= NT) logQ[tid] = hyg_log(hyg_u128_to_f64(suf, 100));
              if (NB == NT && tid == 0) logQ[NT] = HYG_NINF;
            }
            lds_barrier();
            SG_PH(1);
            // the K / log c fixed point (:333-342). When log q is non-increasing
            // along the sorted order (checked; log is only nearly monotone), the
            // count #{p >= a : log q_p > -c(a)} is a prefix length: every a in
            // [0, Np] gets c(a) and its successor next(a) by a binary search at
            // once, then one lane follows a -> next(a) from 0 to the fixed point
            // (the loop's iterates, so K and log c are the loop's). Otherwise the
            // loop runs in wave 0 with counts by ballot.
            const bool lqmono = !block_or<NB>(tid + 1 < Np && logq[tid + 1] > logq[tid], red);
            if (lqmono) {
              double* cval = (double*)cum;           // [NT + 1] c(a)
              int* nxt = (int*)(cval + NT + 1);      // [NT + 1] next(a)
              for (int a = tid; a <= Np; a += NB) {
                const int mk = M - a;
                const double cA = (mk >= 0 ? logm[mk] : HYG_NAN) - logQ[a];
                const double thr = -cA;
                int lo = 0, hi = Np;  // first p with !(log q_p > thr)
                while (lo < hi) {
                  const int mid = (lo + hi) >> 1;
                  if (logq[mid] > thr) lo = mid + 1; else hi = mid;
                }
                nxt[a] = a + (lo > a ? lo - a : 0);
                cval[a] = cA;
              }
              lds_barrier();
              if (tid == 0) {
                int kOld = 1, kNew = 0, iters = 0;
                while (kNew != kOld) {
                  kOld = kNew;
                  kNew = nxt[kOld];
                  ++iters;
                }
                sh.Kk = kNew;
                sh.logC = cval[kOld];
                SG_CNT(10, iters);
              }
            } else if (wv == 0) {
              double lq4[4];
#pragma unroll
              for (int i = 0; i < 4; ++i) lq4[i] = logq[lane + 64 * i];
              int kOld = 1, kNew = 0, iters = 0;
              double logC = 0.0;
              while (kNew != kOld) {
                kOld = kNew;
                // hyg_log(M - kOld) - hyg_log(Q(kOld)) from the tables (log of a negative count is NaN)
                const int mk = M - kOld;
                logC = (mk >= 0 ? logm[mk] : HYG_NAN) - logQ[kOld];
                const double thr = -logC;
                int cnt = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                  const int p = lane + 64 * i;
                  cnt += __builtin_popcountll(__ballot(p >= kOld && p < Np && lq4[i] > thr));
                }
                kNew = kOld + cnt;
                ++iters;
              }
              if (lane == 0) {
                sh.Kk = kNew;
                sh.logC = logC;
              }
              SG_CNT(10, iters);
            }
            lds_barrier();
            SG_PH(2);
            const double logC = sh.logC;
            if (hyg_isfinite(logC)) {
              keep_top = false;
              anc_lds = true;
              const int Kk = sh.Kk, L = M - Kk;
              if (tid < Kk) {
                anc[tid] = idx;
                lwres[tid] = lwP[idx];
              }
              if (L > 0) {
                // residual systematic draw (:372-377, systematicBase :85-117):
                // T_j = (j + u) / L <= Q_i as exact C_i >= ceil(T_j R)
                const bool inres = tid >= Kk && tid < Np;
                // the residual's largest log q: with log q non-increasing along the
                // sorted order (lqmono, checked for the K loop) it is position Kk's
                const double rmax = lqmono ? logq[Kk] : block_max<NB>(inres ? lq : HYG_NINF, red);
                const hyg_u128 m2 = inres ? hyg_exp_fix100(lq - rmax) : hyg_u128_zero();
                // C(p - 1) at sorted position p = tid, and R = C(Np - 1), the
                // block total (m2 is 0 from Np on), in registers
                hyg_u128 exv, R;
                block_scan128_regs<NB>(m2, red, &exv, &R);
                const hyg_u128 incl = hyg_u128_add(exv, m2);
                if (inres) {
                  // target j lands on the first position p >= Kk with C(p) >= ceil(T_j R):
                  // position p takes the targets j in [count(C(p - 1)), count(C(p)))
                  // (position Kk from j = 0), counted per position instead of
                  // searched per target
                  const double uu =
                      (NB == 2 * NT) ? sh.uring[t & 63]
                                     : (double)(hyg_rand64(ch.seed, ch.chain_id, kSgRngSystematic, (uint64_t)t, 0) >> 11) *
                                           1.1102230246251565404e-16;
                  const double invR = 1.0 / hyg_u128_to_f64(R, 100);
                  const int cHi = sg_sys_count(incl, R, invR, L, uu);
                  const int cLo = (tid == Kk) ? 0 : sg_sys_count(exv, R, invR, L, uu);
                  for (int j = cLo; j < cHi; ++j) {
                    anc[Kk + j] = idx;
                    lwres[Kk + j] = logZp - logC;
                  }
                }
              }
            }
          }
        }
        if (keep_top) {
          // keep the M largest log-weights (Smc.h:432-441, resample.h:379-384).
          // The packed words order keys that agree on their top 56 bits by
          // index: every adjacent pair of real positions is checked with the
          // full keys, the pairs inside a wave here, the three across waves
          // behind the barrier below (then the exact pair sort redoes it).
          uint64_t fk = 0;
          double flw = HYG_NINF;
          if (tid < Np) {
            flw = lwP[lidx];
            fk = sg_okey(flw);
          }
          if (tid < M) {
            anc[tid] = lidx;
            lwres[tid] = flw;
          }
          if (tid < NT) {
            const uint64_t nk = ((uint64_t)sg_lane_next((uint32_t)(fk >> 32)) << 32) | sg_lane_next((uint32_t)fk);
            const int ni = (int)sg_lane_next((uint32_t)lidx);
            const bool bad = lane < 63 && tid + 1 < Np && !(fk > nk || (fk == nk && lidx < ni));
            const int wbad = wave_ballot(bad) != 0 ? 1 : 0;
            if (lane == 0) {
              sh.kfirst[wv] = fk;
              sh.ifirst[wv] = lidx;
              sh.kbad[wv] = wbad;
            }
            if (lane == 63) {
              sh.klast[wv] = fk;
              sh.ilast[wv] = lidx;
            }
          }
          check_top = true;
          my_anc = lidx;
          my_lwr = flw;
        }
        SG_CNT(8, keep_top ? 0 : 1);
        SG_CNT(9, keep_top ? 1 : 0);
      } else if (tid < M) {
        anc[tid] = tid;
        lwres[tid] = plw;
        my_lwr = plw;
      }
      // the weights' LDS accumulators, behind this barrier (their last readers
      // were behind the previous step's last barrier; block reductions do not
      // touch them)
      if (tid < K) Amax[tid] = HYG_NINF;
      if (tid < 2 * K) Elimb[tid] = 0ull;
      lds_barrier();
      if (check_top) {
        // every value loaded first (one LDS round trip), then a branch-free test
        constexpr int KW = NT / 64;
        uint64_t kf[KW], kl[KW];
        int jf[KW], jl[KW], kb[KW];
#pragma unroll
        for (int w = 0; w < KW; ++w) {
          kf[w] = sh.kfirst[w];
          kl[w] = sh.klast[w];
          jf[w] = sh.ifirst[w];
          jl[w] = sh.ilast[w];
          kb[w] = sh.kbad[w];
        }
        int redo = 0;
#pragma unroll
        for (int w = 0; w < KW; ++w) {
          redo |= kb[w];
          if (w + 1 < KW) {
            const uint64_t a = kl[w], b = kf[w + 1];
            const bool ok = (a > b) | ((a == b) & (jl[w] < jf[w + 1]));
            redo |= (64 * (w + 1) < Np && !ok) ? 1 : 0;
          }
        }
        if (redo != 0) {  // uniform: the exact pair sort
          uint64_t key = (tid < Np) ? sg_okey(plw) : 0;
          int idx = tid;
          sg_bitonic<NB>(key, idx, xk, xi);
          my_anc = idx;
          my_lwr = (tid < Np) ? lwP[idx] : HYG_NINF;
          if (tid < M) {
            anc[tid] = my_anc;
            lwres[tid] = my_lwr;
          }
          lds_barrier();
          SG_CNT(22, 1);
        }
      }
      SG_PH(3);
      // ---- sampleParticlesCp (:504-522) + computeWeightsCp (:536-574)
      double nlw = HYG_NINF;
      uint32_t nst = 0;
      if (tid < M) {
        const int a = anc_lds ? anc[tid] : my_anc;
        const uint32_t sa = stP[a];
        const int r = sg_r(sa);
        double e = et[0];
#pragma unroll
        for (int q = 1; q < K; ++q) e = (r == q) ? et[q] : e;
        nst = sg_pack(sg_d(sa) + 1, r);
        nlw = (anc_lds ? lwres[tid] : my_lwr) + (contP[a] + e);
      }
      // the hazard parts of this thread's new particle (consumed next step):
      // the L2 loads issued here, in flight through the weights' and the
      // normalisation's barriers (fresh particle q = tid - M: state (1, q))
      double2 nh = make_double2(0.0, 0.0);
      uint8_t nex = 0;
      if (!PE && tid < N) sg_trans_load(md, tid < M ? nst : sg_pack(1, tid - M), nh, nex);
      // backward kernels (:288-326), factorised over the regimes as in
      // oracle/sg_oracle.c: a_n = W_prev[n] + b_n (b_n + log P[r_n][q] = log
      // f((1,q) | n)), A_r = max of a_n over regime r, m_q = max_r (A_r + log
      // P[r][q]), K_q(n) = (e_n G[r_n][q]) / S_q with e_n = exp(a_n - A_{r_n}),
      // G[r][q] = exp((A_r + log P[r][q]) - m_q), S_q = sum_r G[r][q] E_r (E_r:
      // the exact image sum of e_n over regime r); the fresh particle (1, q)
      // has log weight m_q + log S_q + log g_t(q). Per particle one exp, an
      // LDS max and three limb adds (exact, order-free), K^2 exps per step.
      // With 512 threads (K <= 8) thread n < 256 takes rows [0, KH) of previous
      // particle n and thread 256 + n rows [KH, K) (it recomputes e_n); threads
      // 256 .. 256 + K^2 form G.
      constexpr bool SPLIT = (NB == 2 * NT);
      // the G wave below is one wave (64 lanes) forming the K^2 entries of G:
      // the 512-thread build is dispatched for K <= 8 only (SG_CASE)
      static_assert(!SPLIT || K * K <= 64, "the split build's single G wave holds at most 64 entries");
      constexpr int KH = SPLIT ? (K + 1) / 2 : K;
      const int pn = SPLIT ? (tid & (NT - 1)) : tid;  // the previous particle of this thread
      const int q0 = (SPLIT && tid >= NT) ? KH : 0;   // wave-uniform
      double va;
      int vr;
      {
        double vlw = plw, vbase = pbase;
        uint32_t vst = pst;
        if (SPLIT && tid >= NT) {
          vlw = lwP[pn];
          vbase = base_[pb * NT + pn];
          vst = stP[pn];
        }
        va = (pn < Np) ? vlw + vbase : HYG_NINF;
        vr = (va > HYG_NINF) ? sg_r(vst) : 0;  // (no weight: any valid row of G, times e_n = 0)
      }
      if (tid < NT && va > HYG_NINF)
        __hip_atomic_fetch_max(Amax + vr, va, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (!PE) { SG_PH(7); }
      {
        // the continuing particles' part of the block max and finite count of
        // the new log-weights rides on this barrier; the fresh particles' part
        // is added from lsv below (no reduction of its own)
        const double cm = wave_max(nlw);  // -inf beyond the continuing particles
        const int cn = __builtin_popcountll(wave_ballot(tid < M && hyg_isfinite(nlw)));
        if (lane == 0) {
          redc[wv] = cm;
          redn[wv] = cn;
        }
      }
      lds_barrier();
      if (!PE) { SG_PH(16); }
      double ea;
      if (SPLIT && wv == NT / 64) {
        // the G wave (threads NT .. NT + K^2 form G[r][q], below otherwise): its
        // e_n and G exps in one straight-line block, so the two chains interleave
        const int gi = tid - NT;  // (r, q) = (gi / K, gi % K)
        const bool gth = gi < K * K;
        const int r = gth ? gi / K : 0, q = gth ? gi - (gi / K) * K : 0;
        double m = HYG_NINF;
#pragma unroll
        for (int rr = 0; rr < K; ++rr) m = dmax(m, Amax[rr] + logP[rr * K + q]);
        const double xg = (Amax[r] + logP[r * K + q]) - m;
        const double xa = (va > HYG_NINF) ? va - Amax[vr] : 0.0;
        const double eg = hyg_exp(xg), e1 = hyg_exp(xa);
        ea = (va > HYG_NINF) ? e1 : 0.0;
        if (gth) {
          Gq[gi] = (m > HYG_NINF) ? eg : 0.0;
          if (r == 0) mqv[q] = m;
        }
      } else {
        ea = (va > HYG_NINF) ? hyg_exp(va - Amax[vr]) : 0.0;
        const int gi = tid;  // 256 threads: (r, q) = (gi / K, gi % K)
        if (!SPLIT && gi < K * K) {
          const int r = gi / K, q = gi - (gi / K) * K;
          double m = HYG_NINF;
#pragma unroll
          for (int rr = 0; rr < K; ++rr) m = dmax(m, Amax[rr] + logP[rr * K + q]);
          Gq[gi] = (m > HYG_NINF) ? hyg_exp((Amax[r] + logP[r * K + q]) - m) : 0.0;
          if (r == 0) mqv[q] = m;
        }
      }
      if (tid < NT && va > HYG_NINF) {
        // e_n <= 1, so the image is <= 2^100: limbs of 51 and 50 bits, whose sums
        // over <= 256 particles stay below 2^59 (two LDS adds per particle)
        const hyg_u128 im = hyg_fix100(ea);
        unsigned long long* el = Elimb + 2 * vr;
        constexpr unsigned long long kL = (1ull << 51) - 1;
        __hip_atomic_fetch_add(el + 0, im.lo & kL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(el + 1, (im.lo >> 51) | (im.hi << 13), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (!PE) { SG_PH(17); }
      lds_barrier();
      if (!PE) { SG_PH(11); }
      // every wave: lane r converts regime r's exact sum E_r, lane q forms
      // S_q = sum_r G[r][q] E_r with the E_r read across lanes (readlane), in r
      // order (the same FMA chain), and row q's log-normaliser lsq and 1 / S_q;
      // the values are read across lanes below (the same bits in every wave:
      // no LDS hand-off, no barrier)
      double lsq, isq;
      {
        double Er = 0.0;
        if (lane < K) {
          const unsigned long long* el = Elimb + 2 * lane;
          // E_r = l0 + l1 2^51 (l0 < 2^59, l1 < 2^58: sums of <= 256 limbs)
          hyg_u128 e, x;
          e.lo = el[0]; e.hi = 0;
          x.lo = el[1] << 51; x.hi = el[1] >> 13;
          e = hyg_u128_add(e, x);
          Er = hyg_u128_to_f64(e, 100);
        }
        const int q = lane < K ? lane : 0;
        double g[K];
#pragma unroll
        for (int r = 0; r < K; ++r) g[r] = Gq[r * K + q];
        const double m = mqv[q];
        double S = 0.0;
#pragma unroll
        for (int r = 0; r < K; ++r) S = HYG_FMA(g[r], d_of(rdlane64(u_of(Er), r)), S);
        lsq = (m > HYG_NINF) ? m + hyg_log(S) : HYG_NINF;
        isq = (m > HYG_NINF) ? 1.0 / S : 0.0;
      }
      auto lsev_of = [&](int q) { return d_of(rdlane64(u_of(lsq), q)); };  // q wave-uniform
      if (!PE) { SG_PH(18); }
      if (!PE) { SG_PH(19); }
#pragma unroll
      for (int j = 0; j < KH; ++j) {  // this thread's entries of the backward kernels (record of step t)
        const int q = q0 + j < K ? q0 + j : K - 1;
        const double lq = lsev_of(q), iq = d_of(rdlane64(u_of(isq), q));
        BKr[j] = (q0 + j < K && lq > HYG_NINF) ? (ea * Gq[vr * K + q]) * iq : 0.0;
        if (PE && pn < Np && q0 + j < K) BK[q * NT + pn] = BKr[j];
      }
      double lsv[K];  // row q's log-normaliser in every lane (the fresh particles, the normalisation)
#pragma unroll
      for (int q = 0; q < K; ++q) lsv[q] = lsev_of(q);
      if (tid >= M && tid < N) {
        const int q = tid - M;
        double e = et[0], lb = lsv[0];
#pragma unroll
        for (int qq = 1; qq < K; ++qq) {
          e = (q == qq) ? et[qq] : e;
          lb = (q == qq) ? lsv[qq] : lb;
        }
        nlw = (lb > HYG_NINF) ? lb + e : HYG_NINF;
        nst = sg_pack(1, q);
      }
      SG_PH(4);
      // ---- selfNormaliseWeights (:576-579)
      // record t-1 (stored at the end of step t-1) is drained by every wave
      // here, before the barriers of the reductions; published after them
      sg_drain_stores();
      if (!PE) { SG_PH(20); }
      // block max and finite count of the N new log-weights: the continuing
      // particles' wave partials and the K fresh ones (lsv[q] + log g_t(q), as
      // formed above), the same values as one block reduction (a max is exact)
      double mx = redc[0];
      fin = redn[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) {
        mx = dmax(mx, redc[w]);
        fin += redn[w];
      }
#pragma unroll
      for (int q = 0; q < K; ++q) {
        const double lb = lsv[q];
        const double f = (lb > HYG_NINF) ? lb + et[q] : HYG_NINF;
        mx = dmax(mx, f);
        fin += hyg_isfinite(f) ? 1 : 0;
      }
      if (!(mx > HYG_NINF)) {
        status = HYG_ENUMERIC;
        break;
      }
      {
        hyg_u128 fx = hyg_u128_zero();
        if ((NB == NT) || wv < NT / 64) fx = hyg_exp_fix100(nlw - mx);  // waves >= 4 hold no particle
        // (no leading barrier: red's last readers, the weights' partials, are
        // behind the weights' last barrier)
        const hyg_u128 Sx = block_sum128<NB, false>(fx, red);
        if (!PE) { SG_PH(21); }
        logZ = mx + hyg_log(hyg_u128_to_f64(Sx, 100));
      }
      if (tid == 0) sg_st4(ctl, (unsigned)t);  // records 0 .. t-1 are published
      my_lw = nlw;
      my_st = nst;
      my_w = 0.0;
      if (tid < N) my_w = hyg_exp(nlw - logZ);
      if (tid < N) {
        st_[cb * NT + tid] = my_st;
        lw_[cb * NT + tid] = my_lw;
        w_[cb * NT + tid] = my_w;
        if (!PE) sg_trans_form(u, my_st, nh, nex, my_base, my_cont);  // (loaded with the weights)
      }
      SG_PH(5);
      if constexpr (PE) {
        // updatePhi (OnlineParameterEstimation.h:118-150) with the gradients of
        // the log transition density (singleGroup.h:641-717) under the current
        // theta, in the oracle's order (oracle/sg_oracle.c)
        const double* phiP = pc.phi + (size_t)pb * NT * dim;
        double* phiC = pc.phi + (size_t)cb * NT * dim;
        const double* gfrP = gfr + pb * NT;
        const uint32_t* stPP = st_ + pb * NT;
        // continuing particles: phi of the ancestor + the omega entry, one
        // (particle, coordinate) element per thread and iteration (coalesced rows)
        constexpr int kCb0 = (NT * dim + NB - 1) / NB;  // all elements in one round of loads (K <= 6)
        constexpr int kCb = kCb0 < 18 ? kCb0 : 18;
        for (int e0 = 0; e0 < M * dim; e0 += kCb * NB) {
          double v[kCb];
#pragma unroll
          for (int i = 0; i < kCb; ++i) {
            const int e = e0 + i * NB + tid;
            const int n = e / dim, j = e - n * dim;
            v[i] = (e < M * dim) ? phiP[(size_t)anc[n] * dim + j] : 0.0;
          }
#pragma unroll
          for (int i = 0; i < kCb; ++i) {
            const int e = e0 + i * NB + tid;
            if (e < M * dim) {
              const int n = e / dim, j = e - n * dim;
              const int a = anc[n];
              phiC[e] = v[i] + ((j == jw + sg_r(stPP[a])) ? gct[pb * NT + a] : 0.0);
            }
          }
        }
        // fresh particle (1, q), coordinate j: the sum over the previous
        // particles in kCh fixed chunks of rows (hyg_sgpe_fresh_chunks), each
        // in n order, one (chunk, q, j) task per thread. The gradient of
        // log f((1, q) | (d_n, r_n)) at j is nonzero only when q != r_n,
        // d_n >= u and r_n is j's regime rt (the regime of the omega entry or
        // of the P block j lies in): then it is gomg_n, resp. the constant
        // -P[rt][jj] (+1 if jj == q). Per term: one byte compare against
        // rpu[n] (r_n if d_n >= u, else -1) and a select, over batches of kFb
        // previous particles loaded at once (phi rows up to 256 exist; the
        // ones >= Np are not used). Chunk sums meet in LDS (scr) and are added
        // left to right.
        constexpr int kCh = (K <= 8 ? 512 : 256) / (K * K * K) >= 8 ? 8
                          : (K <= 8 ? 512 : 256) / (K * K * K) >= 4 ? 4
                          : (K <= 8 ? 512 : 256) / (K * K * K) >= 2 ? 2 : 1;
        constexpr int kRows = NT / kCh;
        constexpr int kFb = 8;
        double* part = (double*)(smem + lay.scr);  // [kCh][K][dim] when kCh > 1
        const int8_t* rpuP = rpu + pb * NT;
        for (int e = tid; e < kCh * K * dim; e += NB) {
          const int ck = e / (K * dim), pq = e - ck * (K * dim);
          const int q = pq / dim, j = pq - q * dim;
          const bool isw = j >= jw;
          const int rt = isw ? j - jw : j / (K - 1);
          double cval = 0.0;
          if (!isw) {
            const int ii = j - rt * (K - 1), jj = (ii < rt) ? ii : ii + 1;
            cval = -pm->P[rt * K + jj];
            if (jj == q) cval = cval + 1.0;
          }
          const int rsel = (rt == q) ? -2 : rt;  // -2 matches no particle
          const double* col = phiP + j;
          const double* bkq = BK + q * NT;
          const int nb0 = ck * kRows, nb1 = (nb0 + kRows < Np) ? nb0 + kRows : Np;
          double acc = 0.0;
          for (int n0 = nb0; n0 < nb1; n0 += kFb) {
            double v[kFb], bk[kFb], gf[kFb];
            int rp[kFb];
#pragma unroll
            for (int i = 0; i < kFb; ++i) {
              v[i] = col[(size_t)(n0 + i) * dim];
              rp[i] = rpuP[n0 + i];
              bk[i] = bkq[n0 + i];
              gf[i] = gfrP[n0 + i];  // loaded unconditionally, selected below (no exec-mask branches)
            }
            if (n0 + kFb <= nb1) {
#pragma unroll
              for (int i = 0; i < kFb; ++i) {
                const double g = (rp[i] == rsel) ? (isw ? gf[i] : cval) : 0.0;
                acc = acc + bk[i] * (v[i] + g);
              }
            } else {
#pragma unroll
              for (int i = 0; i < kFb; ++i) {
                const double g = (rp[i] == rsel) ? (isw ? gf[i] : cval) : 0.0;
                const double term = bk[i] * (v[i] + g);
                acc = (n0 + i < nb1) ? acc + term : acc;
              }
            }
          }
          if (kCh == 1) phiC[(size_t)(M + q) * dim + j] = acc;
          else part[e] = acc;
        }
        if (kCh > 1) {
          lds_barrier();
          for (int pq = tid; pq < K * dim; pq += NB) {
            double acc = part[pq];
#pragma unroll
            for (int ck = 1; ck < kCh; ++ck) acc = acc + part[ck * K * dim + pq];
            const int q = pq / dim, j = pq - q * dim;
            phiC[(size_t)(M + q) * dim + j] = acc;
          }
        }
        __syncthreads();
        if (t % every == 0) {
          // updateGradients (:151-156): filtered mean of phi, difference to the
          // previous one; GradientAscent::iterate (GradientAscent.h:82-105)
          const double* wCur = w_ + cb * NT;
          for (int j = tid; j < dth; j += NB) {
            double est = 0.0;  // the kappa coordinates (j >= K^2): sum_n W_n (+0) = +0
            if (j < dim) {
              for (int n0 = 0; n0 < N; n0 += kFb) {
                double v[kFb];
#pragma unroll
                for (int i = 0; i < kFb; ++i) v[i] = phiC[(size_t)(n0 + i) * dim + j];
#pragma unroll
                for (int i = 0; i < kFb; ++i)
                  if (n0 + i < N) est = est + wCur[n0 + i] * v[i];
              }
            }
            pc.gc[j] = est - pc.gp[j];
            pc.gp[j] = est;
          }
          __syncthreads();
          double l1 = 0.0;
          if (pe.c.normalise && !pe.c.use_adam)
            for (int j = 0; j < dth; ++j) l1 = l1 + fabs(pc.gc[j]);
          const int it = t / every - 1;
          const double lr = pe.steps[it].lr, c1 = pe.steps[it].c1, c2 = pe.steps[it].c2;
          for (int j = tid; j < dth; j += NB) {
            double am = pc.am[j], av = pc.av[j];
            const double th = hyg_sgpe_update(pe.c.use_adam, pe.c.normalise, pe.c.beta1, pe.c.beta2, pe.c.eps, lr,
                                              c1, c2, pc.th[j], pc.gc[j], l1, &am, &av);
            pc.th[j] = th;
            pc.am[j] = am;
            pc.av[j] = av;
            pe.theta_out[(size_t)(ch.theta_row + t / every) * dth + j] = th;
          }
          // rows for every sojourn the set can reach before the next rebuild
          const int maxd = (int)block_max<NB>((tid < N) ? (double)sg_d(my_st) : 0.0, red);
          __syncthreads();
          SG_PH(12);
          sg_pe_rebuild<NB>(pe, c, pc, pm, peLr, peEx, K, u, maxd + every + 1);
          SG_PH(13);
          SG_CNT(14, maxd + every + 1);
        }
        int ov = 0;
        if (tid < N) {
          double gf, gcn;
          sg_pe_parts(pc, peLr, peEx, u, my_st, my_base, my_cont, gf, gcn, ov);
          gfr[cb * NT + tid] = gf;
          gct[cb * NT + tid] = gcn;
          rpu[cb * NT + tid] = (int8_t)(sg_d(my_st) >= u ? sg_r(my_st) : -1);
        }
        if (__syncthreads_or(ov)) {
          status = HYG_ENOMEM;
          break;
        }
        SG_PH(12);
      }
    }
    // ---- hand the step to the smoothing workgroup (OnlineMarginalSmoothing::update
    //      consumes exactly these: ancestors, regimes, self-normalised weights and
    //      the backward kernels of step t): record t into ring slot t % kSgRing,
    //      once the smoothing workgroup has consumed record t - kSgRing
    if (t - kSgRing + 1 > tail_seen) {  // re-read the tail only when the cached value is not enough
      unsigned spins = 0, tl;
      while ((tl = sg_ld4(ctl + 4)) < (unsigned)(t - kSgRing + 1)) {
        if (++spins > kSgSpinMax) { tl = kSgTailAbort; break; }
        __builtin_amdgcn_s_sleep(2);
      }
      if (tl == kSgTailAbort) {  // the smoothing workgroup stopped (and reports the status)
        status = HYG_EDEVICE;
        break;
      }
      tail_seen = (int)tl;
    }
    {
      uint8_t* rec = ring + (size_t)(t % kSgRing) * rec_bytes;
      if (tid == 0) {
        sg_st8(rec, (uint64_t)(uint32_t)N | ((uint64_t)(uint32_t)Np << 32));
        sg_st8(rec + 8, (uint64_t)(uint32_t)M | ((uint64_t)(uint32_t)t << 32));
      }
      if (tid < NT) {
        const int a = (tid < M) ? anc[tid] : 0;
        const int rg = (tid < N) ? sg_r(my_st) : 0;
        sg_st8(rec + 16 + 8 * (size_t)tid, (uint64_t)(uint32_t)a | ((uint64_t)(uint32_t)rg << 32));
        sg_st8(rec + 16 + 8 * (size_t)(NT + tid), u_of(tid < N ? my_w : 0.0));
      }
      {
        const int pn = (NB == 2 * NT) ? (tid & (NT - 1)) : tid;
        const int q0 = (NB == 2 * NT && tid >= NT) ? KHr : 0;
        if (pn < Np) {
#pragma unroll
          for (int j = 0; j < KHr; ++j)
            if (q0 + j < K) sg_st8(rec + 16 + 8 * (size_t)(2 * NT + (q0 + j) * NT + pn), u_of(BKr[j]));
        }
      }
    }
    if (tid < N) {
      base_[cb * NT + tid] = my_base;
      cont_[cb * NT + tid] = my_cont;
    }
    lds_barrier();
    SG_PH(6);
  }
  // publish the last records, or the abort code for the smoothing workgroup
  sg_drain_stores();
  __syncthreads();
  if (tid == 0) {
    if (status == HYG_OK) sg_st4(ctl, (unsigned)T);
    else sg_st4(ctl + 8, (unsigned)(-status));
  }

  if (dbg && tid < kSgPh - 1) dbg[(size_t)chain * kSgPh + tid] = sh.ph[tid];
  if (dbg && tid == kSgPh - 1) dbg[(size_t)chain * kSgPh + kSgPh - 1] = (unsigned long long)T;
#undef SG_PH
#undef SG_CNT
}


// The online marginal smoothing of one chain (OnlineMarginalSmoothing.h:52-255),
// in its own workgroup: per step t it takes record t of the SMC workgroup
// (N, N_prev, M, ancestors, regimes, self-normalised weights, backward kernels)
// from the ring and runs updatePsi of the pending times, initialisePsi of t and
// storeEstimates with the epsilon rule, as (pending time, regime) tasks over
// all waves; psi rows live in LDS slots (up to 32) and the chain's workspace.
// The same operations in the same order as the in-workgroup smoothing of
// oracle/sg_oracle.c, so the outputs stay bit-identical. Writes status_out.
template <int KT, int NB>
__device__ __forceinline__ void sg_smoother(const SgModelDev md, const SgChainDev ch, int chain,
                                            uint8_t* __restrict__ ws, int cap, double* __restrict__ probs,
                                            int32_t* __restrict__ status_out, const SgCLay lay) {
  constexpr int NT = kSgThreads, NW = NB / 64, K = KT;
  const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  const double eps = md.consts->epsilon;
  const int T = ch.T;
  extern __shared__ __align__(16) unsigned char smem[];
  int* anc = (int*)(smem + lay.anc);
  uint8_t* rgn = smem + lay.rgn;
  double* wC = (double*)(smem + lay.w);
  double* BK = (double*)(smem + lay.BK);
  double* scr = (double*)(smem + lay.scr) + wv * NT;
  double* meanb = (double*)(smem + lay.meanb);
  uint8_t* okb = smem + lay.okb;
  unsigned char* red = smem + lay.red;
  SgCShared& sh = *(SgCShared*)(smem + lay.sh);
  double* psil = (double*)(smem + lay.psil);
  const int nl = lay.nl;
  uint8_t* wbase = ws + ch.psi_offset;
  double* psig = (double*)wbase;
  int32_t* lists = (int32_t*)(wbase + sg_psi_region_bytes(K, cap));
  int32_t* keepf = lists + 4 * (size_t)cap;
  int32_t* freel = lists + 5 * (size_t)cap;
  uint8_t* ring = ws + ch.ring_offset;
  uint8_t* ctl = ws + ch.ctl_offset;
  const size_t rec_bytes = sg_rec_bytes(K);
  double* out = probs + (size_t)ch.out_begin * K;
  auto slot_row = [&](int slot, int r) -> double* {
    return slot < nl ? psil + ((size_t)slot * K + r) * NT : psig + ((size_t)(slot - nl) * K + r) * NT;
  };
  (void)red;
  for (int i = tid; i < cap; i += NB) freel[i] = cap - 1 - i;
  if (tid == 0) {
    sh.npend = 0;
    sh.nfree = cap;
    sh.cur = 0;
    sh.status = HYG_OK;
    sh.avail = 0;
    sh.abort_code = 0;
    sh.lmask = nl >= 32 ? 0xffffffffu : ((1u << nl) - 1u);
  }
  __syncthreads();
  int status = HYG_OK;
  int avail = 0;
  for (int t = 0; t < T; ++t) {
    const bool final = (t == T - 1);
    if (t >= avail) {
      // wait for record t: wave 0 polls head (relaxed), ONE agent-scope acquire
      if (wv == 0) {
        unsigned h = 0, ab = 0, spins = 0;
        for (;;) {
          h = sg_ld4(ctl);
          ab = sg_ld4(ctl + 8);
          if ((int)h > t || ab != 0) break;
          if (++spins > (t == 0 ? kSgSpinFirst : kSgSpinMax)) { ab = (unsigned)(-HYG_EDEVICE); break; }
          __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        sg_drain_stores();
        if (lane == 0) {
          sh.avail = (int)h;
          sh.abort_code = (int)ab;
        }
      }
      __syncthreads();
      avail = sh.avail;
      if (avail <= t) {  // the SMC workgroup stopped (its code) or the wait timed out
        status = sh.abort_code ? -sh.abort_code : HYG_EDEVICE;
        break;
      }
    }
    // ---- record t into LDS (plain loads behind the acquire)
    const uint8_t* rec = ring + (size_t)(t % kSgRing) * rec_bytes;
    // header through vector loads (a wave-uniform plain load could take the scalar cache)
    const uint64_t h0 = __hip_atomic_load((sg_gu64*)rec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t h1 = __hip_atomic_load((sg_gu64*)(rec + 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int N = (int)(uint32_t)h0, Np = (int)(h0 >> 32), M = (int)(uint32_t)h1;
    for (int i = tid; i < NT; i += NB) {
      const uint64_t ar = ((const uint64_t*)(rec + 16))[i];
      anc[i] = (int)(uint32_t)ar;
      rgn[i] = (uint8_t)(ar >> 32);
      wC[i] = ((const double*)(rec + 16))[NT + i];
    }
    for (int i = tid; i < K * NT; i += NB) {
      const int n = i - (i / NT) * NT;
      BK[i] = (n < Np) ? ((const double*)(rec + 16))[2 * NT + i] : 0.0;
    }
    __syncthreads();
    if (tid == 0) sg_st4(ctl + 4, (unsigned)(t + 1));  // slot t % kSgRing may be rewritten
    // ---- online marginal smoothing: updatePsi (OnlineMarginalSmoothing.h:152-197)
    //      of the pending times, initialisePsi (:132-150) of time t, storeEstimates
    //      (:199-253) with the epsilon rule, as (pending time, regime) tasks
    const int cur = sh.cur, nold = sh.npend;
    int32_t* slotA = lists + (size_t)cur * 2 * cap;
    int32_t* timeA = slotA + cap;
    if (tid == 0) {
      int slot = -1;
      if (nold >= cap) {
        slot = -1;  // the pending list holds cap entries
      } else if (sh.lmask) {
        const int b = __builtin_ctz(sh.lmask);
        sh.lmask &= ~(1u << b);
        slot = b;
      } else if (sh.nfree > 0) {
        slot = nl + freel[--sh.nfree];
      }
      if (slot < 0) {
        sh.status = HYG_ENOMEM;
      } else {
        slotA[nold] = slot;
        timeA[nold] = t;
      }
    }
    __syncthreads();
    if (sh.status != HYG_OK) {
      status = sh.status;
      break;
    }
    const int ntot = nold + 1;
    for (int c0 = 0; c0 < ntot; c0 += kSgChunk) {
      const int ne = (ntot - c0 < kSgChunk) ? ntot - c0 : kSgChunk;
      for (int task = wv; task < ne * K; task += NW) {
        const int el = task / K, r = task - el * K, e = c0 + el;
        const bool fresh = (e == nold);
        double* row = slot_row(slotA[e], r);
        double nv[4];
        if (fresh) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int n = lane + 64 * i;
            nv[i] = (n < N && (int)rgn[n] == r) ? 1.0 : 0.0;
          }
        } else {
          double pv[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int n = lane + 64 * i;
            pv[i] = (n < Np) ? row[n] : 0.0;
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) scr[lane + 64 * i] = pv[i];
          wave_lds_sync();
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int n = lane + 64 * i;
            nv[i] = (n < M) ? scr[anc[n]] : 0.0;
          }
          hyg_u128 s[K];
#pragma unroll
          for (int q = 0; q < K; ++q) {
            s[q] = hyg_u128_zero();
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int n = lane + 64 * i;
              if (n < Np) s[q] = hyg_u128_add(s[q], hyg_fix100(BK[q * NT + n] * pv[i]));
            }
          }
#pragma unroll
          for (int q = 0; q < K; ++q) s[q] = wave_sum128(s[q]);
#pragma unroll
          for (int q = 0; q < K; ++q) {
            const double v = hyg_u128_to_f64(s[q], 100);
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (lane + 64 * i == M + q) nv[i] = v;
          }
          wave_lds_sync();
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = lane + 64 * i;
          if (n < N) row[n] = nv[i];
        }
        double wn[4];
        hyg_u128 sm = hyg_u128_zero();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = lane + 64 * i;
          wn[i] = (n < N) ? wC[n] : 0.0;
          if (n < N) sm = hyg_u128_add(sm, hyg_fix100(wn[i] * nv[i]));
        }
        const double mean = hyg_u128_to_f64(wave_sum128(sm), 100);
        bool ok = true;
        if (!final) {
          hyg_u128 sv = hyg_u128_zero();
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int n = lane + 64 * i;
            if (n < N) {
              const double dv = nv[i] - mean;
              sv = hyg_u128_add(sv, hyg_fix100(wn[i] * (dv * dv)));
            }
          }
          ok = hyg_u128_to_f64(wave_sum128(sv), 100) < eps;
        }
        if (lane == 0) {
          meanb[el * K + r] = mean;
          okb[el * K + r] = ok ? 1 : 0;
        }
      }
      __syncthreads();
      if (tid < ne) {
        const int e = c0 + tid;
        bool ok = true;
#pragma unroll
        for (int r = 0; r < K; ++r) ok = ok && okb[tid * K + r];
        const bool store = final || ok;
        if (store) {
          double* o = out + (size_t)timeA[e] * K;
#pragma unroll
          for (int r = 0; r < K; ++r) o[r] = meanb[tid * K + r];
        }
        keepf[e] = store ? 0 : 1;
      }
      __syncthreads();
    }
    // compaction of the pending list into the other buffer; freed slots go
    // back to the LDS mask or the workspace free list (order is immaterial)
    {
      int32_t* slotB = lists + (size_t)(cur ^ 1) * 2 * cap;
      int32_t* timeB = slotB + cap;
      int nk = 0, nf = sh.nfree;
      for (int b = 0; b < ntot; b += NB) {
        const int e = b + tid;
        const bool in = e < ntot;
        const int kp = in ? keepf[e] : 0;
        const int sl = in ? slotA[e] : 0;
        const int v = in ? (kp ? 1 : (sl >= nl ? 0x10000 : 0)) : 0;
        int tot;
        const int ex = block_excl_int<NB>(v, red, &tot);
        if (in) {
          if (kp) {
            const int p = nk + (ex & 0xffff);
            slotB[p] = sl;
            timeB[p] = timeA[e];
          } else if (sl >= nl) {
            freel[nf + (ex >> 16)] = sl - nl;
          } else {
            atomicOr(&sh.lmask, 1u << sl);
          }
        }
        nk += tot & 0xffff;
        nf += tot >> 16;
      }
      __syncthreads();
      if (tid == 0) {
        sh.npend = nk;
        sh.nfree = nf;
        sh.cur = cur ^ 1;
      }
      __syncthreads();
    }
  }
  if (tid == 0) {
    if (status != HYG_OK) sg_st4(ctl + 4, kSgTailAbort);  // the SMC workgroup must not wait for ring space
    status_out[chain] = status;
  }
}

// ------------------------------------------------------------- launches
// One launch per group of at most (resident workgroups / 2) chains, from the
// occupancy query: on an otherwise idle GPU every chain's SMC and smoothing
// workgroups are then resident together and nothing waits for a CU. The
// dispatch tickets (sg_chain_kernel) keep a crowded GPU correct too: a pair
// only waits for a CU to free up.
template <int KT, int NB, bool PE, bool PHS = false>
static void launch_chain_kt(const SgModelDev& md, const SgChainDev* chains_dev, int n_chains, const double* E,
                            uint8_t* ws, int cap, double* probs, int32_t* status, const SgLay& lay,
                            const SgCLay& clay, size_t lds, unsigned long long* dbg, hipStream_t s, const SgPeDev& pe,
                            hipError_t* err) {
  *err = hipFuncSetAttribute((const void*)sg_chain_kernel<KT, NB, PE, PHS>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (*err != hipSuccess) return;
  int dev = 0, cus = 0;
  if ((*err = hipGetDevice(&dev)) != hipSuccess) return;
  if ((*err = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return;
  int nb = 0;
  if ((*err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)sg_chain_kernel<KT, NB, PE, PHS>, NB,
                                                          lds)) != hipSuccess)
    return;
  const int per = nb * cus / 2 > 0 ? nb * cus / 2 : 1;
  for (int c0 = 0; c0 < n_chains; c0 += per) {
    const int nc = (n_chains - c0) < per ? (n_chains - c0) : per;
    hipLaunchKernelGGL((sg_chain_kernel<KT, NB, PE, PHS>), dim3(2 * nc), dim3(NB), lds, s, md, chains_dev + c0, nc, E,
                       ws, cap, probs, status + c0, lay, clay, dbg ? dbg + (size_t)kSgPh * c0 : nullptr, pe);
    if ((*err = hipGetLastError()) != hipSuccess) return;
  }
}
// ------------------------------------------------------------- launches
int sg_launch_emission(const SgModelDev& md, const hyg_sg_consts& c, const uint16_t* meth, const uint16_t* tot,
                       int S, int64_t n_sites, double* E, void* stream) {
  if (n_sites <= 0) return HYG_OK;
  int64_t blocks = (n_sites + 255) / 256;
  if (blocks > 256 * 16) blocks = 256 * 16;
  hipLaunchKernelGGL(sg_emission_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, md.lf, md.lg,
                     md.cst, md.nmax_reads + 1, c.K, meth, tot, S, n_sites, E);
  return hipGetLastError() == hipSuccess ? HYG_OK : HYG_EDEVICE;
}


// The packed sort keeps the top 64 - g_key_drop bits of a key (8 in production;
// tests drop more, so that keys collide and the exact re-sort runs often)
static int g_key_drop = 8;
int sg_force_key_drop(int bits) {
  if (bits != 0 && (bits < 8 || bits > 60)) return HYG_EINVAL;
  g_key_drop = bits ? bits : 8;
  return HYG_OK;
}

int sg_launch_chains(const SgModelDev& md_in, const hyg_sg_consts& c, const SgChainDev* chains_dev, int n_chains,
                     const double* E, uint8_t* ws, int psi_cap, double* probs, int32_t* status, void* ctl,
                     void* stream, const SgPeDev* pe) {
  if (n_chains <= 0) return HYG_OK;
  SgModelDev md = md_in;
  md.key_keep = ~((1ull << g_key_drop) - 1ull);
  if (c.Nmax > kSgThreads || c.K < 2 || c.K > HYG_KMAX) return HYG_EUNSUPPORTED;
  const SgLay lay = sg_layout(c.K, psi_cap, pe != nullptr);
  const SgCLay clay = sg_clayout(c.K, psi_cap);
  const size_t lds = sg_lds_bytes(c, psi_cap, pe != nullptr);
  SgPeDev ped{};
  if (pe) ped = *pe;
  if (lds > kSgLdsBudget) return HYG_EUNSUPPORTED;
  // phase timers: HYG_SG_PHASES=1, in the K = 6 instantiations (the pipeline's shape) only
  static const bool want_env = tuning_env("HYG_SG_PHASES") != nullptr;
  const bool want_dbg = want_env && c.K == 6;
  unsigned long long* dbg = nullptr;
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(ctl, 0, kSgCtlBytes * (size_t)n_chains, s) != hipSuccess) return HYG_EDEVICE;
  if (want_dbg && hipMalloc((void**)&dbg, sizeof(unsigned long long) * kSgPh * n_chains) != hipSuccess) dbg = nullptr;
  if (dbg) (void)hipMemsetAsync(dbg, 0, sizeof(unsigned long long) * kSgPh * n_chains, s);
  hipError_t err = hipErrorInvalidValue;
  switch (c.K) {
#define SG_CASE(k)                                                                                               \
  case k:                                                                                                        \
    if (k == 6 && dbg) {                                                                                         \
      if (pe)                                                                                                    \
        launch_chain_kt<6, 512, true, true>(md, chains_dev, n_chains, E, ws, psi_cap, probs, status, lay, clay,   \
                                            lds, dbg, s, ped, &err);                                             \
      else                                                                                                       \
        launch_chain_kt<6, 512, false, true>(md, chains_dev, n_chains, E, ws, psi_cap, probs, status, lay, clay,  \
                                             lds, dbg, s, ped, &err);                                            \
    } else if (pe)                                                                                               \
      launch_chain_kt<k, (k <= 8 ? 512 : 256), true>(md, chains_dev, n_chains, E, ws, psi_cap, probs, status, lay, \
                                                     clay, lds, dbg, s, ped, &err);                              \
    else                                                                                                         \
      launch_chain_kt<k, (k <= 8 ? 512 : 256), false>(md, chains_dev, n_chains, E, ws, psi_cap, probs, status,     \
                                                      lay, clay, lds, dbg, s, ped, &err);                        \
    break;
    SG_CASE(2) SG_CASE(3) SG_CASE(4) SG_CASE(5) SG_CASE(6) SG_CASE(7) SG_CASE(8) SG_CASE(9)
    SG_CASE(10) SG_CASE(11) SG_CASE(12) SG_CASE(13) SG_CASE(14) SG_CASE(15) SG_CASE(16)
#undef SG_CASE
    default: break;
  }
  if (err != hipSuccess) {
    if (dbg) (void)hipFree(dbg);
    return HYG_EDEVICE;
  }
  if (dbg) {
    std::vector<unsigned long long> h((size_t)kSgPh * n_chains);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), dbg, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost);
    (void)hipFree(dbg);
    // the longest chain (the critical path)
    int lc = 0;
    for (int i = 1; i < n_chains; ++i)
      if (h[(size_t)i * kSgPh + kSgPh - 1] > h[(size_t)lc * kSgPh + kSgPh - 1]) lc = i;
    const unsigned long long* hl = h.data() + (size_t)lc * kSgPh;
    const double steps = (double)hl[kSgPh - 1];
    auto v = [&](int k) { return (double)hl[k] / steps; };
    fprintf(stderr, "[hyg sg phases] K=%d lds=%zu smoothing slots_lds=%d longest chain %d: %.0f steps, cycles/step:",
            c.K, lds, clay.nl, lc, steps);
    double sum = 0;
    if (!pe) {
      const char* nm[22] = {"copy", "sort", "kloop", "resample", "weights.tail", "normalise.tail", "record",
                            "weights.amax", "-", "-", "-", "weights.limbsG", "bitonic", "gather+mono", "log+scan",
                            "-", "weights.bar1", "weights.bar2", "weights.S", "weights.bar3", "normalise.drain",
                            "normalise.sum"};
      for (int k = 0; k < 22; ++k) {
        if (nm[k][0] == '-') continue;
        fprintf(stderr, " %s=%.0f", nm[k], v(k));
        sum += v(k);
      }
    } else {
      const char* nm[7] = {"copy", "sort", "kloop", "resample", "weights", "normalise", "record"};
      for (int k = 0; k < 7; ++k) {
        fprintf(stderr, " %s=%.0f", nm[k], v(k));
        sum += v(k);
      }
      fprintf(stderr, " estimation=%.0f rebuild=%.0f (rows/rebuild %.0f)", v(12), v(13),
              (double)hl[14] / std::max(1.0, steps / (double)pe->c.every));
      sum += v(12) + v(13);
    }
    fprintf(stderr, " total=%.0f | optimal=%.0f keep_top=%.0f kloop_iters/capped=%.2f keep_top_resorts=%.0f\n", sum,
            (double)hl[8], (double)hl[9], (double)hl[10] / std::max(1.0, (double)(hl[8] + hl[9])), (double)hl[22]);
  }
  return HYG_OK;
}

}  // namespace hyg
