// tg_kernels.hip -- CDNA4 (gfx950) kernels of the two-group change-point path.
//
//   tg_emission_kernel  per-site Beta-Binomial emission table (HBM streaming)
//   tg_forward_kernel   particle filter with optimal finite-state resampling,
//                       one 256-thread workgroup per chain, persistent over T
//   tg_backward_kernel  backward simulation of B trajectories, one workgroup
//                       per chain, regenerating each step's particles from the
//                       forward's ancestor history
//
// Every index decision uses the arithmetic contract of include/hyg_arith.h
// (exact integer mass sums, deterministic exp/log, Philox streams), so the
// results are bit-identical to the CPU oracle (oracle/tg_oracle.c) whatever
// the reduction tree; that freedom is what the kernels use to parallelise.
// Reference semantics: see the oracle header and DESIGN.md.
#include <hip/hip_runtime.h>

#include "../../include/hyg_arith.h"
#include "tg_common.h"

namespace hyg {

enum { MODE_KEEP = 0, MODE_OPTIMAL = 1, MODE_UNBIASED = 2, MODE_INIT = 3 };

// ----------------------------------------------------------- small helpers
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

__device__ __forceinline__ unsigned long long shx(unsigned long long v, int o) { return __shfl_xor(v, o); }
__device__ __forceinline__ unsigned long long shu(unsigned long long v, int o) { return __shfl_up(v, o); }

__device__ __forceinline__ double wave_max(double v) {
  for (int o = 32; o > 0; o >>= 1) {
    const double w = __shfl_xor(v, o);
    v = (w > v) ? w : v;
  }
  return v;
}
__device__ __forceinline__ int wave_sum(int v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ hyg_u128 wave_sum128(hyg_u128 v) {
  for (int o = 32; o > 0; o >>= 1) {
    hyg_u128 w;
    w.lo = shx(v.lo, o);
    w.hi = shx(v.hi, o);
    v = hyg_u128_add(v, w);
  }
  return v;
}

// Block-wide reductions (4 waves). `red` is a 128-byte LDS scratch; every call
// begins with a barrier so back-to-back calls may reuse it.
__device__ __forceinline__ double block_max(double v, unsigned char* red) {
  double* r = (double*)red;
  v = wave_max(v);
  __syncthreads();
  if (lane_id() == 0) r[wave_id()] = v;
  __syncthreads();
  double m = r[0];
  for (int w = 1; w < kThreads / 64; ++w) m = (r[w] > m) ? r[w] : m;
  return m;
}
__device__ __forceinline__ int block_sum(int v, unsigned char* red) {
  int* r = (int*)red;
  v = wave_sum(v);
  __syncthreads();
  if (lane_id() == 0) r[wave_id()] = v;
  __syncthreads();
  int s = 0;
  for (int w = 0; w < kThreads / 64; ++w) s += r[w];
  return s;
}
__device__ __forceinline__ hyg_u128 block_sum128(hyg_u128 v, unsigned char* red) {
  hyg_u128* r = (hyg_u128*)red;
  v = wave_sum128(v);
  __syncthreads();
  if (lane_id() == 0) r[wave_id()] = v;
  __syncthreads();
  hyg_u128 s = hyg_u128_zero();
  for (int w = 0; w < kThreads / 64; ++w) s = hyg_u128_add(s, r[w]);
  return s;
}

// Exclusive block scans; out[tid] = exclusive prefix, out[kThreads] = total.
__device__ __forceinline__ void block_scan192(hyg_u192 v, hyg_u192* out, unsigned char* red) {
  hyg_u192* r = (hyg_u192*)red;
  hyg_u192 inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    hyg_u192 n;
    n.w0 = shu(inc.w0, o);
    n.w1 = shu(inc.w1, o);
    n.w2 = shu(inc.w2, o);
    if (lane_id() >= o) inc = hyg_u192_add(inc, n);
  }
  __syncthreads();
  if (lane_id() == 63) r[wave_id()] = inc;
  __syncthreads();
  hyg_u192 pre = hyg_u192_zero(), tot = hyg_u192_zero();
  for (int w = 0; w < kThreads / 64; ++w) {
    if (w < wave_id()) pre = hyg_u192_add(pre, r[w]);
    tot = hyg_u192_add(tot, r[w]);
  }
  out[threadIdx.x] = hyg_u192_add(pre, hyg_u192_sub(inc, v));
  if (threadIdx.x == 0) out[kThreads] = tot;
}
__device__ __forceinline__ void block_scan128(hyg_u128 v, hyg_u128* out, unsigned char* red) {
  hyg_u128* r = (hyg_u128*)red;
  hyg_u128 inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    hyg_u128 n;
    n.lo = shu(inc.lo, o);
    n.hi = shu(inc.hi, o);
    if (lane_id() >= o) inc = hyg_u128_add(inc, n);
  }
  __syncthreads();
  if (lane_id() == 63) r[wave_id()] = inc;
  __syncthreads();
  hyg_u128 pre = hyg_u128_zero(), tot = hyg_u128_zero();
  for (int w = 0; w < kThreads / 64; ++w) {
    if (w < wave_id()) pre = hyg_u128_add(pre, r[w]);
    tot = hyg_u128_add(tot, r[w]);
  }
  // exclusive = inclusive - v, computed without a 128-bit subtract
  hyg_u128 ex = pre;
  {
    hyg_u128 e2;  // inc - v
    e2.lo = inc.lo - v.lo;
    e2.hi = inc.hi - v.hi - (inc.lo < v.lo ? 1u : 0u);
    ex = hyg_u128_add(ex, e2);
  }
  out[threadIdx.x] = ex;
  if (threadIdx.x == 0) out[kThreads] = tot;
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

// --------------------------------------------------------------- model
struct Hz4 {
  double lrc, l1c, lrk, l1k;  // log rho / log(1-rho), control (d_c, r_c) and case (d_k, r_k)
};

__device__ __forceinline__ double2 hz_at(const ModelDev& md, int K, int g, int r, int d) {
  d = d < 0 ? 0 : (d >= md.dcap ? md.dcap - 1 : d);
  return *(const double2*)(md.hz + ((size_t)(g * K + r) * md.dcap + d) * 2);
}
__device__ __forceinline__ Hz4 hz_of(const ModelDev& md, int K, uint64_t s) {
  const double2 a = hz_at(md, K, 0, hyg_st_rc(s), hyg_st_dc(s));
  const double2 b = hz_at(md, K, 1, hyg_st_rk(s), hyg_st_dk(s));
  Hz4 h;
  h.lrc = a.x; h.l1c = a.y; h.lrk = b.x; h.l1k = b.y;
  return h;
}

// log f_t(next | prev), t >= 1 (case_control_regime_model.py:80-193,
// case_control_distributions.py:138-151, 246-291); h = hazard of prev.
// Same branch structure and addition order as oracle/tg_oracle.c:tg_trans.
__device__ __forceinline__ double tg_trans(const hyg_tg_consts* __restrict__ c, int K, uint64_t prev, uint64_t next,
                                           const Hz4& h) {
  const double NINF = HYG_NINF;
  const int m = hyg_st_m(prev), dc = hyg_st_dc(prev), rc = hyg_st_rc(prev), dk = hyg_st_dk(prev),
            rk = hyg_st_rk(prev);
  const int m2 = hyg_st_m(next), dc2 = hyg_st_dc(next), rc2 = hyg_st_rc(next), dk2 = hyg_st_dk(next),
            rk2 = hyg_st_rk(next);
  double lm;
  if ((dk < dc ? dk : dc) >= c->u) lm = c->lPm[m * 2 + m2];
  else lm = (m2 == m) ? 0.0 : NINF;
  double lc;
  if (dc2 == 1) lc = h.lrc + c->lPc[rc * K + rc2];
  else lc = (dc2 == dc + 1 && rc2 == rc) ? h.l1c : NINF;
  double lk;
  if (m2 == 1) {
    lk = (rk2 == rc2 && dk2 == dc2) ? 0.0 : NINF;
  } else if (m == 1 && dc2 != 1) {
    lk = (dk2 == 1 && rk2 != rc2) ? c->lU1 : NINF;
  } else if (rc2 == rk && m == 0) {
    lk = (dk2 == 1 && rk2 != rc2) ? c->lU1 : NINF;
  } else {
    if (dk2 == 1) lk = (rk2 != rc2 && rk2 != rk) ? h.lrk + ((rc2 == rk) ? c->lU1 : c->lU2) : NINF;
    else lk = (dk2 == dk + 1 && rk2 == rk) ? h.l1k : NINF;
  }
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

// ----------------------------------------------------------- LDS layout
struct Shared {  // broadcast scalars of one workgroup
  double mx, logS, lse;
  float c_new, log_c, U;
  int cnt, n_sig, np, mode, Kk, status, r_ph;
  unsigned sig_ctr;
  hyg_u192 preK, R;
  int ng;
};

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
__host__ __device__ inline int next_pow2(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

struct Lay {  // byte offsets into the dynamic LDS
  size_t W, L, keys, mass, pst, pw, phz, ering, cp, parents, sysp, X, grp, gst, red, sh, total;
  int npad, nsort;
};

__host__ __device__ inline Lay make_layout(int K, int M, int B, int Nmax, bool backward) {
  Lay l{};
  l.npad = (int)align_up((size_t)Nmax, kThreads);
  l.nsort = next_pow2(Nmax < 64 ? 64 : Nmax);
  size_t o = 0;
  l.W = o; o = align_up(o + sizeof(double) * l.npad, 16);
  if (backward) { l.L = o; o = align_up(o + sizeof(double) * l.npad, 16); }
  if (!backward) {
    l.keys = o; o = align_up(o + sizeof(uint64_t) * l.nsort, 16);
    l.mass = o; o = align_up(o + sizeof(float) * l.npad, 16);
  }
  l.pst = o; o = align_up(o + sizeof(uint64_t) * 2 * M, 16);
  l.pw = o; o = align_up(o + sizeof(double) * 2 * M, 16);
  l.phz = o; o = align_up(o + sizeof(double) * 4 * M, 16);
  l.ering = o; o = align_up(o + sizeof(double) * kEBlock * 2 * K, 16);
  l.cp = o; o = align_up(o + sizeof(hyg_u192) * (kThreads + 1), 16);
  l.parents = o; o = align_up(o + sizeof(int) * (M > B ? M : B), 16);
  l.sysp = o; o = align_up(o + sizeof(int) * M, 16);
  l.X = o; o = align_up(o + sizeof(uint64_t) * B, 16);
  l.grp = o; o = align_up(o + sizeof(int) * B, 16);
  l.gst = o; o = align_up(o + sizeof(uint64_t) * B, 16);
  l.red = o; o = align_up(o + 128, 16);
  l.sh = o; o = align_up(o + sizeof(Shared), 16);
  l.total = o;
  return l;
}

// ---------------------------------------------------------- shared steps
// Stage emission rows [bi*EB, min(bi*EB+EB, T)) of the chain into the ring.
__device__ __forceinline__ void load_eblock(double* ering, const double* __restrict__ Ech, int bi, int T, int K2) {
  const int t0 = bi * kEBlock;
  const int rows = (T - t0) < kEBlock ? (T - t0) : kEBlock;
  const int n = rows * K2;
  for (int i = threadIdx.x; i < n; i += kThreads) ering[i] = Ech[(size_t)t0 * K2 + i];
}

// Weights of the particles of step t >= 1 from the record (pst, pw, phz and
// the step scalars); _filter_one_step :235-270 and expand_collapsed_results.
__device__ __forceinline__ void gen_weights(const hyg_tg_consts* __restrict__ c, int K, int I, int np, int mode,
                                            float log_c, double lse, const uint64_t* pst, const double* pw,
                                            const double* phz, const double* Et, double* W) {
  const int N = I * np;
  for (int n = threadIdx.x; n < N; n += kThreads) {
    const int s = n / np, a = n - s * np;
    const uint64_t par = pst[a];
    const uint64_t x = tg_xi(K, par, s);
    Hz4 h;
    h.lrc = phz[4 * a + 0]; h.l1c = phz[4 * a + 1]; h.lrk = phz[4 * a + 2]; h.l1k = phz[4 * a + 3];
    const double tr = tg_trans(c, K, par, x, h);
    double w;
    if (!hyg_isfinite(tr)) {
      w = HYG_NINF;
    } else {
      const double lg = tr + (Et[hyg_st_rc(x)] + Et[K + hyg_st_rk(x)]);
      if (mode == MODE_KEEP) {
        w = pw[a] + lg;
      } else if (mode == MODE_UNBIASED) {
        w = (-c->log_M + lse) + lg;
      } else {
        const double v = (double)log_c + (pw[a] - lse);
        w = (pw[a] + lg) - (v < 0.0 ? v : 0.0);
      }
    }
    W[n] = w;
  }
}
__device__ __forceinline__ void gen_weights_init(const hyg_tg_consts* __restrict__ c, int K, int r_ph,
                                                 const double* Et, double* W) {
  for (int n = threadIdx.x; n < K * K; n += kThreads) {
    const int i = n / K, j = n - (n / K) * K;
    const double obs = Et[i] + Et[K + j];
    const double tr = (i == j) ? c->lPc[r_ph * K + i] : HYG_NINF;
    W[n] = obs + tr;
  }
}

// max and log of the exact mass sum of W[0..N): tf.reduce_logsumexp /
// tf.nn.log_softmax with the F=100 fixed-point sum of hyg_arith.h.
__device__ __forceinline__ void lse_block(const double* W, int N, unsigned char* red, double* mx_out,
                                          double* logS_out, int* cnt_out) {
  double m = HYG_NINF;
  int cnt = 0;
  for (int n = threadIdx.x; n < N; n += kThreads) {
    const double w = W[n];
    m = (w > m) ? w : m;
    cnt += (w > HYG_NINF) ? 1 : 0;
  }
  const double mx = block_max(m, red);
  const int tot = block_sum(cnt, red);
  hyg_u128 s = hyg_u128_zero();
  if (mx > HYG_NINF) {
    for (int n = threadIdx.x; n < N; n += kThreads) {
      const double x = W[n] - mx;
      if (x >= -70.0) s = hyg_u128_add(s, hyg_fix100(hyg_exp(x)));  // exp(x < -70) < 2^-100 -> 0
    }
  }
  const hyg_u128 S = block_sum128(s, red);
  *mx_out = mx;
  *logS_out = hyg_log(hyg_u128_to_f64(S, 100));
  *cnt_out = tot;
}

// Categorical draws (tfd.Categorical(logits).sample, TF multinomial CDF
// semantics): for each draw q in [0, n_draw) with random bits rnd(q), the
// first n with cdf_n > floor(u * total). logits(n) is recomputed on demand.
template <typename LogitFn, typename ActiveFn, typename RandFn, typename OutFn>
__device__ __forceinline__ void categorical_block(int N, double lmax, LogitFn logit, int n_draw, ActiveFn active,
                                                  RandFn rnd, OutFn out, hyg_u128* cp, unsigned char* red) {
  const int cs = (N + kThreads - 1) / kThreads;
  const int p0 = threadIdx.x * cs, p1 = (p0 + cs < N) ? p0 + cs : N;
  hyg_u128 loc = hyg_u128_zero();
  for (int n = p0; n < p1; ++n) {
    const double x = logit(n) - lmax;
    if (x >= -70.0) loc = hyg_u128_add(loc, hyg_fix100(hyg_exp(x)));
  }
  block_scan128(loc, cp, red);
  __syncthreads();
  const hyg_u128 total = cp[kThreads];
  for (int q = threadIdx.x; q < n_draw; q += kThreads) {
    if (!active(q)) continue;
    const hyg_u128 target = hyg_scale_target(rnd(q), total);
    // chunk: last ch with cp[ch] <= target (cp is the exclusive prefix)
    int lo = 0, hi = kThreads - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (hyg_u128_lt(target, cp[mid])) hi = mid - 1; else lo = mid;
    }
    // skip empty chunks whose prefix equals the target (first n with cdf > target)
    int ch = lo;
    hyg_u128 cdf = cp[ch];
    int sel = -1;
    for (; ch < kThreads && sel < 0; ++ch) {
      cdf = cp[ch];
      const int a0 = ch * cs, a1 = (a0 + cs < N) ? a0 + cs : N;
      for (int n = a0; n < a1; ++n) {
        const double x = logit(n) - lmax;
        if (x >= -70.0) cdf = hyg_u128_add(cdf, hyg_fix100(hyg_exp(x)));
        if (hyg_u128_lt(target, cdf)) { sel = n; break; }
      }
    }
    out(q, sel < 0 ? N - 1 : sel);
  }
}

// --------------------------------------------------------------- kernels
__global__ void __launch_bounds__(kThreads)
tg_emission_kernel(const double* __restrict__ lf, const double* __restrict__ lg, const double* __restrict__ cst,
                   int L, int K, const uint16_t* __restrict__ meth_c, const uint16_t* __restrict__ tot_c, int s_c,
                   const uint16_t* __restrict__ meth_k, const uint16_t* __restrict__ tot_k, int s_k, int64_t T,
                   double* __restrict__ E) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < T; t += (int64_t)gridDim.x * blockDim.x) {
    for (int g = 0; g < 2; ++g) {
      const int S = g ? s_k : s_c;
      const uint16_t* my = g ? meth_k + t * s_k : meth_c + t * s_c;
      const uint16_t* nt = g ? tot_k + t * s_k : tot_c + t * s_c;
      double e[HYG_KMAX];
      for (int r = 0; r < K; ++r) e[r] = 0.0;
      for (int s = 0; s < S; ++s) {
        int n = nt[s], y = my[s];
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
      for (int r = 0; r < K; ++r) E[t * 2 * K + g * K + r] = e[r];
    }
  }
}

__global__ void __launch_bounds__(kThreads)
tg_forward_kernel(ModelDev md, const ChainDev* __restrict__ chains, const double* __restrict__ E,
                  uint8_t* __restrict__ ws, int32_t* status_out, double* __restrict__ logz_out,
                  double* __restrict__ finalw_out, Lay lay) {
  const hyg_tg_consts* __restrict__ c = md.consts;
  const int K = c->K, M = c->M, I = c->I, K2 = 2 * K, tid = threadIdx.x;
  const ChainDev ch = chains[blockIdx.x];
  const int T = ch.T;
  extern __shared__ __align__(16) unsigned char smem[];
  double* W = (double*)(smem + lay.W);
  uint64_t* keys = (uint64_t*)(smem + lay.keys);
  float* mass = (float*)(smem + lay.mass);
  uint64_t* pst = (uint64_t*)(smem + lay.pst);
  double* pw = (double*)(smem + lay.pw);
  double* phz = (double*)(smem + lay.phz);
  double* ering = (double*)(smem + lay.ering);
  hyg_u192* cp = (hyg_u192*)(smem + lay.cp);
  hyg_u128* cp128 = (hyg_u128*)(smem + lay.cp);
  int* parents = (int*)(smem + lay.parents);
  int* sysp = (int*)(smem + lay.sysp);
  unsigned char* red = smem + lay.red;
  Shared& sh = *(Shared*)(smem + lay.sh);

  uint8_t* rec0 = ws + ch.ws_offset;
  const size_t rstride = record_bytes(M);
  const double* Ech = E + ch.site_begin * K2;

  // ---- t = 0 (_filter_first_step)
  load_eblock(ering, Ech, 0, T, K2);
  if (tid == 0) {
    sh.r_ph = (int)hyg_mulhi64(hyg_rand64(ch.seed, ch.chain_id, HYG_RNG_PHANTOM, 0, 0), (uint64_t)K);
    sh.status = HYG_OK;
    StepScalars* s0 = (StepScalars*)rec0;
    s0->mode = MODE_INIT; s0->n_par = 0; s0->log_c = 0.0f; s0->r_ph = sh.r_ph; s0->lse = 0.0; s0->pad = 0.0;
  }
  __syncthreads();
  gen_weights_init(c, K, sh.r_ph, ering, W);
  int N = K * K, np_prev = 0, prev_mode = MODE_INIT, cur = 0;
  __syncthreads();

  for (int t = 1; t < T; ++t) {
    if ((t % kEBlock) == 0) load_eblock(ering, Ech, t / kEBlock, T, K2);  // read after later barriers
    // ---- weights of step t-1: max, count, log-sum-exp
    double mx, logS;
    int cnt;
    lse_block(W, N, red, &mx, &logS, &cnt);
    if (!(mx > HYG_NINF)) {
      if (tid == 0) sh.status = HYG_ENUMERIC;
      break;  // uniform
    }
    const double lse = logS + mx;
    int mode, np;
    float log_c = 0.0f;
    if (cnt <= M) {
      // ---- keep every particle with non-zero weight, in index order
      mode = MODE_KEEP;
      np = cnt;
      const int cs = (N + kThreads - 1) / kThreads;
      const int p0 = tid * cs, p1 = (p0 + cs < N) ? p0 + cs : N;
      int loc = 0;
      for (int n = p0; n < p1; ++n) loc += (W[n] > HYG_NINF);
      // exclusive scan of counts via the u128 scan (values are small)
      hyg_u128 v; v.lo = (uint64_t)loc; v.hi = 0;
      block_scan128(v, cp128, red);
      __syncthreads();
      int o = (int)cp128[tid].lo;
      for (int n = p0; n < p1; ++n)
        if (W[n] > HYG_NINF) parents[o++] = n;
    } else {
      // ---- OptimalFiniteState (resampling_functions.py:7-52)
      if (tid == 0) sh.sig_ctr = 0;
      __syncthreads();
      const float thr = c->sig_thresh;
      const int iters = (N + kThreads - 1) / kThreads;
      for (int it = 0; it < iters; ++it) {
        const int n = it * kThreads + tid;
        bool sig = false;
        uint64_t key = 0;
        if (n < N) {
          const double w = W[n];
          if (w > HYG_NINF) {
            const float lw = (float)((w - mx) - logS);
            if (lw >= thr) { sig = true; key = sort_key(lw, n); }
          }
        }
        const unsigned long long mask = __ballot(sig);
        const int pc = __popcll(mask);
        unsigned base = 0;
        if (lane_id() == 0 && pc) base = atomicAdd(&sh.sig_ctr, (unsigned)pc);
        base = __shfl(base, 0);
        if (sig) keys[base + __popcll(mask & ((1ull << lane_id()) - 1ull))] = key;
      }
      __syncthreads();
      const int n_sig = (int)sh.sig_ctr;
      const int n2 = next_pow2(n_sig < 64 ? 64 : n_sig);
      for (int i = n_sig + tid; i < n2; i += kThreads) keys[i] = ~0ull;
      __syncthreads();
      // bitonic sort of keys[0, n2)
      for (int k = 2; k <= n2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int i = tid; i < (n2 >> 1); i += kThreads) {
            const int lo = 2 * j * (i / j) + (i % j);
            const int hi = lo + j;
            const uint64_t a = keys[lo], b = keys[hi];
            const bool up = (lo & k) == 0;
            if ((a > b) == up) { keys[lo] = b; keys[hi] = a; }
          }
          __syncthreads();
        }
      }
      // masses and exact chunk prefix sums over the sorted significant set
      const int cs = (n_sig + kThreads - 1) / kThreads;
      {
        const int p0 = tid * cs, p1 = (p0 + cs < n_sig) ? p0 + cs : n_sig;
        hyg_u192 loc = hyg_u192_zero();
        for (int p = p0; p < p1; ++p) {
          const float m = hyg_expf(key_value(keys[p]));
          mass[p] = m;
          loc = hyg_u192_add(loc, hyg_fix149f(m));
        }
        block_scan192(loc, cp, red);
      }
      __syncthreads();
      const hyg_u192 total = cp[kThreads];
      // iterative K / log c with the TF loop-variable semantics
      int a = 0, b = -1;
      float lc = -1.0f;
      while (a != b && a < N && a < M) {
        if (tid == 0) {
          hyg_u192 rv = hyg_u192_zero();
          if (a < n_sig) {
            const int chk = a / cs;
            hyg_u192 pre = cp[chk];
            for (int p = chk * cs; p < a; ++p) pre = hyg_u192_add(pre, hyg_fix149f(mass[p]));
            rv = hyg_u192_sub(total, pre);
          }
          const double rvd = hyg_u192_to_f64(rv);
          const float l1 = hyg_logf((float)(M - a));
          const float l2 = (rvd == 0.0) ? HYG_NINFF : (float)hyg_log(rvd);
          sh.c_new = l1 - l2;
        }
        __syncthreads();
        const float cn = sh.c_new;
        int loc = 0;
        if (hyg_isfinitef(cn)) {
          const int p0 = tid * cs, p1 = (p0 + cs < n_sig) ? p0 + cs : n_sig;
          for (int p = (p0 > a ? p0 : a); p < p1; ++p) loc += ((float)(cn + key_value(keys[p])) > 0.0f) ? 1 : 0;
        } else if (tid == 0 && cn > 0.0f) {
          loc = (cnt - a) > 0 ? cnt - a : 0;  // +inf: every finite particle at position >= a
        }
        const int tot = block_sum(loc, red);
        b = a;
        a = a + tot;
        lc = cn;
      }
      int Kk = b;
      log_c = lc;
      if (Kk >= N) { Kk = N; log_c = HYG_NINFF; }
      if (!hyg_isfinitef(log_c)) {
        // ---- unbiased fallback: M categorical draws from log_weights (:42-47)
        mode = MODE_UNBIASED;
        np = M;
        log_c = 0.0f;
        const double lmax = (double)key_value(keys[0]);
        auto logit = [&](int n) -> double {
          const double w = W[n];
          return (w > HYG_NINF) ? (double)(float)((w - mx) - logS) : HYG_NINF;
        };
        auto rnd = [&](int q) -> uint64_t {
          return hyg_rand64(ch.seed, ch.chain_id, HYG_RNG_MULTINOMIAL, (uint64_t)t, (uint64_t)q);
        };
        auto out = [&](int q, int n) { parents[q] = n; };
        auto all = [](int) { return true; };
        __syncthreads();
        categorical_block(N, lmax, logit, M, all, rnd, out, cp128, red);
      } else {
        // ---- deterministic top-K plus systematic residual (:32-40, :56-69)
        mode = MODE_OPTIMAL;
        np = M;
        const int L = M - Kk;
        if (tid == 0) {
          hyg_u192 pre = hyg_u192_zero();
          if (Kk < n_sig) {
            const int chk = Kk / cs;
            pre = cp[chk];
            for (int p = chk * cs; p < Kk; ++p) pre = hyg_u192_add(pre, hyg_fix149f(mass[p]));
          } else {
            pre = total;
          }
          sh.preK = pre;
          sh.R = hyg_u192_sub(total, pre);
        }
        for (int p = tid; p < Kk; p += kThreads) parents[p] = key_index(keys[p]);
        for (int j = tid; j < L; j += kThreads) sysp[j] = Kk;
        __syncthreads();
        const double Rd = hyg_u192_to_f64(sh.R);
        const float U = hyg_u01f(hyg_rand64(ch.seed, ch.chain_id, HYG_RNG_SYSTEMATIC, (uint64_t)t, 0));
        const float Lf = (float)L;
        const int p0 = tid * cs, p1 = (p0 + cs < n_sig) ? p0 + cs : n_sig;
        const int lo = (p0 > Kk) ? p0 : Kk;
        if (lo < p1 && L > 0) {
          hyg_u192 C = hyg_u192_zero();
          int j = 0;
          if (p0 > Kk) {
            C = hyg_u192_sub(cp[tid], sh.preK);
            const double Qprev = hyg_u192_to_f64(C) / Rd;
            while (j < L && (double)(((float)j + U) / Lf) <= Qprev) ++j;
          }
          for (int p = lo; p < p1 && j < L; ++p) {
            C = hyg_u192_add(C, hyg_fix149f(mass[p]));
            const double Q = hyg_u192_to_f64(C) / Rd;
            while (j < L && (double)(((float)j + U) / Lf) <= Q) { sysp[j] = p; ++j; }
          }
        }
        __syncthreads();
        for (int j = tid; j < L; j += kThreads) parents[Kk + j] = key_index(keys[sysp[j]]);
      }
    }
    __syncthreads();
    // ---- gather the ancestors (states, weights, hazards) and record them
    {
      const int nxt = cur ^ 1;
      StepScalars* rs = (StepScalars*)(rec0 + (size_t)t * rstride);
      uint64_t* rst = (uint64_t*)(rs + 1);
      double* rw = (double*)(rst + M);
      for (int a = tid; a < np; a += kThreads) {
        const int n = parents[a];
        uint64_t s;
        if (prev_mode == MODE_INIT) {
          s = init_state(K, n);
        } else {
          const int sl = n / np_prev;
          s = tg_xi(K, pst[cur * M + (n - sl * np_prev)], sl);
        }
        const double w = W[n];
        pst[nxt * M + a] = s;
        pw[nxt * M + a] = w;
        rst[a] = s;
        rw[a] = w;
        const Hz4 h = hz_of(md, K, s);
        phz[4 * a + 0] = h.lrc; phz[4 * a + 1] = h.l1c; phz[4 * a + 2] = h.lrk; phz[4 * a + 3] = h.l1k;
      }
      if (tid == 0) {
        rs->mode = mode; rs->n_par = np; rs->log_c = log_c; rs->r_ph = 0; rs->lse = lse; rs->pad = 0.0;
      }
      cur = nxt;
      np_prev = np;
      prev_mode = mode;
    }
    __syncthreads();
    // ---- propose and weight the particles of step t
    gen_weights(c, K, I, np, mode, log_c, lse, pst + cur * M, pw + cur * M, phz, ering + (t % kEBlock) * K2, W);
    N = I * np;
    __syncthreads();
  }
  // ---- final weights: log normalising constant and run()'s second output
  double mx, logS;
  int cnt;
  lse_block(W, N, red, &mx, &logS, &cnt);
  if (tid == 0) {
    int st = sh.status;
    if (st == HYG_OK && !(mx > HYG_NINF)) st = HYG_ENUMERIC;
    status_out[blockIdx.x] = st;
    logz_out[blockIdx.x] = logS + mx;
    // the last record's scalars carry N_{T-1} for the backward pass
  }
  if (finalw_out) {
    const int Nmax = c->Nmax;
    for (int n = tid; n < Nmax; n += kThreads)
      finalw_out[(size_t)blockIdx.x * Nmax + n] = (n < N) ? W[n] : HYG_NINF;
  }
}

__global__ void __launch_bounds__(kThreads)
tg_backward_kernel(ModelDev md, const ChainDev* __restrict__ chains, const double* __restrict__ E,
                   const uint8_t* __restrict__ ws, const int32_t* status_in, int16_t* __restrict__ o_merged,
                   int16_t* __restrict__ o_control, int16_t* __restrict__ o_case, float* __restrict__ o_split,
                   float* __restrict__ o_regime, int32_t* status_out, Lay lay) {
  const hyg_tg_consts* __restrict__ c = md.consts;
  const int K = c->K, M = c->M, B = c->B, I = c->I, K2 = 2 * K, tid = threadIdx.x;
  const ChainDev ch = chains[blockIdx.x];
  const int T = ch.T;
  if (status_in[blockIdx.x] != HYG_OK) return;  // uniform
  extern __shared__ __align__(16) unsigned char smem[];
  double* W = (double*)(smem + lay.W);
  double* Lg = (double*)(smem + lay.L);
  uint64_t* pst = (uint64_t*)(smem + lay.pst);
  double* pw = (double*)(smem + lay.pw);
  double* phz = (double*)(smem + lay.phz);
  double* ering = (double*)(smem + lay.ering);
  hyg_u128* cp128 = (hyg_u128*)(smem + lay.cp);
  int* idx = (int*)(smem + lay.parents);
  uint64_t* X = (uint64_t*)(smem + lay.X);
  int* grp = (int*)(smem + lay.grp);
  uint64_t* gst = (uint64_t*)(smem + lay.gst);
  unsigned char* red = smem + lay.red;
  Shared& sh = *(Shared*)(smem + lay.sh);

  const uint8_t* rec0 = ws + ch.ws_offset;
  const size_t rstride = record_bytes(M);
  const double* Ech = E + ch.site_begin * K2;
  if (tid == 0) sh.status = HYG_OK;

  for (int t = T - 1; t >= 0; --t) {
    if (t == T - 1 || (t % kEBlock) == kEBlock - 1) {
      __syncthreads();
      load_eblock(ering, Ech, t / kEBlock, T, K2);
    }
    // ---- regenerate the particles of step t from its record
    const StepScalars* rs = (const StepScalars*)(rec0 + (size_t)t * rstride);
    const StepScalars s = *rs;
    const uint64_t* rst = (const uint64_t*)(rs + 1);
    const double* rw = (const double*)(rst + M);
    __syncthreads();
    for (int a = tid; a < s.n_par; a += kThreads) {
      const uint64_t st = rst[a];
      pst[a] = st;
      pw[a] = rw[a];
      const Hz4 h = hz_of(md, K, st);
      phz[4 * a + 0] = h.lrc; phz[4 * a + 1] = h.l1c; phz[4 * a + 2] = h.lrk; phz[4 * a + 3] = h.l1k;
    }
    __syncthreads();
    const double* Et = ering + (t % kEBlock) * K2;
    int N;
    if (s.mode == MODE_INIT) {
      gen_weights_init(c, K, s.r_ph, Et, W);
      N = K * K;
    } else {
      gen_weights(c, K, I, s.n_par, s.mode, s.log_c, s.lse, pst, pw, phz, Et, W);
      N = I * s.n_par;
    }
    __syncthreads();
    const int np = s.n_par;
    auto state_of = [&](int n) -> uint64_t {
      if (s.mode == MODE_INIT) return init_state(K, n);
      const int sl = n / np;
      return tg_xi(K, pst[n - sl * np], sl);
    };
    if (t == T - 1) {
      // ---- B draws from the final weights (:383-385)
      double m = HYG_NINF;
      for (int n = tid; n < N; n += kThreads) m = (W[n] > m) ? W[n] : m;
      const double lmax = block_max(m, red);
      if (!(lmax > HYG_NINF)) { if (tid == 0) sh.status = HYG_ENUMERIC; __syncthreads(); break; }
      auto logit = [&](int n) -> double { return W[n]; };
      auto rnd = [&](int q) -> uint64_t {
        return hyg_rand64(ch.seed, ch.chain_id, HYG_RNG_BACKWARD, (uint64_t)t, (uint64_t)q);
      };
      auto out = [&](int q, int n) { idx[q] = n; };
      auto all = [](int) { return true; };
      __syncthreads();
      categorical_block(N, lmax, logit, B, all, rnd, out, cp128, red);
    } else {
      // ---- backward kernel rows (:400-435), one per distinct next state
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
      __syncthreads();
      const int ng = sh.ng;
      bool fail = false;
      for (int g = 0; g < ng; ++g) {
        const uint64_t xn = gst[g];
        double m = HYG_NINF;
        for (int n = tid; n < N; n += kThreads) {
          const double w = W[n];
          double l = HYG_NINF;
          if (w > HYG_NINF) {
            const uint64_t x = state_of(n);
            const Hz4 h = hz_of(md, K, x);
            const double f = tg_trans(c, K, x, xn, h);
            if (hyg_isfinite(f)) l = f + w;
          }
          Lg[n] = l;
          m = (l > m) ? l : m;
        }
        const double lmax = block_max(m, red);
        if (!(lmax > HYG_NINF)) { fail = true; break; }  // uniform
        auto logit = [&](int n) -> double { return Lg[n]; };
        // the draws of the trajectories whose next state is group g
        auto in_g = [&](int b) { return grp[b] == g; };
        auto rnd = [&](int b) -> uint64_t {
          return hyg_rand64(ch.seed, ch.chain_id, HYG_RNG_BACKWARD, (uint64_t)t, (uint64_t)b);
        };
        auto out = [&](int b, int n) { idx[b] = n; };
        __syncthreads();
        categorical_block(N, lmax, logit, B, in_g, rnd, out, cp128, red);
        __syncthreads();
      }
      if (fail) { if (tid == 0) sh.status = HYG_ENUMERIC; __syncthreads(); break; }
    }
    __syncthreads();
    // ---- trajectories and test-function means at t (run_inference_two_groups.py:233-240, 294-314)
    for (int b = tid; b < B; b += kThreads) {
      const uint64_t x = state_of(idx[b]);
      X[b] = x;
      const size_t o = (size_t)(ch.out_begin + t) * B + b;
      o_merged[o] = (int16_t)hyg_st_m(x);
      o_control[2 * o + 0] = (int16_t)hyg_st_dc(x);
      o_control[2 * o + 1] = (int16_t)hyg_st_rc(x);
      o_case[2 * o + 0] = (int16_t)hyg_st_dk(x);
      o_case[2 * o + 1] = (int16_t)hyg_st_rk(x);
    }
    __syncthreads();
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
  __syncthreads();
  if (tid == 0 && status_out) status_out[blockIdx.x] = sh.status;
}

// -------------------------------------------------------------- launchers
// Optional per-kernel timing with HIP events recorded on the launch stream
// (bench.py reads them back with hyg_tg_last_kernel_ms).
namespace {
bool g_timing = false;
hipEvent_t g_ev[6] = {};
bool g_ev_used[3] = {false, false, false};
void ev_record(int k, bool end, hipStream_t s) {
  if (!g_timing) return;
  hipEvent_t& e = g_ev[2 * k + (end ? 1 : 0)];
  if (!e) (void)hipEventCreate(&e);
  (void)hipEventRecord(e, s);
  g_ev_used[k] = true;
}
}  // namespace

void set_kernel_timing(bool on) { g_timing = on; }

int last_kernel_ms(float* out3) {
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

size_t forward_lds_bytes(const hyg_tg_consts& c) { return make_layout(c.K, c.M, c.B, c.Nmax, false).total; }
size_t backward_lds_bytes(const hyg_tg_consts& c) { return make_layout(c.K, c.M, c.B, c.Nmax, true).total; }

int launch_emission(const ModelDev& md, const hyg_tg_consts& c, const uint16_t* meth_c, const uint16_t* tot_c,
                    int s_c, const uint16_t* meth_k, const uint16_t* tot_k, int s_k, int64_t n_sites, double* E,
                    void* stream) {
  if (n_sites <= 0) return HYG_OK;
  int64_t blocks = (n_sites + kThreads - 1) / kThreads;
  if (blocks > 256 * 16) blocks = 256 * 16;
  ev_record(0, false, (hipStream_t)stream);
  hipLaunchKernelGGL(tg_emission_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, (hipStream_t)stream, md.lf, md.lg,
                     md.cst, md.nmax_reads + 1, c.K, meth_c, tot_c, s_c, meth_k, tot_k, s_k, n_sites, E);
  ev_record(0, true, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? HYG_OK : HYG_EDEVICE;
}

int launch_chains(const ModelDev& md, const hyg_tg_consts& c, const ChainDev* chains_dev, int n_chains,
                  const double* E, uint8_t* ws, const hyg_tg_outputs& out, void* stream) {
  if (n_chains <= 0) return HYG_OK;
  const Lay lf = make_layout(c.K, c.M, c.B, c.Nmax, false);
  const Lay lb = make_layout(c.K, c.M, c.B, c.Nmax, true);
  if (lf.total > 160 * 1024 || lb.total > 160 * 1024) return HYG_EUNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  if (hipFuncSetAttribute((const void*)tg_forward_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lf.total) != hipSuccess)
    return HYG_EDEVICE;
  if (hipFuncSetAttribute((const void*)tg_backward_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lb.total) != hipSuccess)
    return HYG_EDEVICE;
  ev_record(1, false, s);
  hipLaunchKernelGGL(tg_forward_kernel, dim3(n_chains), dim3(kThreads), lf.total, s, md, chains_dev, E, ws,
                     out.status, out.log_z, out.final_log_weights, lf);
  ev_record(1, true, s);
  if (hipGetLastError() != hipSuccess) return HYG_EDEVICE;
  ev_record(2, false, s);
  hipLaunchKernelGGL(tg_backward_kernel, dim3(n_chains), dim3(kThreads), lb.total, s, md, chains_dev, E,
                     (const uint8_t*)ws, (const int32_t*)out.status, out.merged, out.control, out.kase,
                     out.split_probs, out.regime_probs, out.status, lb);
  ev_record(2, true, s);
  return hipGetLastError() == hipSuccess ? HYG_OK : HYG_EDEVICE;
}

}  // namespace hyg
