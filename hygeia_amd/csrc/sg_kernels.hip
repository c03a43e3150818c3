// sg_kernels.hip -- CDNA4 (gfx950) kernels of the single-group path.
//
//   sg_emission_kernel  per-site Beta-Binomial table E[t][r] (HBM streaming)
//   sg_chain_kernel     SMC for the change-point model + online marginal
//                       smoothing, one 256-thread workgroup per chain, one
//                       particle per thread (N_max <= 256), persistent over T.
//
// Same computations as oracle/sg_oracle.c (the arithmetic contract of
// include/hyg_arith.h: exact fixed-point sums, hyg_exp / hyg_log, Philox), so
// the smoothed regime probabilities are bit-identical to the oracle's.
// Reference: src/single_group/src/cpp/algorithms/Smc.h:114-579,
// misc/resample.h:85-117,289-409, algorithms/OnlineMarginalSmoothing.h:52-255,
// algorithms/OnlineCombinedInference.h:48-118, singleGroup.h:556-627.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../../include/hyg_arith.h"
#include "hyg_dev.h"
#include "sg_common.h"

namespace hyg {

__device__ __forceinline__ uint32_t sg_pack(int d, int r) { return (uint32_t)d | ((uint32_t)r << 24); }
__device__ __forceinline__ int sg_d(uint32_t s) { return (int)(s & 0xffffffu); }
__device__ __forceinline__ int sg_r(uint32_t s) { return (int)(s >> 24); }

// Model::evaluateLogTransitionDensity for (1, rc) or (dc > 1, rc == rp) from (dp, rp)
__device__ __forceinline__ double sg_trans(const SgModelDev& md, const hyg_sg_consts& c, int dc, int rc, int dp,
                                           int rp) {
  int d = dp - 1;
  if (d >= md.dcap) d = md.dcap - 1;
  const double2 h = *(const double2*)(md.hz + ((size_t)rp * md.dcap + d) * 2);
  if (dc == 1 && rc != rp && dp >= c.u) {
    const double lp = c.logP[rp * c.K + rc];
    return md.ex[(size_t)rp * md.dcap + d] ? lp : (h.x + lp);
  }
  if (dc > 1 && rc == rp) return h.y;
  return HYG_NINF;
}

// exact wave sum of u128 values (all 64 lanes active)
__device__ __forceinline__ double wave_fixsum(hyg_u128 v) { return hyg_u128_to_f64(wave_sum128(v), 100); }

// ceil(T * R) for a double T in [0, 1] and R < 2^127 (oracle/sg_oracle.c:ceil_mul_f64)
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
struct SgShared {
  int npend, nfree, cur, status;
};

struct SgLay {
  size_t stP, stC, lwP, lwC, wP, wC, lwres, anc, idx, cum, BK, scr, mean, red, sh, total;
};

__host__ __device__ inline size_t sg_align(size_t x) { return (x + 15) / 16 * 16; }

__host__ __device__ inline SgLay sg_layout(int K) {
  SgLay l{};
  const int NT = kSgThreads, NW = NT / 64;
  size_t o = 0;
  l.stP = o; o = sg_align(o + 4 * NT);
  l.stC = o; o = sg_align(o + 4 * NT);
  l.lwP = o; o = sg_align(o + 8 * NT);
  l.lwC = o; o = sg_align(o + 8 * NT);
  l.wP = o; o = sg_align(o + 8 * NT);
  l.wC = o; o = sg_align(o + 8 * NT);
  l.lwres = o; o = sg_align(o + 8 * NT);
  l.anc = o; o = sg_align(o + 4 * NT);
  l.idx = o; o = sg_align(o + 4 * NT);
  l.cum = o; o = sg_align(o + 16 * (NT + 1));
  l.BK = o; o = sg_align(o + 8 * (size_t)K * NT);
  l.scr = o; o = sg_align(o + 8 * (size_t)NW * NT);
  l.mean = o; o = sg_align(o + 8 * (size_t)NW * HYG_KMAX);
  l.red = o; o = sg_align(o + 16 * NW);
  l.sh = o; o = sg_align(o + sizeof(SgShared));
  l.total = o;
  return l;
}

size_t sg_lds_bytes(const hyg_sg_consts& c) { return sg_layout(c.K).total; }

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

// --------------------------------------------------------- chain kernel
// Block-wide exact log-sum-exp (thread n holds x_n, -inf when unused).
__device__ __forceinline__ double sg_block_lse(double x, unsigned char* red) {
  const double mx = block_max<kSgThreads>(x, red);
  if (!(mx > HYG_NINF)) return HYG_NINF;
  const hyg_u128 s = block_sum128<kSgThreads>(hyg_fix100(hyg_exp(x - mx)), red);
  return mx + hyg_log(hyg_u128_to_f64(s, 100));
}
// Wave-level exact log-sum-exp over the 4 values per lane (n = lane + 64 i)
__device__ __forceinline__ double sg_wave_lse4(const double v[4]) {
  double mx = dmax(dmax(v[0], v[1]), dmax(v[2], v[3]));
  mx = wave_max(mx);
  if (!(mx > HYG_NINF)) return HYG_NINF;
  hyg_u128 s = hyg_u128_zero();
#pragma unroll
  for (int i = 0; i < 4; ++i) s = hyg_u128_add(s, hyg_fix100(hyg_exp(v[i] - mx)));
  return mx + hyg_log(hyg_u128_to_f64(wave_sum128(s), 100));
}
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}
// sorted position of value v of thread `me` among vals[0, n): descending, ties by index
__device__ __forceinline__ int sg_rank_desc(const double* vals, int n, double v, int me) {
  int rank = 0;
  for (int m = 0; m < n; ++m) {
    const double w = vals[m];
    rank += (w > v || (w == v && m < me)) ? 1 : 0;
  }
  return rank;
}

// One workgroup per chain, thread n = particle n. The pending smoothing times
// live in the chain's workspace region: cap slots of psi [K][256] doubles and
// the lists slot[2][cap], time[2][cap], keep[cap], free[cap] (int32).
__global__ void __launch_bounds__(kSgThreads)
sg_chain_kernel(SgModelDev md, const SgChainDev* __restrict__ chains, const double* __restrict__ E,
                uint8_t* __restrict__ ws, int cap, double* __restrict__ probs, int32_t* __restrict__ status_out,
                SgLay lay) {
  constexpr int NT = kSgThreads, NW = NT / 64;
  const hyg_sg_consts& c = *md.consts;
  const int K = c.K, Nmax = c.Nmax, tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  const SgChainDev ch = chains[blockIdx.x];
  const int T = ch.T;
  extern __shared__ __align__(16) unsigned char smem[];
  uint32_t* stP = (uint32_t*)(smem + lay.stP);
  uint32_t* stC = (uint32_t*)(smem + lay.stC);
  double* lwP = (double*)(smem + lay.lwP);
  double* lwC = (double*)(smem + lay.lwC);
  double* wP = (double*)(smem + lay.wP);
  double* wC = (double*)(smem + lay.wC);
  double* lwres = (double*)(smem + lay.lwres);
  int* anc = (int*)(smem + lay.anc);
  int* idx = (int*)(smem + lay.idx);
  hyg_u128* cum = (hyg_u128*)(smem + lay.cum);
  double* BK = (double*)(smem + lay.BK);
  double* scr = (double*)(smem + lay.scr) + wv * NT;
  double* meanb = (double*)(smem + lay.mean) + wv * HYG_KMAX;
  unsigned char* red = smem + lay.red;
  SgShared& sh = *(SgShared*)(smem + lay.sh);
  uint8_t* base = ws + ch.psi_offset;
  double* psi = (double*)base;
  int32_t* lists = (int32_t*)(base + sg_psi_region_bytes(K, cap));
  int32_t* keepf = lists + 4 * (size_t)cap;
  int32_t* freel = lists + 5 * (size_t)cap;
  double* out = probs + (size_t)ch.out_begin * K;
  const double* Ech = E + (size_t)ch.site_begin * K;

  for (int i = tid; i < cap; i += NT) freel[i] = cap - 1 - i;
  if (tid == 0) {
    sh.npend = 0;
    sh.nfree = cap;
    sh.cur = 0;
    sh.status = HYG_OK;
  }
  // ---- t = 0 (Smc.h:114-188): N = K particles (1, r), log w = -log K + log g_0(r)
  int N = K;
  double x = HYG_NINF;
  if (tid < K) {
    stC[tid] = sg_pack(1, tid);
    x = -c.log_K + Ech[tid];
    lwC[tid] = x;
  }
  double logZ = sg_block_lse(x, red);
  if (!(logZ > HYG_NINF)) {
    if (tid == 0) status_out[blockIdx.x] = HYG_ENUMERIC;
    return;
  }
  if (tid < K) wC[tid] = hyg_exp(lwC[tid] - logZ);
  __syncthreads();

  int status = HYG_OK;
  for (int t = 0; t < T; ++t) {
    const bool final = (t == T - 1);
    int M = 0, Np = N;
    if (t > 0) {
      // ---- Smc::iterate (:190-286): previous <- current
      if (tid < Np) {
        stP[tid] = stC[tid];
        lwP[tid] = lwC[tid];
        wP[tid] = wC[tid];
      }
      const double logZp = logZ;
      N = (Np + K > Nmax) ? Nmax : Np + K;
      M = N - K;
      lds_barrier();
      // ---- resampleCp (:406-450)
      if (N < Np + K) {
        int fin;
        (void)block_excl_int<NT>((tid < Np && hyg_isfinite(lwP[tid])) ? 1 : 0, red, &fin);
        bool keep_top = true;
        if (fin > M) {
          // optimalFiniteState (resample.h:289-409) on the sorted self-normalised weights
          if (tid < Np) idx[sg_rank_desc(wP, Np, wP[tid], tid)] = tid;
          lds_barrier();
          double lq = HYG_NINF;
          hyg_u128 mq = hyg_u128_zero();
          if (tid < Np) {
            const double q = wP[idx[tid]];
            lq = hyg_log(q);
            mq = hyg_fix100(q);
          }
          // reverse cumulative sums Q(k) = total - exclusive prefix (exact)
          block_scan128<NT>(mq, cum, red);
          lds_barrier();
          {
            const hyg_u128 tot = cum[NT], ex = cum[tid];
            hyg_u128 suf;
            suf.lo = tot.lo - ex.lo;
            suf.hi = tot.hi - ex.hi - (tot.lo < ex.lo ? 1u : 0u);
            lds_barrier();
            cum[tid] = suf;
            if (tid == 0) cum[NT] = hyg_u128_zero();
          }
          lds_barrier();
          // the K / log c fixed point (:333-342), counts block-parallel
          int kOld = 1, kNew = 0;
          double logC = 0.0;
          while (kNew != kOld) {
            kOld = kNew;
            const double Qk = hyg_u128_to_f64(cum[kOld], 100);
            logC = hyg_log((double)(M - kOld)) - hyg_log(Qk);
            int cnt;
            (void)block_excl_int<NT>((tid >= kOld && tid < Np && lq > -logC) ? 1 : 0, red, &cnt);
            kNew = kOld + cnt;
          }
          if (hyg_isfinite(logC)) {
            keep_top = false;
            const int Kk = kNew, L = M - Kk;
            if (tid < Kk) {
              anc[tid] = idx[tid];
              lwres[tid] = lwP[idx[tid]];
            }
            if (L > 0) {
              // residual systematic draw (:372-377, systematicBase :85-117):
              // T_j = (j + u) / L <= Q_i as exact C_i >= ceil(T_j R)
              const double rv = (tid >= Kk && tid < Np) ? lq : HYG_NINF;
              const double rmax = block_max<NT>(rv, red);
              hyg_u128 m2 = hyg_u128_zero();
              if (tid >= Kk && tid < Np) m2 = hyg_fix100(hyg_exp(lq - rmax));
              block_scan128<NT>(m2, cum, red);  // also a barrier before the overwrite
              const hyg_u128 incl = hyg_u128_add(cum[tid], m2);
              lds_barrier();
              cum[tid] = incl;
              lds_barrier();
              const hyg_u128 R = cum[Np - 1];
              if (tid < L) {
                const double uu =
                    (double)(hyg_rand64(ch.seed, ch.chain_id, kSgRngSystematic, (uint64_t)t, 0) >> 11) *
                    1.1102230246251565404e-16;
                const double Tj = ((double)tid + uu) / (double)L;
                const hyg_u128 thr = sg_ceil_mul_f64(Tj, R);
                int lo = Kk, hi = Np - 1;
                while (lo < hi) {
                  const int mid = (lo + hi) >> 1;
                  if (hyg_u128_lt(cum[mid], thr)) lo = mid + 1; else hi = mid;
                }
                anc[Kk + tid] = idx[lo];
                lwres[Kk + tid] = logZp - logC;
              }
            }
          }
        }
        if (keep_top) {
          // keep the M largest log-weights (Smc.h:432-441, resample.h:379-384)
          if (tid < Np) {
            const double v = lwP[tid];
            const int rank = sg_rank_desc(lwP, Np, v, tid);
            if (rank < M) {
              anc[rank] = tid;
              lwres[rank] = v;
            }
          }
        }
      } else if (tid < M) {
        anc[tid] = tid;
        lwres[tid] = lwP[tid];
      }
      lds_barrier();
      // ---- sampleParticlesCp (:504-522) + computeWeightsCp (:536-574)
      const double* Et = Ech + (size_t)t * K;
      if (tid < M) {
        const uint32_t a = stP[anc[tid]];
        const int d = sg_d(a) + 1, r = sg_r(a);
        stC[tid] = sg_pack(d, r);
        lwC[tid] = lwres[tid] + (sg_trans(md, c, d, r, sg_d(a), r) + Et[r]);
      }
      // new particles (1, q) and the backward kernels (:288-326), one row q per wave
      for (int q = wv; q < K; q += NW) {
        const double eq = Et[q];
        double vn[4], vb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = lane + 64 * i;
          vn[i] = HYG_NINF;
          vb[i] = HYG_NINF;
          if (n < Np) {
            const uint32_t s = stP[n];
            const double tr = sg_trans(md, c, 1, q, sg_d(s), sg_r(s));
            vn[i] = (tr + eq) + lwP[n];
            vb[i] = lwP[n] + tr;
          }
        }
        const double ln = sg_wave_lse4(vn);
        const double lb = sg_wave_lse4(vb);
        if (lane == 0) {
          lwC[M + q] = ln;
          stC[M + q] = sg_pack(1, q);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = lane + 64 * i;
          if (n < Np) BK[q * NT + n] = (lb > HYG_NINF) ? hyg_exp(vb[i] - lb) : 0.0;
        }
      }
      lds_barrier();
      // ---- selfNormaliseWeights (:576-579)
      logZ = sg_block_lse(tid < N ? lwC[tid] : HYG_NINF, red);
      if (!(logZ > HYG_NINF)) {
        status = HYG_ENUMERIC;
        break;
      }
      if (tid < N) wC[tid] = hyg_exp(lwC[tid] - logZ);
    }
    // ---- online marginal smoothing: updatePsi (OnlineMarginalSmoothing.h:152-197)
    //      of the pending times, initialisePsi (:132-150) of time t, storeEstimates
    //      (:199-253) with the epsilon rule
    const int cur = sh.cur, nold = sh.npend;
    int32_t* slotA = lists + (size_t)cur * 2 * cap;
    int32_t* timeA = slotA + cap;
    if (tid == 0) {
      if (sh.nfree == 0) {
        sh.status = HYG_ENOMEM;
      } else {
        const int f = --sh.nfree;
        slotA[nold] = freel[f];
        timeA[nold] = t;
      }
    }
    __syncthreads();
    if (sh.status != HYG_OK) {
      status = sh.status;
      break;
    }
    const int ntot = nold + 1;
    for (int e = wv; e < ntot; e += NW) {
      const bool fresh = (e == nold);
      double* sp = psi + (size_t)slotA[e] * K * NT;
      bool ok = true;
      for (int r = 0; r < K; ++r) {
        double* row = sp + (size_t)r * NT;
        double nv[4];
        if (fresh) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int n = lane + 64 * i;
            nv[i] = (n < N && sg_r(stC[n]) == r) ? 1.0 : 0.0;
          }
        } else {
          double pv[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int n = lane + 64 * i;
            pv[i] = (n < Np) ? row[n] : 0.0;
            scr[n] = pv[i];
          }
          wave_lds_sync();
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int n = lane + 64 * i;
            nv[i] = (n < M) ? scr[anc[n]] : 0.0;
          }
          for (int q = 0; q < K; ++q) {
            hyg_u128 s = hyg_u128_zero();
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int n = lane + 64 * i;
              if (n < Np) s = hyg_u128_add(s, hyg_fix100(BK[q * NT + n] * pv[i]));
            }
            const double v = hyg_u128_to_f64(wave_sum128(s), 100);
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
        hyg_u128 sm = hyg_u128_zero();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = lane + 64 * i;
          if (n < N) sm = hyg_u128_add(sm, hyg_fix100(wC[n] * nv[i]));
        }
        const double mean = hyg_u128_to_f64(wave_sum128(sm), 100);
        if (lane == 0) meanb[r] = mean;
        if (!final && ok) {
          hyg_u128 sv = hyg_u128_zero();
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int n = lane + 64 * i;
            if (n < N) {
              const double dv = nv[i] - mean;
              sv = hyg_u128_add(sv, hyg_fix100(wC[n] * (dv * dv)));
            }
          }
          if (!(hyg_u128_to_f64(wave_sum128(sv), 100) < c.epsilon)) ok = false;
        }
      }
      const bool store = final || ok;
      wave_lds_sync();
      if (store && lane < K) out[(size_t)timeA[e] * K + lane] = meanb[lane];
      if (lane == 0) keepf[e] = store ? 0 : 1;
      wave_lds_sync();
    }
    __syncthreads();
    // compaction of the pending list into the other buffer; freed slots go
    // back on the free list (the order of pending times does not matter)
    {
      int32_t* slotB = lists + (size_t)(cur ^ 1) * 2 * cap;
      int32_t* timeB = slotB + cap;
      int nk = 0, nf = sh.nfree;
      for (int b = 0; b < ntot; b += NT) {
        const int e = b + tid;
        const int kp = (e < ntot) ? keepf[e] : 0;
        const int v = (e < ntot) ? (kp ? 1 : 0x10000) : 0;
        int tot;
        const int ex = block_excl_int<NT>(v, red, &tot);
        if (e < ntot) {
          if (kp) {
            const int p = nk + (ex & 0xffff);
            slotB[p] = slotA[e];
            timeB[p] = timeA[e];
          } else {
            freel[nf + (ex >> 16)] = slotA[e];
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
  if (tid == 0) status_out[blockIdx.x] = status;
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

int sg_launch_chains(const SgModelDev& md, const hyg_sg_consts& c, const SgChainDev* chains_dev, int n_chains,
                     const double* E, uint8_t* ws, int psi_cap, double* probs, int32_t* status, void* stream) {
  if (n_chains <= 0) return HYG_OK;
  if (c.Nmax > kSgThreads) return HYG_EUNSUPPORTED;
  const SgLay lay = sg_layout(c.K);
  if (lay.total > 160 * 1024) return HYG_EUNSUPPORTED;
  if (hipFuncSetAttribute((const void*)sg_chain_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lay.total) != hipSuccess)
    return HYG_EDEVICE;
  hipLaunchKernelGGL(sg_chain_kernel, dim3(n_chains), dim3(kSgThreads), lay.total, (hipStream_t)stream, md,
                     chains_dev, E, ws, psi_cap, probs, status, lay);
  return hipGetLastError() == hipSuccess ? HYG_OK : HYG_EDEVICE;
}

}  // namespace hyg
