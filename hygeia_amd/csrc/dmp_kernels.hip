// dmp_kernels.hip -- aggregation and DMP calling on the MI355X path
// (aggregate_results.py:71-206, get_dmps.py:46-180,
// multiple_testing.py:3-22), on trajectories that stay resident in HBM after
// hyg_tg_run_chains.
//
//   dmp_site_counts_kernel  per (site, regime): counts over every seed's
//                           trajectories -- #(merged == 0), #(r_ctrl != r_case),
//                           #(r_ctrl == r), #(r_case == r), #(r_ctrl == r, r_case == j)
//   dmp_hist_kernel         histogram of one count column (the FDR sort key:
//                           t = 1 - n / P is decreasing in n, so ascending t is a
//                           counting sort by n)
//   dmp_rank_kernel         weighted-FDR ranking (multiple_testing.py:15-16) as
//                           order-preserving u64 keys, and the excess error rates
//   radix_*                 stable LSD radix sort of (u64 key, u32 index):
//                           8-bit digits, 4096-key tiles, per-wave digit match
//                           by ballots (ties keep ascending index order)
//
// The sequential parts of the reference -- numpy's float64 cumsum over the
// sorted statistics -- are emulated exactly on the host (capi.cpp): a
// parallel scan would round differently.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/hyg_arith.h"
#include "../../include/hygeia_amd.h"
#include "dmp_common.h"
#include "hyg_dev.h"

namespace hyg {

// ---------------------------------------------------------------- counts
// Thread (row, r): row = reported site row of group g (global row index over
// the groups), r = regime. Reads the row's B particles of every seed block.
template <bool PAIRS>
__global__ void __launch_bounds__(256)
dmp_site_counts_kernel(const int16_t* __restrict__ merged, const int16_t* __restrict__ control,
                       const int16_t* __restrict__ kase, int B, int K, const int64_t* __restrict__ grp_row0,
                       const int64_t* __restrict__ grp_site, const int64_t* __restrict__ blk_row, int n_groups,
                       int n_seeds, int64_t n_rows_total, int32_t* __restrict__ counts,
                       int32_t* __restrict__ pairs) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = gid / K;
  const int r = (int)(gid - row * K);
  if (row >= n_rows_total) return;
  int lo = 0, hi = n_groups - 1;  // last group with grp_row0 <= row
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (grp_row0[mid] <= row) lo = mid; else hi = mid - 1;
  }
  const int g = lo;
  const int64_t rr = row - grp_row0[g];
  const int64_t site = grp_site[g] + rr;
  const int C = 2 + 2 * K;
  int n_m0 = 0, n_dm = 0, n_c = 0, n_k = 0;
  int pr[HYG_KMAX];
#pragma unroll
  for (int j = 0; j < HYG_KMAX; ++j) pr[j] = 0;
  for (int s = 0; s < n_seeds; ++s) {
    const int64_t orow = blk_row[(int64_t)g * n_seeds + s] + rr;
    const int16_t* __restrict__ pm = merged + orow * B;
    const int16_t* __restrict__ pc = control + orow * B * 2;
    const int16_t* __restrict__ pk = kase + orow * B * 2;
    for (int b = 0; b < B; ++b) {
      const int c = pc[2 * b + 1], k = pk[2 * b + 1];
      n_m0 += (pm[b] == 0) ? 1 : 0;
      n_dm += (c != k) ? 1 : 0;
      n_c += (c == r) ? 1 : 0;
      n_k += (k == r) ? 1 : 0;
      if constexpr (PAIRS) {
#pragma unroll
        for (int j = 0; j < HYG_KMAX; ++j) pr[j] += (c == r && k == j) ? 1 : 0;
      }
    }
  }
  int32_t* out = counts + site * C;
  if (r == 0) {
    out[0] = n_m0;
    out[1] = n_dm;
  }
  out[2 + r] = n_c;
  out[2 + K + r] = n_k;
  if constexpr (PAIRS) {
    int32_t* po = pairs + (site * K + r) * K;
#pragma unroll
    for (int j = 0; j < HYG_KMAX; ++j)
      if (j < K) po[j] = pr[j];
  }
}

// ------------------------------------------------- posterior counts
// The job's gather of hyg_tg_run_chains outputs (bench.py, parallel.py):
// counts[site][0] += rint(B split[row]), counts[site][1 + j] += rint(B regime[row][j])
// over every trimmed row of every segment (out_row, site, n). The probabilities
// are means over the B trajectories, so B p is an integer in f64; rint is
// torch.round's half-to-even. One thread per count element of a segment's
// contiguous [site0 (1 + 2K), (site0 + n)(1 + 2K)) range (coalesced), grid-
// strided in x, blockIdx.y = segment. EXCL: the call's segments cover disjoint
// sites (the caller's guarantee: one seed's chains), so a plain read-add-write;
// otherwise integer atomics (order-free, but each a read-modify-write beyond L2:
// about 10x slower at the C3 size).
template <bool EXCL>
__global__ void __launch_bounds__(256)
post_counts_kernel(const float* __restrict__ split, const float* __restrict__ regime, int K2, double Bd,
                   const int64_t* __restrict__ seg, int32_t* __restrict__ counts) {
  const int64_t row0 = seg[3 * (int64_t)blockIdx.y], site0 = seg[3 * (int64_t)blockIdx.y + 1],
                n = seg[3 * (int64_t)blockIdx.y + 2];
  const int C = 1 + K2;
  const int64_t ne = n * C;
  int32_t* __restrict__ out = counts + site0 * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / C;
    const int c = (int)(e - i * C);
    const float p = (c == 0) ? split[row0 + i] : regime[(row0 + i) * K2 + (c - 1)];
    const int32_t v = (int32_t)rint((double)p * Bd);
    if constexpr (EXCL) out[e] += v;
    else atomicAdd(out + e, v);
  }
}

// ------------------------------------------------------- FDR histogram
__global__ void __launch_bounds__(256)
dmp_hist_kernel(const int32_t* __restrict__ counts, int stride, int col, int64_t n, int P,
                uint32_t* __restrict__ hist, int32_t* __restrict__ bad) {
  extern __shared__ uint32_t lh[];  // P + 1 bins when they fit, else global atomics
  const bool use_lds = (P + 1) <= 8192;
  if (use_lds)
    for (int i = threadIdx.x; i <= P; i += blockDim.x) lh[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int v = counts[i * stride + col];
    if (v < 0 || v > P) {
      atomicAdd(bad, 1);
      continue;
    }
    if (use_lds) atomicAdd(&lh[v], 1u);
    else atomicAdd(&hist[v], 1u);
  }
  __syncthreads();
  if (use_lds)
    for (int i = threadIdx.x; i <= P; i += blockDim.x)
      if (lh[i]) atomicAdd(&hist[i], lh[i]);
}

// ------------------------------------------------- weighted FDR ranking
// ranking = w_fp (t - thr) / (w_fn (1 - t) + w_fp |t - thr|) with
// t = 1 - n / P (get_dmps.py:69); numpy's elementwise order of operations.
__device__ __forceinline__ uint64_t f64_order_key(double x) {
  if (x != x) return ~0ull;  // NaN last, as np.argsort
  uint64_t u = hyg_f64_bits(x);
  if (u == 0x8000000000000000ull) u = 0;  // -0 == +0
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__global__ void __launch_bounds__(256)
dmp_rank_kernel(const int32_t* __restrict__ counts, int stride, int col, int64_t n, int P, double thr,
                const double* __restrict__ w_fp, const double* __restrict__ w_fn, uint64_t* __restrict__ keys,
                uint32_t* __restrict__ vals, double* __restrict__ excess) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double t = 1.0 - (double)counts[i * stride + col] / (double)P;
    const double fp = w_fp[i], fn = w_fn[i];
    const double d = t - thr;
    const double num = fp * d;
    const double den = fn * (1.0 - t) + fp * __builtin_fabs(d);
    keys[i] = f64_order_key(num / den);
    vals[i] = (uint32_t)i;
    excess[i] = num;  // weights_false_positives * (test_statistics - fdr_threshold)
  }
}

__global__ void __launch_bounds__(256)
dmp_gather_kernel(const uint32_t* __restrict__ idx, const double* __restrict__ src, int64_t n,
                  double* __restrict__ dst, int64_t* __restrict__ idx64) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t j = idx[i];
    dst[i] = src[j];
    if (idx64) idx64[i] = (int64_t)j;
  }
}

// ------------------------------------------------------------ radix sort
constexpr int kRadixThreads = 256;
constexpr int kRadixRounds = 16;
constexpr int kRadixTile = kRadixThreads * kRadixRounds;  // 4096 keys

// digit histogram of one tile -> hist[digit * n_tiles + tile]
__global__ void __launch_bounds__(kRadixThreads)
radix_hist_kernel(const uint64_t* __restrict__ keys, int64_t n, int shift, int n_tiles, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * kRadixTile;
  for (int j = 0; j < kRadixRounds; ++j) {
    const int64_t i = t0 + j * kRadixThreads + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[(int64_t)threadIdx.x * n_tiles + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan of m entries in place, one workgroup of 1024 threads
__global__ void __launch_bounds__(1024) radix_scan_kernel(uint32_t* __restrict__ a, int64_t m) {
  __shared__ uint32_t part[1024];
  const int64_t per = (m + 1023) / 1024;
  const int64_t b0 = threadIdx.x * per;
  const int64_t b1 = (b0 + per < m) ? b0 + per : m;
  uint32_t s = 0;
  for (int64_t i = b0; i < b1; ++i) s += a[i];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
    const uint32_t v = (threadIdx.x >= (unsigned)off) ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = part[threadIdx.x] - s;
  for (int64_t i = b0; i < b1; ++i) {
    const uint32_t v = a[i];
    a[i] = run;
    run += v;
  }
}

// stable scatter: tile-local rank of each key among the keys of its digit, in
// index order (round j, lane order), plus the tile's global digit offset
__global__ void __launch_bounds__(kRadixThreads)
radix_scatter_kernel(const uint64_t* __restrict__ kin, const uint32_t* __restrict__ vin, int64_t n, int shift,
                     int n_tiles, const uint32_t* __restrict__ offs, uint64_t* __restrict__ kout,
                     uint32_t* __restrict__ vout) {
  constexpr int NW = kRadixThreads / 64;
  __shared__ uint32_t base[256];
  __shared__ uint32_t wcnt[NW][256];
  const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  base[tid] = offs[(int64_t)tid * n_tiles + blockIdx.x];
  for (int w = 0; w < NW; ++w) wcnt[w][tid] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * kRadixTile;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int j = 0; j < kRadixRounds; ++j) {
    const int64_t i = t0 + j * kRadixThreads + tid;
    const bool v = i < n;
    const uint64_t key = v ? kin[i] : 0ull;
    const uint32_t val = v ? vin[i] : 0u;
    const uint32_t d = (uint32_t)((key >> shift) & 255u);
    uint64_t peers = wave_ballot(v);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t m = wave_ballot(v && ((d >> b) & 1u));
      peers &= ((d >> b) & 1u) ? m : ~m;
    }
    const int rank = __builtin_popcountll(peers & lt);
    const bool leader = v && rank == 0;
    if (leader) wcnt[wv][d] = (uint32_t)__builtin_popcountll(peers);
    __syncthreads();
    if (v) {
      uint32_t pos = base[d] + (uint32_t)rank;
      for (int w = 0; w < wv; ++w) pos += wcnt[w][d];
      kout[pos] = key;
      vout[pos] = val;
    }
    __syncthreads();
    uint32_t add = 0;  // thread tid owns digit tid: advance its base, clear the wave counts
    for (int w = 0; w < NW; ++w) {
      add += wcnt[w][tid];
      wcnt[w][tid] = 0;
    }
    base[tid] += add;
    __syncthreads();
  }
}

// ---------------------------------------------------------------- launchers
int launch_dmp_site_counts(const int16_t* merged, const int16_t* control, const int16_t* kase, int B, int K,
                           const int64_t* grp_row0, const int64_t* grp_site, const int64_t* blk_row, int n_groups,
                           int n_seeds, int64_t n_rows_total, int32_t* counts, int32_t* pairs, void* stream) {
  const int64_t threads = n_rows_total * K;
  if (threads <= 0) return 0;
  const int64_t blocks = (threads + 255) / 256;
  if (pairs)
    hipLaunchKernelGGL(dmp_site_counts_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       merged, control, kase, B, K, grp_row0, grp_site, blk_row, n_groups, n_seeds, n_rows_total,
                       counts, pairs);
  else
    hipLaunchKernelGGL(dmp_site_counts_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       merged, control, kase, B, K, grp_row0, grp_site, blk_row, n_groups, n_seeds, n_rows_total,
                       counts, pairs);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_post_counts(const float* split, const float* regime, int K2, int B, const int64_t* seg, int n_seg,
                       int64_t max_rows, int exclusive, int32_t* counts, void* stream) {
  if (n_seg <= 0 || max_rows <= 0) return 0;
  int64_t bx = (max_rows * (1 + K2) + 255) / 256;
  if (bx > 256) bx = 256;  // elements grid-strided: up to 256 x 256 threads per segment
  constexpr int kMaxY = 65535;  // grid y limit: segments in launches of at most this many
  for (int s0 = 0; s0 < n_seg; s0 += kMaxY) {
    const int ns = (n_seg - s0 < kMaxY) ? n_seg - s0 : kMaxY;
    const int64_t* sg = seg + 3 * (int64_t)s0;
    if (exclusive)
      hipLaunchKernelGGL(post_counts_kernel<true>, dim3((unsigned)bx, (unsigned)ns), dim3(256), 0,
                         (hipStream_t)stream, split, regime, K2, (double)B, sg, counts);
    else
      hipLaunchKernelGGL(post_counts_kernel<false>, dim3((unsigned)bx, (unsigned)ns), dim3(256), 0,
                         (hipStream_t)stream, split, regime, K2, (double)B, sg, counts);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_dmp_hist(const int32_t* counts, int stride, int col, int64_t n, int P, uint32_t* hist, int32_t* bad,
                    void* stream) {
  const size_t lds = ((P + 1) <= 8192) ? sizeof(uint32_t) * (size_t)(P + 1) : 0;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(dmp_hist_kernel, dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)stream, counts, stride,
                     col, n, P, hist, bad);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_dmp_rank(const int32_t* counts, int stride, int col, int64_t n, int P, double thr, const double* w_fp,
                    const double* w_fn, uint64_t* keys, uint32_t* vals, double* excess, void* stream) {
  int64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(dmp_rank_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, counts, stride,
                     col, n, P, thr, w_fp, w_fn, keys, vals, excess);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_dmp_gather(const uint32_t* idx, const double* src, int64_t n, double* dst, int64_t* idx64,
                      void* stream) {
  int64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(dmp_gather_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, idx, src, n,
                     dst, idx64);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t radix_temp_bytes(int64_t n) {
  const int64_t n_tiles = (n + kRadixTile - 1) / kRadixTile;
  return (size_t)n * (8 + 4) + (size_t)n_tiles * 256 * 4 + 256;
}

// Sorts (keys, vals) ascending by key, stable; results end in keys/vals.
int radix_sort_pairs(uint64_t* keys, uint32_t* vals, int64_t n, void* temp, void* stream) {
  if (n <= 1) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int64_t n_tiles = (n + kRadixTile - 1) / kRadixTile;
  uint64_t* k2 = (uint64_t*)temp;
  uint32_t* v2 = (uint32_t*)(k2 + n);
  uint32_t* hist = (uint32_t*)(((uintptr_t)(v2 + n) + 255) & ~(uintptr_t)255);
  uint64_t *ka = keys, *kb = k2;
  uint32_t *va = vals, *vb = v2;
  for (int pass = 0; pass < 8; ++pass) {
    const int shift = pass * 8;
    hipLaunchKernelGGL(radix_hist_kernel, dim3((unsigned)n_tiles), dim3(kRadixThreads), 0, s, ka, n, shift,
                       (int)n_tiles, hist);
    hipLaunchKernelGGL(radix_scan_kernel, dim3(1), dim3(1024), 0, s, hist, (int64_t)n_tiles * 256);
    hipLaunchKernelGGL(radix_scatter_kernel, dim3((unsigned)n_tiles), dim3(kRadixThreads), 0, s, ka, va, n, shift,
                       (int)n_tiles, hist, kb, vb);
    uint64_t* tk = ka; ka = kb; kb = tk;
    uint32_t* tv = va; va = vb; vb = tv;
  }
  // 8 passes: the result is back in (keys, vals)
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace hyg
