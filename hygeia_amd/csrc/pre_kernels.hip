// pre_kernels.hip -- `hygeia preprocess`: strand collapse of
// per-strand methylation BED records and their counts on the chromosome's CpG
// grid, for one sample.
//
// Reference: src/two_group/preprocess_bed.py (polars 1.8.2)
//   collapse_strands :183-259   full join of "+" rows (key end) with "-" rows
//                               (key start); coverage / percent of a missing
//                               strand 0; total = cov+ + cov-; key = start+ or
//                               start- - 1; rows with total > 0 kept;
//                               avg = (cov+ pct+ + cov- pct-) / total
//   process_sample_data :298-317 meth = round(total avg / 100),
//                               unmeth = round(total (100 - avg) / 100)
//   :325-336, :497-543          full joins on Pos0 whose unmatched sample rows
//                               get a null Pos0 and are dropped (:365-369): a
//                               left join onto the CpG positions, missing -> 0
//                               (np.nan_to_num, :384)
// Both strands' records are sorted by start with unique starts (the host
// checks), so the joins are binary searches: pre_mark_kernel marks the "-"
// records a "+" record pairs with; pre_grid_kernel resolves every CpG site
// independently (HBM-bound: a few searches and one output pair per site).
#include <hip/hip_runtime.h>

#include "../../include/hygeia_amd.h"

namespace hyg {

__device__ __forceinline__ int64_t pre_lower(const int64_t* a, int64_t lo, int64_t hi, int64_t key) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}
// index of key in a[lo, hi) (sorted, unique), or -1
__device__ __forceinline__ int64_t pre_find_in(const int64_t* a, int64_t lo, int64_t hi, int64_t key) {
  const int64_t i = pre_lower(a, lo, hi, key);
  return (i < hi && a[i] == key) ? i : -1;
}
__device__ __forceinline__ int64_t pre_find(const int64_t* __restrict__ a, int64_t n, int64_t key) {
  return pre_find_in(a, 0, n, key);
}

// polars f64 round (Rust f64::round: half away from zero)
__device__ __forceinline__ double pre_round(double x) {
  const double a = fabs(x);
  double f = floor(a);
  f = (a - f >= 0.5) ? f + 1.0 : f;
  return copysign(f, x);
}

// "-" records paired with a "+" record (matched on end == start): one chunk
// of 256 "+" records per block and iteration, searches bounded to the "-"
// records between the chunk's first and last end when the end lies there.
__global__ void __launch_bounds__(256)
pre_mark_kernel(const int64_t* __restrict__ plus_end, int64_t n_plus, const int64_t* __restrict__ minus_start,
                int64_t n_minus, uint8_t* __restrict__ matched) {
  __shared__ int64_t win[2];
  const int64_t n_chunks = (n_plus + 255) / 256;
  for (int64_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
    const int64_t i0 = c * 256, i1 = (i0 + 256 < n_plus) ? i0 + 256 : n_plus;
    __syncthreads();
    if (threadIdx.x == 0) win[0] = pre_lower(minus_start, 0, n_minus, plus_end[i0]);
    else if (threadIdx.x == 64) win[1] = pre_lower(minus_start, 0, n_minus, plus_end[i1 - 1] + 1);
    __syncthreads();
    const int64_t i = i0 + threadIdx.x;
    if (i >= n_plus) continue;
    const int64_t e = plus_end[i];
    const int64_t lo = win[0], hi = win[1];
    const bool inwin = lo < hi && e >= minus_start[lo] && e <= minus_start[hi - 1];
    const int64_t j = inwin ? pre_find_in(minus_start, lo, hi, e) : pre_find(minus_start, n_minus, e);
    if (j >= 0) matched[j] = 1;
  }
}

// One 256-site chunk of the (sorted) grid per block and iteration: the
// chunk's key range bounds every search to the records inside it (found once
// per chunk by two threads), so a site's searches touch a few cache lines
// instead of ~25 random ones per search over the whole chromosome.
__global__ void __launch_bounds__(256)
pre_grid_kernel(const int64_t* __restrict__ pos0, int64_t T, const int64_t* __restrict__ plus_start,
                const int64_t* __restrict__ plus_end, const double* __restrict__ plus_cov,
                const double* __restrict__ plus_pct, int64_t n_plus, const int64_t* __restrict__ minus_start,
                const double* __restrict__ minus_cov, const double* __restrict__ minus_pct, int64_t n_minus,
                const uint8_t* __restrict__ matched, int single_base, double* __restrict__ out, int stride, int col,
                int* __restrict__ conflicts) {
  constexpr int kWin = 1024;
  __shared__ int64_t win[4];  // plus [lo, hi), minus [lo, hi) of the chunk
  __shared__ int64_t sp[kWin], sm[kWin];
  const int64_t n_chunks = (T + 255) / 256;
  for (int64_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
    const int64_t t0 = c * 256, t1 = (t0 + 256 < T) ? t0 + 256 : T;
    __syncthreads();
    if (threadIdx.x == 0) {
      win[0] = pre_lower(plus_start, 0, n_plus, pos0[t0]);
      win[2] = pre_lower(minus_start, 0, n_minus, pos0[t0] + 1);
    } else if (threadIdx.x == 64) {
      win[1] = pre_lower(plus_start, 0, n_plus, pos0[t1 - 1] + 1);
      win[3] = pre_lower(minus_start, 0, n_minus, pos0[t1 - 1] + 2);
    }
    __syncthreads();
    // the windows' starts staged in LDS with coalesced loads (windows larger
    // than kWin records -- records between grid sites -- search HBM instead)
    const int64_t np_w = win[1] - win[0], nm_w = win[3] - win[2];
    const bool lp = np_w <= kWin, lm = nm_w <= kWin;
    if (lp)
      for (int64_t i = threadIdx.x; i < np_w; i += 256) sp[i] = plus_start[win[0] + i];
    if (lm)
      for (int64_t i = threadIdx.x; i < nm_w; i += 256) sm[i] = minus_start[win[2] + i];
    __syncthreads();
    const int64_t t = t0 + threadIdx.x;
    if (t >= T) continue;
    const int64_t k = pos0[t];
    // the collapsed row with key k: a "+" record starting at k (with its "-"
    // partner starting at its end), or an unpaired "-" record starting at k + 1
    int64_t ip, jm;
    if (lp) {
      ip = pre_find_in(sp, 0, np_w, k);
      ip = ip >= 0 ? win[0] + ip : -1;
    } else {
      ip = pre_find_in(plus_start, win[0], win[1], k);
    }
    if (lm) {
      jm = pre_find_in(sm, 0, nm_w, k + 1);
      jm = jm >= 0 ? win[2] + jm : -1;
    } else {
      jm = pre_find_in(minus_start, win[2], win[3], k + 1);
    }
    // single-base "+" records: the only "+" record ending at k + 1 starts at k
    const bool minus_only = jm >= 0 && (single_base ? ip < 0 : !matched[jm]);
    double cp = 0.0, pp = 0.0, cn = 0.0, pn = 0.0;
    bool have = false;
    if (ip >= 0) {
      cp = plus_cov[ip];
      pp = plus_pct[ip];
      const int64_t e = plus_end[ip];
      // the partner usually lies in the chunk's window (single-base records)
      int64_t jn;
      if (lm && nm_w > 0 && e >= sm[0] && e <= sm[nm_w - 1]) {
        jn = pre_find_in(sm, 0, nm_w, e);
        jn = jn >= 0 ? win[2] + jn : -1;
      } else {
        jn = pre_find(minus_start, n_minus, e);
      }
      if (jn >= 0) {
        cn = minus_cov[jn];
        pn = minus_pct[jn];
      }
      have = true;
      if (minus_only) atomicAdd(conflicts, 1);  // two collapsed rows with one key
    } else if (minus_only) {
      cn = minus_cov[jm];
      pn = minus_pct[jm];
      have = true;
    }
    const double total = cp + cn;
    // no collapsed row (or coverage 0, filtered at :228-230): null, i.e. NaN
    double meth = __builtin_nan(""), unmeth = __builtin_nan("");
    if (have && total > 0.0) {
      const double avg = ((cp * pp) + (cn * pn)) / total;
      meth = pre_round((total * avg) / 100.0);
      unmeth = pre_round((total * (100.0 - avg)) / 100.0);
    }
    out[t * stride + col] = meth;
    out[t * stride + col + 1] = unmeth;
  }
}

int pre_launch_collapse(const int64_t* pos0, int64_t T, const int64_t* plus_start, const int64_t* plus_end,
                        const double* plus_cov, const double* plus_pct, int64_t n_plus, const int64_t* minus_start,
                        const double* minus_cov, const double* minus_pct, int64_t n_minus, int single_base,
                        uint8_t* matched, double* out, int stride, int col, int* conflicts, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!single_base && n_minus > 0 && hipMemsetAsync(matched, 0, (size_t)n_minus, s) != hipSuccess) return HYG_EDEVICE;
  auto grid = [](int64_t n) {
    int64_t b = (n + 255) / 256;
    return (unsigned)(b < 1 ? 1 : (b > 256 * 32 ? 256 * 32 : b));
  };
  if (!single_base && n_plus > 0 && n_minus > 0)
    hipLaunchKernelGGL(pre_mark_kernel, dim3(grid(n_plus)), dim3(256), 0, s, plus_end, n_plus, minus_start, n_minus,
                       matched);
  if (T > 0)
    hipLaunchKernelGGL(pre_grid_kernel, dim3(grid(T)), dim3(256), 0, s, pos0, T, plus_start, plus_end, plus_cov,
                       plus_pct, n_plus, minus_start, minus_cov, minus_pct, n_minus, matched, single_base, out, stride,
                       col, conflicts);
  return hipGetLastError() == hipSuccess ? HYG_OK : HYG_EDEVICE;
}

}  // namespace hyg
