// bed_kernels.hip -- regime BED tracks from the smoothed
// regime probabilities resident in HBM.
//
// Reference: src/single_group/bin/make_bed_file:19-66 (data.table):
//   score = pmax over the regime columns; tie_count = #(columns == score);
//   name  = "equiprobable" if tie_count > 1, else the first column attaining
//           the maximum (max.col ties.method = "first").
// bed_label_kernel computes (label, score) per site: label = the regime index,
// or -1 for "equiprobable". HBM-bound: K f64 read and 9 bytes written per site,
// a grid-stride loop with the K values of a site in registers.
#include <hip/hip_runtime.h>

#include "../../include/hygeia_amd.h"

namespace hyg {

template <bool VEC>
__global__ void __launch_bounds__(256)
bed_label_kernel(const double* __restrict__ probs, int K, int64_t n, int8_t* __restrict__ label,
                 double* __restrict__ score) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double* row = probs + i * K;
    double v[HYG_KMAX];
    if (VEC) {  // even K and a 16-byte aligned base: 16-byte loads
      const double2* r2 = (const double2*)row;
#pragma unroll
      for (int r = 0; r < HYG_KMAX / 2; ++r) {
        const double2 x = (2 * r < K) ? r2[r] : make_double2(0.0, 0.0);
        v[2 * r] = x.x;
        v[2 * r + 1] = x.y;
      }
    } else {
#pragma unroll
      for (int r = 0; r < HYG_KMAX; ++r) v[r] = (r < K) ? row[r] : 0.0;
    }
    // pmax (NA-free rows): the largest value; the first index attaining it
    double mx = v[0];
    int arg = 0;
#pragma unroll
    for (int r = 1; r < HYG_KMAX; ++r)
      if (r < K && v[r] > mx) {
        mx = v[r];
        arg = r;
      }
    int ties = 0;
#pragma unroll
    for (int r = 0; r < HYG_KMAX; ++r) ties += (r < K && v[r] == mx) ? 1 : 0;
    label[i] = (int8_t)(ties > 1 ? -1 : arg);
    score[i] = mx;
  }
}

int bed_launch_labels(const double* probs, int K, int64_t n, int8_t* label, double* score, void* stream) {
  if (n <= 0) return HYG_OK;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 256 * 32) blocks = 256 * 32;
  // the 16-byte row loads need every row 16-byte aligned: K even and the base
  // aligned (a caller may pass any 8-byte aligned view, e.g. buf[1:])
  const bool vec = (K & 1) == 0 && ((uintptr_t)probs & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(bed_label_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, probs, K, n,
                       label, score);
  else
    hipLaunchKernelGGL(bed_label_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, probs, K, n,
                       label, score);
  return hipGetLastError() == hipSuccess ? HYG_OK : HYG_EDEVICE;
}

}  // namespace hyg
