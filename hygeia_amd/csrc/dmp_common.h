// Launchers of the aggregation / DMP-calling kernels (dmp_kernels.hip), used
// by the C ABI in capi.cpp. Not part of the public ABI.
#pragma once

#include <stddef.h>
#include <stdint.h>

namespace hyg {

int launch_dmp_site_counts(const int16_t* merged, const int16_t* control, const int16_t* kase, int B, int K,
                           const int64_t* grp_row0, const int64_t* grp_site, const int64_t* blk_row, int n_groups,
                           int n_seeds, int64_t n_rows_total, int32_t* counts, int32_t* pairs, void* stream);
int launch_post_counts(const float* split, const float* regime, int K2, int B, const int64_t* seg, int n_seg,
                       int64_t max_rows, int exclusive, int32_t* counts, void* stream);
int launch_dmp_hist(const int32_t* counts, int stride, int col, int64_t n, int P, uint32_t* hist, int32_t* bad,
                    void* stream);
int launch_dmp_rank(const int32_t* counts, int stride, int col, int64_t n, int P, double thr, const double* w_fp,
                    const double* w_fn, uint64_t* keys, uint32_t* vals, double* excess, void* stream);
int launch_dmp_gather(const uint32_t* idx, const double* src, int64_t n, double* dst, int64_t* idx64,
                      void* stream);
size_t radix_temp_bytes(int64_t n);
int radix_sort_pairs(uint64_t* keys, uint32_t* vals, int64_t n, void* temp, void* stream);

}  // namespace hyg
