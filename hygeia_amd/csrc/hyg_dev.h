// hyg_dev.h -- device primitives shared by the chain kernels (gfx950):
// lane/wave ids, LDS-only workgroup barriers, DPP wave reductions and scans,
// block reductions and scans of exact integer sums.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "../../include/hyg_arith.h"

namespace hyg {

// Tuning and profiling switches read from the environment (HYG_THREADS,
// HYG_THREADS_FWD / _BWD, HYG_LOWOCC_THREADS, HYG_NO_SHAPE, HYG_TOPSET_R,
// HYG_DEBUG_PHASES, HYG_SG_PHASES) exist only in a build made with -DHYG_TUNING
// (`bash tools/build_variant.sh tuning -DHYG_TUNING`, selected with
// HYG_LIB_PATH). The default library never reads them, so an inherited
// environment cannot change which kernels it launches.
inline const char* tuning_env(const char* name) {
#ifdef HYG_TUNING
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// ----------------------------------------------------------- small helpers
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
// wave index as a wave-uniform (SGPR) value, so branches on it are scalar
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

// Workgroup barrier for LDS hand-offs only. __syncthreads() is a full
// workgroup fence: it also waits for every outstanding global load and store
// of the wave (vmcnt(0)), which would stall each step on the ancestor-history
// stores and on the hazard-row / emission prefetches. Nothing a chain kernel
// writes to global memory is read back by another wave of the same launch.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ------------------------------------------------- DPP wave primitives
// Cross-lane traffic goes through DPP (row shifts / mirrors / broadcasts,
// a few cycles each) and v_readlane, never ds_bpermute (an LDS round trip
// per step). Sums are exact integer sums and maxima are exact, so the
// reduction tree is free.
enum : int {
  kDppQuad1032 = 0xB1,      // quad_perm [1,0,3,2]
  kDppQuad2301 = 0x4E,      // quad_perm [2,3,0,1]
  kDppRowMirror = 0x140,
  kDppRowHalfMirror = 0x141,
  kDppRowBcast15 = 0x142,
  kDppRowBcast31 = 0x143,
  kDppRowShr = 0x110,       // + n, n = 1..15
};
template <int CTRL, int RM = 0xf, int BM = 0xf>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  // bound_ctrl: a lane whose source is outside its row reads 0; lanes of
  // rows disabled by RM keep `old` = 0 as well
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, BM, true);
}
template <int CTRL, int RM = 0xf, int BM = 0xf>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  const uint32_t lo = dpp32<CTRL, RM, BM>((uint32_t)v), hi = dpp32<CTRL, RM, BM>((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
// Value of lane (lane ^ LM) for LM = 1..32: quad perms, row shifts, row_ror:8
// and the gfx950 permlane16/32 swaps (no LDS round trip).
template <int LM>
__device__ __forceinline__ uint32_t xshfl32(uint32_t v) {
  static_assert(LM == 1 || LM == 2 || LM == 4 || LM == 8 || LM == 16 || LM == 32, "lane xor mask");
  if constexpr (LM == 1) {
    return dpp32<kDppQuad1032>(v);
  } else if constexpr (LM == 2) {
    return dpp32<kDppQuad2301>(v);
  } else if constexpr (LM == 4) {
    // row_shl:4 everywhere, then row_shr:4 merged into banks 1 and 3 (lanes
    // with bit 2 set) by the DPP bank mask: no lane-mask select
    const uint32_t up = dpp32<0x104>(v);
    return (uint32_t)__builtin_amdgcn_update_dpp((int)up, (int)v, 0x114, 0xf, 0xa, false);
  } else if constexpr (LM == 8) {
    return dpp32<0x128>(v);  // row_ror:8
  } else if constexpr (LM == 16) {
    // lanes with bit 4 set take r[0], the others r[1]: r[1] merged into rows
    // 0 and 2 by an identity DPP move with a row mask (a lane-mask select would
    // be a loop-invariant SGPR pair the compiler spills and reloads per use)
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (uint32_t)__builtin_amdgcn_update_dpp((int)r[0], (int)r[1], 0xE4, 0x5, 0xf, false);
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);  // rows 0-1 take r[1]
    return (uint32_t)__builtin_amdgcn_update_dpp((int)r[0], (int)r[1], 0xE4, 0x3, 0xf, false);
  }
}
// Lanes l of a wave with (l & j) == 0, for j = 1, 2, ..., 32 (a constant after unrolling)
__device__ __forceinline__ constexpr uint64_t lanes_bit_clear(int j) {
  return j == 1 ? 0x5555555555555555ull
       : j == 2 ? 0x3333333333333333ull
       : j == 4 ? 0x0F0F0F0F0F0F0F0Full
       : j == 8 ? 0x00FF00FF00FF00FFull
       : j == 16 ? 0x0000FFFF0000FFFFull
                 : 0x00000000FFFFFFFFull;
}
// Per-lane select by a wave-uniform lane mask: bit l set -> if1 on lane l.
// v_cndmask with the mask in an SGPR pair, written directly: built from a
// constant lane pattern by scalar ops, the mask stays rematerialisable.
__device__ __forceinline__ uint32_t lane_select32(uint64_t m, uint32_t if0, uint32_t if1) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if0), "v"(if1), "s"(m));
  return r;
}
__device__ __forceinline__ uint64_t lane_select64(uint64_t m, uint64_t if0, uint64_t if1) {
  const uint32_t lo = lane_select32(m, (uint32_t)if0, (uint32_t)if1);
  const uint32_t hi = lane_select32(m, (uint32_t)(if0 >> 32), (uint32_t)(if1 >> 32));
  return ((uint64_t)hi << 32) | lo;
}
template <int LM>
__device__ __forceinline__ uint64_t xshfl64(uint64_t v) {
  return ((uint64_t)xshfl32<LM>((uint32_t)(v >> 32)) << 32) | xshfl32<LM>((uint32_t)v);
}
// LDS hand-off between the lanes of one wave (no workgroup barrier)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}
__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __ballot(p); }
// number of set bits of `mask` below this lane
__device__ __forceinline__ int lanes_below(uint64_t mask) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ double d_of(uint64_t u) { return __builtin_bit_cast(double, u); }
__device__ __forceinline__ uint64_t u_of(double d) { return __builtin_bit_cast(uint64_t, d); }

__device__ __forceinline__ double dmax(double a, double b) { return (b > a) ? b : a; }

// reduce inside each 16-lane row (every lane of the row gets the row result)
template <typename F>
__device__ __forceinline__ double row_reduce_d(double v, F op) {
  v = op(v, d_of(dpp64<kDppQuad1032>(u_of(v))));
  v = op(v, d_of(dpp64<kDppQuad2301>(u_of(v))));
  v = op(v, d_of(dpp64<kDppRowHalfMirror>(u_of(v))));
  v = op(v, d_of(dpp64<kDppRowMirror>(u_of(v))));
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
  auto mx = [](double a, double b) { return dmax(a, b); };
  v = row_reduce_d(v, mx);
  const double a = d_of(rdlane64(u_of(v), 0)), b = d_of(rdlane64(u_of(v), 16));
  const double c = d_of(rdlane64(u_of(v), 32)), d = d_of(rdlane64(u_of(v), 48));
  return dmax(dmax(a, b), dmax(c, d));
}
__device__ __forceinline__ int wave_sum(int v) {
  uint32_t x = (uint32_t)v;
  x += dpp32<kDppQuad1032>(x);
  x += dpp32<kDppQuad2301>(x);
  x += dpp32<kDppRowHalfMirror>(x);
  x += dpp32<kDppRowMirror>(x);
  return __builtin_amdgcn_readlane((int)x, 0) + __builtin_amdgcn_readlane((int)x, 16) +
         __builtin_amdgcn_readlane((int)x, 32) + __builtin_amdgcn_readlane((int)x, 48);
}
__device__ __forceinline__ hyg_u128 wave_sum128(hyg_u128 v) {
  hyg_u128 w;
  w.lo = dpp64<kDppQuad1032>(v.lo); w.hi = dpp64<kDppQuad1032>(v.hi); v = hyg_u128_add(v, w);
  w.lo = dpp64<kDppQuad2301>(v.lo); w.hi = dpp64<kDppQuad2301>(v.hi); v = hyg_u128_add(v, w);
  w.lo = dpp64<kDppRowHalfMirror>(v.lo); w.hi = dpp64<kDppRowHalfMirror>(v.hi); v = hyg_u128_add(v, w);
  w.lo = dpp64<kDppRowMirror>(v.lo); w.hi = dpp64<kDppRowMirror>(v.hi); v = hyg_u128_add(v, w);
  hyg_u128 s = hyg_u128_zero();
  for (int r = 0; r < 64; r += 16) {
    hyg_u128 x;
    x.lo = rdlane64(v.lo, r);
    x.hi = rdlane64(v.hi, r);
    s = hyg_u128_add(s, x);
  }
  return s;
}

// wave total of an exact u192 sum: quad / row mirrors, then the four row
// results read out (fewer dependent steps than an inclusive scan)
__device__ __forceinline__ hyg_u192 wave_sum192(hyg_u192 v) {
  hyg_u192 w;
  w.w0 = dpp64<kDppQuad1032>(v.w0); w.w1 = dpp64<kDppQuad1032>(v.w1); w.w2 = dpp64<kDppQuad1032>(v.w2);
  v = hyg_u192_add(v, w);
  w.w0 = dpp64<kDppQuad2301>(v.w0); w.w1 = dpp64<kDppQuad2301>(v.w1); w.w2 = dpp64<kDppQuad2301>(v.w2);
  v = hyg_u192_add(v, w);
  w.w0 = dpp64<kDppRowHalfMirror>(v.w0); w.w1 = dpp64<kDppRowHalfMirror>(v.w1); w.w2 = dpp64<kDppRowHalfMirror>(v.w2);
  v = hyg_u192_add(v, w);
  w.w0 = dpp64<kDppRowMirror>(v.w0); w.w1 = dpp64<kDppRowMirror>(v.w1); w.w2 = dpp64<kDppRowMirror>(v.w2);
  v = hyg_u192_add(v, w);
  hyg_u192 s = hyg_u192_zero();
  for (int r = 0; r < 64; r += 16) {
    hyg_u192 x;
    x.w0 = rdlane64(v.w0, r); x.w1 = rdlane64(v.w1, r); x.w2 = rdlane64(v.w2, r);
    s = hyg_u192_add(s, x);
  }
  return s;
}

// inclusive wave scans (Hillis-Steele inside rows, then row broadcasts)
template <int CTRL, int RM>
__device__ __forceinline__ hyg_u192 dpp192(hyg_u192 v) {
  hyg_u192 r;
  r.w0 = dpp64<CTRL, RM>(v.w0); r.w1 = dpp64<CTRL, RM>(v.w1); r.w2 = dpp64<CTRL, RM>(v.w2);
  return r;
}
__device__ __forceinline__ hyg_u192 wave_incl192(hyg_u192 v) {
  v = hyg_u192_add(v, dpp192<kDppRowShr + 1, 0xf>(v));
  v = hyg_u192_add(v, dpp192<kDppRowShr + 2, 0xf>(v));
  v = hyg_u192_add(v, dpp192<kDppRowShr + 4, 0xf>(v));
  v = hyg_u192_add(v, dpp192<kDppRowShr + 8, 0xf>(v));
  v = hyg_u192_add(v, dpp192<kDppRowBcast15, 0xa>(v));
  v = hyg_u192_add(v, dpp192<kDppRowBcast31, 0xc>(v));
  return v;
}
__device__ __forceinline__ hyg_u192 rdlane192(hyg_u192 v, int l) {
  hyg_u192 r;
  r.w0 = rdlane64(v.w0, l); r.w1 = rdlane64(v.w1, l); r.w2 = rdlane64(v.w2, l);
  return r;
}
template <int CTRL, int RM>
__device__ __forceinline__ hyg_u128 dpp128(hyg_u128 v) {
  hyg_u128 r;
  r.lo = dpp64<CTRL, RM>(v.lo); r.hi = dpp64<CTRL, RM>(v.hi);
  return r;
}
__device__ __forceinline__ hyg_u128 wave_incl128(hyg_u128 v) {
  v = hyg_u128_add(v, dpp128<kDppRowShr + 1, 0xf>(v));
  v = hyg_u128_add(v, dpp128<kDppRowShr + 2, 0xf>(v));
  v = hyg_u128_add(v, dpp128<kDppRowShr + 4, 0xf>(v));
  v = hyg_u128_add(v, dpp128<kDppRowShr + 8, 0xf>(v));
  v = hyg_u128_add(v, dpp128<kDppRowBcast15, 0xa>(v));
  v = hyg_u128_add(v, dpp128<kDppRowBcast31, 0xc>(v));
  return v;
}
__device__ __forceinline__ int wave_incl_int(int v) {
  uint32_t x = (uint32_t)v;
  x += dpp32<kDppRowShr + 1, 0xf>(x);
  x += dpp32<kDppRowShr + 2, 0xf>(x);
  x += dpp32<kDppRowShr + 4, 0xf>(x);
  x += dpp32<kDppRowShr + 8, 0xf>(x);
  x += dpp32<kDppRowBcast15, 0xa>(x);
  x += dpp32<kDppRowBcast31, 0xc>(x);
  return (int)x;
}

// ---- combining the per-wave partials of a block reduction
// Up to HYG_SEQ_WAVES waves: every lane reads all of them from LDS (broadcast
// reads) and adds them in wave order. More waves (768-thread chains): lane
// l < NW reads wave l's partial and a DPP row reduction / scan combines them,
// so the registers and instructions do not grow with the workgroup (NW <= 16).
#ifndef HYG_SEQ_WAVES
#define HYG_SEQ_WAVES 4
#endif
template <int CTRL>
__device__ __forceinline__ hyg_u192 dpp192f(hyg_u192 v) {
  hyg_u192 r;
  r.w0 = dpp64<CTRL>(v.w0); r.w1 = dpp64<CTRL>(v.w1); r.w2 = dpp64<CTRL>(v.w2);
  return r;
}
__device__ __forceinline__ hyg_u192 row_sum192(hyg_u192 v) {  // every lane of a row: the row's sum
  v = hyg_u192_add(v, dpp192f<kDppQuad1032>(v));
  v = hyg_u192_add(v, dpp192f<kDppQuad2301>(v));
  v = hyg_u192_add(v, dpp192f<kDppRowHalfMirror>(v));
  v = hyg_u192_add(v, dpp192f<kDppRowMirror>(v));
  return v;
}
__device__ __forceinline__ hyg_u128 row_sum128(hyg_u128 v) {
  hyg_u128 w;
  w.lo = dpp64<kDppQuad1032>(v.lo); w.hi = dpp64<kDppQuad1032>(v.hi); v = hyg_u128_add(v, w);
  w.lo = dpp64<kDppQuad2301>(v.lo); w.hi = dpp64<kDppQuad2301>(v.hi); v = hyg_u128_add(v, w);
  w.lo = dpp64<kDppRowHalfMirror>(v.lo); w.hi = dpp64<kDppRowHalfMirror>(v.hi); v = hyg_u128_add(v, w);
  w.lo = dpp64<kDppRowMirror>(v.lo); w.hi = dpp64<kDppRowMirror>(v.hi); v = hyg_u128_add(v, w);
  return v;
}
template <int NW>
__device__ __forceinline__ hyg_u192 sum_waves192(const hyg_u192* r) {
  static_assert(NW >= 1 && NW <= 16, "waves per workgroup");
  if constexpr (NW <= HYG_SEQ_WAVES) {
    hyg_u192 s = r[0];
    for (int w = 1; w < NW; ++w) s = hyg_u192_add(s, r[w]);
    return s;
  } else {
    const int l = lane_id();
    hyg_u192 v = hyg_u192_zero();
    if (l < NW) v = r[l];
    return rdlane192(row_sum192(v), 0);
  }
}
template <int NW>
__device__ __forceinline__ hyg_u128 sum_waves128(const hyg_u128* r) {
  static_assert(NW >= 1 && NW <= 16, "waves per workgroup");
  if constexpr (NW <= HYG_SEQ_WAVES) {
    hyg_u128 s = r[0];
    for (int w = 1; w < NW; ++w) s = hyg_u128_add(s, r[w]);
    return s;
  } else {
    const int l = lane_id();
    hyg_u128 v = hyg_u128_zero();
    if (l < NW) v = r[l];
    v = row_sum128(v);
    hyg_u128 o;
    o.lo = rdlane64(v.lo, 0);
    o.hi = rdlane64(v.hi, 0);
    return o;
  }
}

// Block-wide reductions. `red` is an LDS scratch of at least 32 B per wave;
// every call starts with a barrier so consecutive calls may reuse it
// (LEAD = false: the caller guarantees that every read of `red` by an earlier
// reduction is behind a barrier already, e.g. its own slot of `red`).
template <int NT, bool LEAD = true>
__device__ __forceinline__ void block_max_cnt(double m, int c, unsigned char* red, double* m_out, int* c_out) {
  m = wave_max(m);
  c = wave_sum(c);
  if (NT == 64) { *m_out = m; *c_out = c; return; }
  if constexpr (LEAD) lds_barrier();
  if (lane_id() == 0) {
    ((double*)red)[2 * wave_id()] = m;
    ((int*)red)[4 * wave_id() + 2] = c;
  }
  lds_barrier();
  if constexpr (NT / 64 <= HYG_SEQ_WAVES) {
    double mm = ((double*)red)[0];
    int cc = ((int*)red)[2];
    for (int w = 1; w < NT / 64; ++w) {
      mm = dmax(mm, ((double*)red)[2 * w]);
      cc += ((int*)red)[4 * w + 2];
    }
    *m_out = mm;
    *c_out = cc;
  } else {
    const int l = lane_id();
    double mm = HYG_NINF;
    uint32_t cc = 0;
    if (l < NT / 64) {
      mm = ((double*)red)[2 * l];
      cc = (uint32_t)((int*)red)[4 * l + 2];
    }
    auto mx = [](double a, double b) { return dmax(a, b); };
    mm = row_reduce_d(mm, mx);
    cc += dpp32<kDppQuad1032>(cc);
    cc += dpp32<kDppQuad2301>(cc);
    cc += dpp32<kDppRowHalfMirror>(cc);
    cc += dpp32<kDppRowMirror>(cc);
    *m_out = d_of(rdlane64(u_of(mm), 0));
    *c_out = __builtin_amdgcn_readlane((int)cc, 0);
  }
}
template <int NT>
__device__ __forceinline__ double block_max(double v, unsigned char* red) {
  v = wave_max(v);
  if (NT == 64) return v;
  lds_barrier();
  if (lane_id() == 0) ((double*)red)[wave_id()] = v;
  lds_barrier();
  if constexpr (NT / 64 <= HYG_SEQ_WAVES) {
    double m = ((double*)red)[0];
    for (int w = 1; w < NT / 64; ++w) m = dmax(m, ((double*)red)[w]);
    return m;
  } else {
    const double m = lane_id() < NT / 64 ? ((double*)red)[lane_id()] : HYG_NINF;
    auto mx = [](double a, double b) { return dmax(a, b); };
    return d_of(rdlane64(u_of(row_reduce_d(m, mx)), 0));
  }
}
template <int NT, bool LEAD = true>
__device__ __forceinline__ hyg_u128 block_sum128(hyg_u128 v, unsigned char* red) {
  hyg_u128* r = (hyg_u128*)red;
  v = wave_sum128(v);
  if (NT == 64) return v;
  if constexpr (LEAD) lds_barrier();
  if (lane_id() == 0) r[wave_id()] = v;
  lds_barrier();
  return sum_waves128<NT / 64>(r);
}

// Block-wide OR of a predicate through LDS (no vmcnt drain, unlike
// __syncthreads_or, so outstanding global stores are not waited for).
template <int NT>
__device__ __forceinline__ bool block_or(bool p, unsigned char* red) {
  const bool w = wave_ballot(p) != 0;
  if (NT == 64) return w;
  lds_barrier();
  if (lane_id() == 0) ((int*)red)[wave_id()] = w ? 1 : 0;
  lds_barrier();
  int any = 0;
  for (int i = 0; i < NT / 64; ++i) any |= ((int*)red)[i];
  return any != 0;
}

// Exclusive block scans. The register forms return this thread's exclusive
// prefix and the block total; the array form writes out[tid] (exclusive) and
// out[NT] (total) for searches.
template <int NT, bool LEAD = true>
__device__ __forceinline__ hyg_u192 block_excl192(hyg_u192 v, unsigned char* red, hyg_u192* total) {
  hyg_u192* r = (hyg_u192*)red;
  const hyg_u192 inc = wave_incl192(v);
  hyg_u192 wt;  // this wave's total
  wt.w0 = rdlane64(inc.w0, 63); wt.w1 = rdlane64(inc.w1, 63); wt.w2 = rdlane64(inc.w2, 63);
  if constexpr (LEAD) lds_barrier();
  if (lane_id() == 0) r[wave_id()] = wt;
  lds_barrier();
  hyg_u192 pre = hyg_u192_zero(), tot = hyg_u192_zero();
  if constexpr (NT / 64 <= HYG_SEQ_WAVES) {
    for (int w = 0; w < NT / 64; ++w) {
      if (w < wave_id()) pre = hyg_u192_add(pre, r[w]);
      tot = hyg_u192_add(tot, r[w]);
    }
  } else {  // lane l: waves 0..l inclusive; this wave's prefix at lane wave - 1
    const int l = lane_id(), wv = wave_id();
    hyg_u192 x = hyg_u192_zero();
    if (l < NT / 64) x = r[l];
    x = wave_incl192(x);
    tot = rdlane192(x, NT / 64 - 1);
    if (wv > 0) pre = rdlane192(x, wv - 1);
  }
  *total = tot;
  return hyg_u192_add(pre, hyg_u192_sub(inc, v));
}
template <int NT>
__device__ __forceinline__ int block_excl_int(int v, unsigned char* red, int* total) {
  int* r = (int*)red;
  const int inc = wave_incl_int(v);
  const int wt = __builtin_amdgcn_readlane(inc, 63);
  lds_barrier();
  if (lane_id() == 0) r[wave_id()] = wt;
  lds_barrier();
  int pre = 0, tot = 0;
  for (int w = 0; w < NT / 64; ++w) {
    if (w < wave_id()) pre += r[w];
    tot += r[w];
  }
  *total = tot;
  return pre + inc - v;
}
template <int NT>
__device__ __forceinline__ void block_scan128(hyg_u128 v, hyg_u128* out, unsigned char* red) {
  hyg_u128* r = (hyg_u128*)red;
  const hyg_u128 inc = wave_incl128(v);
  hyg_u128 wt;
  wt.lo = rdlane64(inc.lo, 63); wt.hi = rdlane64(inc.hi, 63);
  lds_barrier();
  if (lane_id() == 0) r[wave_id()] = wt;
  lds_barrier();
  hyg_u128 pre = hyg_u128_zero(), tot = hyg_u128_zero();
  if constexpr (NT / 64 <= HYG_SEQ_WAVES) {
    for (int w = 0; w < NT / 64; ++w) {
      if (w < wave_id()) pre = hyg_u128_add(pre, r[w]);
      tot = hyg_u128_add(tot, r[w]);
    }
  } else {
    const int l = lane_id(), wv = wave_id();
    hyg_u128 x = hyg_u128_zero();
    if (l < NT / 64) x = r[l];
    x = wave_incl128(x);
    tot.lo = rdlane64(x.lo, NT / 64 - 1);
    tot.hi = rdlane64(x.hi, NT / 64 - 1);
    if (wv > 0) {
      pre.lo = rdlane64(x.lo, wv - 1);
      pre.hi = rdlane64(x.hi, wv - 1);
    }
  }
  hyg_u128 e2;  // inc - v
  e2.lo = inc.lo - v.lo;
  e2.hi = inc.hi - v.hi - (inc.lo < v.lo ? 1u : 0u);
  out[threadIdx.x] = hyg_u128_add(pre, e2);
  if (threadIdx.x == 0) out[NT] = tot;
}
// The same scan with this thread's exclusive prefix and the block total
// returned in registers: no LDS output, so a caller that needs only its own
// prefix and the total needs no barrier behind it (red's readers are done when
// it returns; its next writer must still be behind a barrier).
template <int NT>
__device__ __forceinline__ void block_scan128_regs(hyg_u128 v, unsigned char* red, hyg_u128* excl, hyg_u128* total) {
  hyg_u128* r = (hyg_u128*)red;
  const hyg_u128 inc = wave_incl128(v);
  hyg_u128 wt;
  wt.lo = rdlane64(inc.lo, 63); wt.hi = rdlane64(inc.hi, 63);
  lds_barrier();
  if (lane_id() == 0) r[wave_id()] = wt;
  lds_barrier();
  hyg_u128 pre = hyg_u128_zero(), tot = hyg_u128_zero();
  if constexpr (NT / 64 <= HYG_SEQ_WAVES) {
    for (int w = 0; w < NT / 64; ++w) {
      if (w < wave_id()) pre = hyg_u128_add(pre, r[w]);
      tot = hyg_u128_add(tot, r[w]);
    }
  } else {
    const int l = lane_id(), wv = wave_id();
    hyg_u128 x = hyg_u128_zero();
    if (l < NT / 64) x = r[l];
    x = wave_incl128(x);
    tot.lo = rdlane64(x.lo, NT / 64 - 1);
    tot.hi = rdlane64(x.hi, NT / 64 - 1);
    if (wv > 0) {
      pre.lo = rdlane64(x.lo, wv - 1);
      pre.hi = rdlane64(x.hi, wv - 1);
    }
  }
  hyg_u128 e2;  // inc - v
  e2.lo = inc.lo - v.lo;
  e2.hi = inc.hi - v.hi - (inc.lo < v.lo ? 1u : 0u);
  *excl = hyg_u128_add(pre, e2);
  *total = tot;
}


}  // namespace hyg
