/*
 * hyg_arith.h -- the deterministic arithmetic contract of hygeia_amd.
 *
 * Everything on the change-point inference path that decides an index (which
 * ancestors survive resampling, which particle a backward trajectory picks)
 * is computed with the primitives in this header, on the CPU oracle and in the
 * HIP kernels alike, so that both produce bit-identical trajectories:
 *
 *   - hyg_exp / hyg_log: exp and log built from IEEE-754 basic operations only
 *     (+ - * / floor and EXPLICIT fused multiply-adds, fma() / v_fma_f64, which
 *     IEEE 754 defines with one rounding, so host and device agree; no implicit
 *     contraction: every translation unit is compiled with -ffp-contract=off).
 *     libm / ocml differ in the last ulp between host and device; these do
 *     not. Accuracy is ~1 ulp (tests/test_arith.py pins them against libm).
 *   - exact fixed-point mass sums. The reference sums exp(weights) with
 *     order-dependent float cumsums (resampling_functions.py:10,59; the TF
 *     multinomial CDF behind tfd.Categorical.sample,
 *     filter_and_smoother_algorithm.py:385,426). Here every such sum is an
 *     exact integer sum, so it does not depend on summation order and any
 *     parallel reduction tree on the GPU gives the oracle's value:
 *       * resampling masses exp(f32 log-weight) are f32 values >= 2^-149 and
 *         are summed EXACTLY in 192-bit integers scaled by 2^149 (no rounding
 *         at all, the ideal the reference's f32 cumsum approximates);
 *       * categorical masses exp(logit - max) (f64) are truncated to 2^-100
 *         and summed exactly in 128-bit integers.
 *   - Philox4x64-10 (Salmon et al., SC'11) counter-based uniforms keyed by
 *     (seed, chain), countered by (stream, step, index): the "injected
 *     randomness" both implementations consume. Pinned against numpy's Philox
 *     in tests/test_arith.py.
 *   - the packed 64-bit particle state (merged, d_ctrl, r_ctrl, d_case, r_case).
 *
 * C99-compatible so that the plain-C oracle (oracle/tg_oracle.c) includes it;
 * under hipcc every function is __host__ __device__.
 */
#ifndef HYG_ARITH_H
#define HYG_ARITH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define HYG_HD __host__ __device__ __forceinline__
#define HYG_FLOOR(x) __builtin_floor(x)
#define HYG_FMIN(a, b) __builtin_fmin(a, b)
#define HYG_FMAX(a, b) __builtin_fmax(a, b)
#define HYG_FLOORF(x) __builtin_floorf(x)
#define HYG_FMA(a, b, c) __builtin_fma(a, b, c)
#define HYG_FMAF(a, b, c) __builtin_fmaf(a, b, c)
#define HYG_FMINF(a, b) __builtin_fminf(a, b)
#define HYG_FMAXF(a, b) __builtin_fmaxf(a, b)
#else
#include <math.h>
#define HYG_HD static inline
/* host forms that compile inline (no libm calls) with the same results on the
 * arguments the contract uses: floor of |v| < 2^62, maxNum/minNum semantics
 * for a NaN first argument */
static inline double hyg__floor(double v) {
  const double t = (double)(long long)v;
  return (t > v) ? t - 1.0 : t;
}
static inline double hyg__fmin(double a, double b) { return (a < b) ? a : ((a != a) ? b : b); }
static inline double hyg__fmax(double a, double b) { return (a > b) ? a : ((a != a) ? b : b); }
static inline float hyg__floorf(float v) { /* |v| < 2^31 */
  const float t = (float)(long long)v;
  return (t > v) ? t - 1.0f : t;
}
static inline float hyg__fminf(float a, float b) { return (a < b) ? a : ((a != a) ? b : b); }
static inline float hyg__fmaxf(float a, float b) { return (a > b) ? a : ((a != a) ? b : b); }
#define HYG_FLOOR(x) hyg__floor(x)
#define HYG_FMIN(a, b) hyg__fmin(a, b)
#define HYG_FMAX(a, b) hyg__fmax(a, b)
#define HYG_FLOORF(x) hyg__floorf(x)
/* IEEE fused multiply-add (one rounding): C99 fma / fmaf, correctly rounded by
 * definition (the oracle builds with -mfma: the x86 FMA3 instructions) */
#define HYG_FMA(a, b, c) fma(a, b, c)
#define HYG_FMAF(a, b, c) fmaf(a, b, c)
#define HYG_FMINF(a, b) hyg__fminf(a, b)
#define HYG_FMAXF(a, b) hyg__fmaxf(a, b)
#endif

/* ------------------------------------------------------------------ bits */
HYG_HD uint64_t hyg_f64_bits(double x) { union { double d; uint64_t u; } c; c.d = x; return c.u; }
HYG_HD double hyg_bits_f64(uint64_t u) { union { double d; uint64_t u; } c; c.u = u; return c.d; }
HYG_HD uint32_t hyg_f32_bits(float x) { union { float f; uint32_t u; } c; c.f = x; return c.u; }
HYG_HD float hyg_bits_f32(uint32_t u) { union { float f; uint32_t u; } c; c.u = u; return c.f; }

#define HYG_INF (hyg_bits_f64(0x7ff0000000000000ull))
#define HYG_NINF (hyg_bits_f64(0xfff0000000000000ull))
#define HYG_NAN (hyg_bits_f64(0x7ff8000000000000ull))
#define HYG_NINFF (hyg_bits_f32(0xff800000u))

HYG_HD int hyg_isfinite(double x) { return (hyg_f64_bits(x) & 0x7ff0000000000000ull) != 0x7ff0000000000000ull; }
HYG_HD int hyg_isfinitef(float x) { return (hyg_f32_bits(x) & 0x7f800000u) != 0x7f800000u; }

/* 2^e as a double, e in [-1022, 1023] (exact). */
HYG_HD double hyg_pow2(int e) { return hyg_bits_f64((uint64_t)(e + 1023) << 52); }

/* ------------------------------------------------------------- exp / log */
/* ln2 split: hi has 21 trailing zero bits so k*hi is exact for |k| < 2^11. */
#define HYG_LN2_HI 6.93147180369123816490e-01
#define HYG_LN2_LO 1.90821492927058770002e-10
#define HYG_INV_LN2 1.44269504088896338700e+00

/* exp(x) for double x. Range reduction x = k ln2 + r, |r| <= ln2/2, the
 * degree-13 Taylor polynomial of e^r (remainder < 4e-18) evaluated by
 * Estrin's scheme (dependency depth 8 instead of Horner's 26: the GPU
 * kernels are latency-bound on these chains), then an exact (or
 * single-rounding, for subnormal results) scale by 2^k. Written without
 * branches: special inputs are resolved by selects at the end. */
/* e^r for |r| <= ln2/2: the degree-13 Taylor polynomial by Estrin's scheme,
 * every pair a + b x one fused multiply-add */
HYG_HD double hyg__exp_poly(double r) {
  const double r2 = r * r;
  const double r4 = r2 * r2;
  const double r8 = r4 * r4;
  const double q0 = HYG_FMA(1.0, r, 1.0);
  const double q1 = HYG_FMA(1.6666666666666665741e-01, r, 0.5);                   /* 1/2!, 1/3! */
  const double q2 = HYG_FMA(8.3333333333333332177e-03, r, 4.1666666666666664354e-02); /* 1/4!, 1/5! */
  const double q3 = HYG_FMA(1.9841269841269841253e-04, r, 1.3888888888888888889e-03); /* 1/6!, 1/7! */
  const double q4 = HYG_FMA(2.7557319223985890653e-06, r, 2.4801587301587301566e-05); /* 1/8!, 1/9! */
  const double q5 = HYG_FMA(2.5052108385441718775e-08, r, 2.7557319223985890653e-07); /* 1/10!, 1/11! */
  const double q6 = HYG_FMA(1.6059043836821614599e-10, r, 2.0876756987868098979e-09); /* 1/12!, 1/13! */
  const double s0 = HYG_FMA(q1, r2, q0);
  const double s1 = HYG_FMA(q3, r2, q2);
  const double s2 = HYG_FMA(q5, r2, q4);
  const double u0 = HYG_FMA(s1, r4, s0);
  const double u1 = HYG_FMA(q6, r4, s2);
  return HYG_FMA(u1, r8, u0);
}
HYG_HD double hyg_exp(double x) {
  const double xc = HYG_FMIN(HYG_FMAX(x, -746.0), 710.0); /* NaN -> -746 (result selected below) */
  const double kd = HYG_FLOOR(xc * HYG_INV_LN2 + 0.5);
  const int k = (int)kd;
  const double hi = xc - kd * HYG_LN2_HI;         /* exact */
  const double r = HYG_FMA(-kd, HYG_LN2_LO, hi);   /* one rounding */
  const double p = hyg__exp_poly(r);
  /* k > 1023: (p*2) 2^(k-1); k >= -1021: p 2^k; else (p 2^(k+54)) 2^-54 */
  const int big = k > 1023, sub = k < -1021;
  const int k1 = big ? k - 1 : (sub ? k + 54 : k);
  const double p1 = big ? p * 2.0 : p;
  double v = p1 * hyg_pow2(k1);
  v = sub ? v * 5.5511151231257827021e-17 : v; /* 2^-54 */
  v = (x < -745.13321910194110842) ? 0.0 : v;
  v = (x > 709.782712893383973096) ? HYG_INF : v;
  return (x != x) ? x : v;
}

/* log(x) for double x: x = 2^e m, m in (sqrt(1/2), sqrt(2)], f = m - 1,
 * s = f/(2+f), log(1+f) = f - (f^2/2 - s (f^2/2 + R(s^2))) with the atanh
 * series R(z) = sum_{i>=1} 2 z^i/(2i+1) to i = 11 (|s| <= 0.1716), the
 * polynomial by Estrin's scheme. Branch-free like hyg_exp. */
HYG_HD double hyg_log(double x) {
  uint64_t b = hyg_f64_bits(x);
  const int subn = (b >> 52) == 0; /* zero or subnormal */
  const double xs = subn ? x * 18014398509481984.0 : x; /* 2^54 */
  b = hyg_f64_bits(xs);
  int e = (subn ? -54 : 0) + (int)((b >> 52) & 0x7ff) - 1023;
  double m = hyg_bits_f64((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
  const int hi_m = m > 1.41421356237309504880;
  m = hi_m ? m * 0.5 : m;
  e += hi_m;
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s;
  const double z2 = z * z;
  const double z4 = z2 * z2;
  const double z8 = z4 * z4;
  /* R/z = sum_{i=0}^{10} a_i z^i, a_i = 2/(2i+3) */
  const double a01 = HYG_FMA(0.40000000000000000000, z, 0.66666666666666666667);
  const double a23 = HYG_FMA(0.22222222222222222222, z, 0.28571428571428571429);
  const double a45 = HYG_FMA(0.15384615384615384615, z, 0.18181818181818181818);
  const double a67 = HYG_FMA(0.11764705882352941176, z, 0.13333333333333333333);
  const double a89 = HYG_FMA(0.09523809523809523810, z, 0.10526315789473684211);
  const double a10 = 0.08695652173913043478;
  const double b0 = HYG_FMA(a23, z2, a01);
  const double b1 = HYG_FMA(a67, z2, a45);
  const double b2 = HYG_FMA(a10, z2, a89);
  const double c0 = HYG_FMA(b1, z4, b0);
  const double R = z * HYG_FMA(b2, z8, c0);
  const double hfsq = 0.5 * f * f;
  const double l1p = f - HYG_FMA(-s, hfsq + R, hfsq);
  const double ed = (double)e;
  double v = HYG_FMA(ed, HYG_LN2_HI, HYG_FMA(ed, HYG_LN2_LO, l1p));
  v = ((b >> 52) == 0x7ff) ? xs : v; /* +inf */
  v = (x == 0.0) ? HYG_NINF : v;
  return (x != x || x < 0.0) ? HYG_NAN : v;
}

/* exp(x) for float x in float32 arithmetic only, ~1 ulp: the resampling
 * masses (resampling_functions.py:10,59 take tf.exp of the float32
 * log-weights). Cody-Waite reduction x = k ln2 + r (ln2_hi has 15 significant
 * bits, so k*ln2_hi is exact for |k| <= 150), the degree-7 Taylor polynomial of
 * e^r (|r| <= 0.347, truncation < 0.05 ulp) by Estrin's scheme, then a scale
 * by 2^k in one product (normal results; two products, the first exact, for
 * subnormal ones; k > 127: (2p) 2^(k-1)), every step an IEEE f32 basic
 * operation, so host and device give the same bits. */
HYG_HD float hyg_expf(float x) {
  /* (the clamp and the floor in f32: the same values as through double, since
   * -104, 89 and the floor of an f32 value are f32 values) */
  const float xc = HYG_FMINF(HYG_FMAXF(x, -104.0f), 89.0f); /* NaN -> -104 */
  const float kf = HYG_FLOORF(xc * 0x1.715476p+0f + 0.5f);
  const float hi = xc - kf * 0x1.62e4p-1f;                  /* exact */
  const float r = HYG_FMAF(-kf, 0x1.7f7d1cp-20f, hi);       /* one rounding */
  const float r2 = r * r;
  const float r4 = r2 * r2;
  const float q0 = 1.0f + r;
  const float q1 = HYG_FMAF(0x1.555556p-3f, r, 0.5f);           /* 1/2!, 1/3! */
  const float q2 = HYG_FMAF(0x1.111112p-7f, r, 0x1.555556p-5f); /* 1/4!, 1/5! */
  const float q3 = HYG_FMAF(0x1.a01a02p-13f, r, 0x1.6c16c2p-10f); /* 1/6!, 1/7! */
  const float p = HYG_FMAF(HYG_FMAF(q3, r2, q2), r4, HYG_FMAF(q1, r2, q0));
  const int k = (int)kf;
  const int big = k > 127, sub = k < -126;
  const int k1 = big ? k - 1 : (sub ? k + 64 : k);
  const float p1 = big ? p * 2.0f : p;
  float v = p1 * hyg_bits_f32((uint32_t)(k1 + 127) << 23);
  v = sub ? v * 0x1p-64f : v;
  v = (x < -104.0f) ? 0.0f : v;
  v = (x > 89.0f) ? hyg_bits_f32(0x7f800000u) : v;
  return (x != x) ? x : v;
}
HYG_HD float hyg_logf(float x) { return (float)hyg_log((double)x); }

/* ------------------------------------------------------ 64-bit integer help */
HYG_HD uint64_t hyg_mulhi64(uint64_t a, uint64_t b) {
  const uint64_t a0 = a & 0xffffffffu, a1 = a >> 32, b0 = b & 0xffffffffu, b1 = b >> 32;
  const uint64_t p00 = a0 * b0, p01 = a0 * b1, p10 = a1 * b0, p11 = a1 * b1;
  const uint64_t mid = (p00 >> 32) + (p01 & 0xffffffffu) + (p10 & 0xffffffffu);
  return p11 + (p01 >> 32) + (p10 >> 32) + (mid >> 32);
}

HYG_HD int hyg_clz64(uint64_t x) { return x ? __builtin_clzll(x) : 64; }

/* ------------------------------------------------------------ u128 (F=100) */
typedef struct { uint64_t lo, hi; } hyg_u128;

HYG_HD hyg_u128 hyg_u128_zero(void) { hyg_u128 r; r.lo = 0; r.hi = 0; return r; }
#if defined(__HIPCC__)
/* Multiword add / subtract / compare as 32-bit carry chains (v_add_co_u32 +
 * v_addc_co_u32 on the GPU: 4 VALU ops per u128 add, 6 per u192, instead of
 * 64-bit adds with compare-and-select carries). Same integers as the C forms
 * below, which the gcc-built oracle uses. */
#define HYG__L32(x) ((unsigned)(x))
#define HYG__H32(x) ((unsigned)((x) >> 32))
#define HYG__J64(l, h) ((uint64_t)(l) | ((uint64_t)(h) << 32))
HYG_HD hyg_u128 hyg_u128_add(hyg_u128 a, hyg_u128 b) {
  unsigned c0, c1, c2, c3;
  const unsigned r0 = __builtin_addc(HYG__L32(a.lo), HYG__L32(b.lo), 0u, &c0);
  const unsigned r1 = __builtin_addc(HYG__H32(a.lo), HYG__H32(b.lo), c0, &c1);
  const unsigned r2 = __builtin_addc(HYG__L32(a.hi), HYG__L32(b.hi), c1, &c2);
  const unsigned r3 = __builtin_addc(HYG__H32(a.hi), HYG__H32(b.hi), c2, &c3);
  hyg_u128 r; r.lo = HYG__J64(r0, r1); r.hi = HYG__J64(r2, r3); return r;
}
/* a < b: the borrow out of a - b */
HYG_HD int hyg_u128_lt(hyg_u128 a, hyg_u128 b) {
  unsigned c0, c1, c2, c3;
  (void)__builtin_subc(HYG__L32(a.lo), HYG__L32(b.lo), 0u, &c0);
  (void)__builtin_subc(HYG__H32(a.lo), HYG__H32(b.lo), c0, &c1);
  (void)__builtin_subc(HYG__L32(a.hi), HYG__L32(b.hi), c1, &c2);
  (void)__builtin_subc(HYG__H32(a.hi), HYG__H32(b.hi), c2, &c3);
  return (int)c3;
}
#else
HYG_HD hyg_u128 hyg_u128_add(hyg_u128 a, hyg_u128 b) {
  hyg_u128 r; r.lo = a.lo + b.lo; r.hi = a.hi + b.hi + (r.lo < a.lo ? 1u : 0u); return r;
}
HYG_HD int hyg_u128_lt(hyg_u128 a, hyg_u128 b) { return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo); }
#endif
HYG_HD int hyg_u128_is_zero(hyg_u128 a) { return (a.lo | a.hi) == 0; }

/* floor(e * 2^100) for e in [0, 2^16) (masses are in [0, 1]); masses below
 * 2^-100, non-positive or NaN e, and e >= 2^16 give 0. Computed in f64 basic
 * operations, every step exact: v = e 2^100 (a power-of-two scaling), its
 * 32-bit limbs by floor and exact differences (v - floor(v / 2^64) 2^64 is v
 * mod 2^64, which has at most 53 significant bits), the last limb truncated
 * by the conversion. No shifts and no branches, so unrolled GPU loops
 * interleave independent masses. */
HYG_HD hyg_u128 hyg_fix100(double e) {
  const double v = (e > 0.0 && e < 65536.0) ? e * 0x1p100 : 0.0;
  const double hf = HYG_FLOOR(v * 0x1p-64);  /* < 2^52 */
  const double lf = v - hf * 0x1p64;         /* [0, 2^64) */
  const double lhf = HYG_FLOOR(lf * 0x1p-32); /* [0, 2^32) */
  const double llf = lf - lhf * 0x1p32;       /* [0, 2^32), fractional below 2^52 */
  const double hhf = HYG_FLOOR(hf * 0x1p-32);
  const double hlf = hf - hhf * 0x1p32;
  hyg_u128 r;
  r.lo = ((uint64_t)(uint32_t)lhf << 32) | (uint64_t)(uint32_t)llf;
  r.hi = ((uint64_t)(uint32_t)hhf << 32) | (uint64_t)(uint32_t)hlf;
  return r;
}

/* hyg_fix100(hyg_exp(x)), the same integer computed from the pieces of the
 * exponential instead of through its double value: for -70 <= x < 11,
 * hyg_exp(x) = p 2^k exactly (the polynomial value p, a normal double in
 * (0.7, 1.42), scaled by a power of two without rounding), so
 * floor(e 2^100) = m 2^(E_p + k + 48) for p's 53-bit significand m and exponent
 * E_p -- a shift, no float floors. Below -70 the exact image is 0
 * (e^x 2^100 < 1 for x < -69.32). The identity is claimed for x <= 0 only,
 * the only range its callers pass (x - max of a set): for x >= 11 this returns
 * 0 while hyg_fix100(hyg_exp(x)) stays nonzero up to ln 65536 = 11.09, so a
 * caller with x > 0 must use hyg_fix100(hyg_exp(x)).
 * tests/test_arith.py checks the two forms integer for integer on x <= 0. */
HYG_HD hyg_u128 hyg_exp_fix100_pk(double p, int k, double x) {
  const uint64_t pb = hyg_f64_bits(p);
  const int sh = (int)((pb >> 52) & 0x7ff) - 1023 + k + 48; /* in [-54, 64] on the range */
  const uint64_t m = (pb & 0x000fffffffffffffull) | 0x0010000000000000ull;
  const int shp = sh > 0 ? sh : 0, shn = sh < 0 ? -sh : 0;
  const uint64_t mr = m >> (shn & 63);
  const int in = (x >= -70.0) && (x < 11.0);
  hyg_u128 r;
  r.lo = (!in || shp >= 64) ? 0 : (mr << (shp & 63));
  r.hi = (!in || shp == 0) ? 0 : ((shp >= 64) ? mr : (mr >> ((64 - shp) & 63)));
  return r;
}
HYG_HD hyg_u128 hyg_exp_fix100(double x) {
  const double xc = HYG_FMIN(HYG_FMAX(x, -746.0), 710.0);
  const double kd = HYG_FLOOR(xc * HYG_INV_LN2 + 0.5);
  const int k = (int)kd;
  const double hi = xc - kd * HYG_LN2_HI;
  const double r = HYG_FMA(-kd, HYG_LN2_LO, hi);
  const double p = hyg__exp_poly(r);
  return hyg_exp_fix100_pk(p, k, x);
}

/* value * 2^-scale as a double: the top 53 bits (truncated), exact scaling. */
HYG_HD double hyg_u128_to_f64(hyg_u128 a, int scale) {
  int p; uint64_t top;
  if (a.hi) {
    p = 127 - hyg_clz64(a.hi);
  } else if (a.lo) {
    p = 63 - hyg_clz64(a.lo);
  } else {
    return 0.0;
  }
  if (p <= 52) return (double)a.lo * hyg_pow2(-scale);
  const int sh = p - 52; /* 1..75 */
  if (sh >= 64) top = a.hi >> (sh - 64);
  else top = (a.lo >> sh) | (a.hi << (64 - sh));
  top &= 0x001fffffffffffffull;
  return (double)top * hyg_pow2(sh - scale);
}

/* ------------------------------------------------------------ u192 (F=149) */
typedef struct { uint64_t w0, w1, w2; } hyg_u192;

HYG_HD hyg_u192 hyg_u192_zero(void) { hyg_u192 r; r.w0 = 0; r.w1 = 0; r.w2 = 0; return r; }
#if defined(__HIPCC__)
HYG_HD hyg_u192 hyg_u192_add(hyg_u192 a, hyg_u192 b) {
  unsigned c0, c1, c2, c3, c4, c5;
  const unsigned r0 = __builtin_addc(HYG__L32(a.w0), HYG__L32(b.w0), 0u, &c0);
  const unsigned r1 = __builtin_addc(HYG__H32(a.w0), HYG__H32(b.w0), c0, &c1);
  const unsigned r2 = __builtin_addc(HYG__L32(a.w1), HYG__L32(b.w1), c1, &c2);
  const unsigned r3 = __builtin_addc(HYG__H32(a.w1), HYG__H32(b.w1), c2, &c3);
  const unsigned r4 = __builtin_addc(HYG__L32(a.w2), HYG__L32(b.w2), c3, &c4);
  const unsigned r5 = __builtin_addc(HYG__H32(a.w2), HYG__H32(b.w2), c4, &c5);
  hyg_u192 r; r.w0 = HYG__J64(r0, r1); r.w1 = HYG__J64(r2, r3); r.w2 = HYG__J64(r4, r5); return r;
}
HYG_HD hyg_u192 hyg_u192_sub(hyg_u192 a, hyg_u192 b) { /* a >= b */
  unsigned c0, c1, c2, c3, c4, c5;
  const unsigned r0 = __builtin_subc(HYG__L32(a.w0), HYG__L32(b.w0), 0u, &c0);
  const unsigned r1 = __builtin_subc(HYG__H32(a.w0), HYG__H32(b.w0), c0, &c1);
  const unsigned r2 = __builtin_subc(HYG__L32(a.w1), HYG__L32(b.w1), c1, &c2);
  const unsigned r3 = __builtin_subc(HYG__H32(a.w1), HYG__H32(b.w1), c2, &c3);
  const unsigned r4 = __builtin_subc(HYG__L32(a.w2), HYG__L32(b.w2), c3, &c4);
  const unsigned r5 = __builtin_subc(HYG__H32(a.w2), HYG__H32(b.w2), c4, &c5);
  hyg_u192 r; r.w0 = HYG__J64(r0, r1); r.w1 = HYG__J64(r2, r3); r.w2 = HYG__J64(r4, r5); return r;
}
/* a >= b: no borrow out of a - b */
HYG_HD int hyg_u192_ge(hyg_u192 a, hyg_u192 b) {
  unsigned c0, c1, c2, c3, c4, c5;
  (void)__builtin_subc(HYG__L32(a.w0), HYG__L32(b.w0), 0u, &c0);
  (void)__builtin_subc(HYG__H32(a.w0), HYG__H32(b.w0), c0, &c1);
  (void)__builtin_subc(HYG__L32(a.w1), HYG__L32(b.w1), c1, &c2);
  (void)__builtin_subc(HYG__H32(a.w1), HYG__H32(b.w1), c2, &c3);
  (void)__builtin_subc(HYG__L32(a.w2), HYG__L32(b.w2), c3, &c4);
  (void)__builtin_subc(HYG__H32(a.w2), HYG__H32(b.w2), c4, &c5);
  return (int)(c5 ^ 1u);
}
#else
HYG_HD hyg_u192 hyg_u192_add(hyg_u192 a, hyg_u192 b) {
  hyg_u192 r;
  r.w0 = a.w0 + b.w0;
  const uint64_t c0 = r.w0 < a.w0 ? 1u : 0u;
  const uint64_t t1 = a.w1 + b.w1;
  const uint64_t c1a = t1 < a.w1 ? 1u : 0u;
  r.w1 = t1 + c0;
  const uint64_t c1b = r.w1 < t1 ? 1u : 0u;
  r.w2 = a.w2 + b.w2 + c1a + c1b;
  return r;
}
HYG_HD hyg_u192 hyg_u192_sub(hyg_u192 a, hyg_u192 b) { /* a >= b */
  hyg_u192 r;
  r.w0 = a.w0 - b.w0;
  const uint64_t br0 = a.w0 < b.w0 ? 1u : 0u;
  const uint64_t t1 = a.w1 - b.w1;
  const uint64_t br1a = a.w1 < b.w1 ? 1u : 0u;
  r.w1 = t1 - br0;
  const uint64_t br1b = t1 < br0 ? 1u : 0u;
  r.w2 = a.w2 - b.w2 - br1a - br1b;
  return r;
}
HYG_HD int hyg_u192_ge(hyg_u192 a, hyg_u192 b) {
  if (a.w2 != b.w2) return a.w2 > b.w2;
  if (a.w1 != b.w1) return a.w1 > b.w1;
  return a.w0 >= b.w0;
}
#endif
HYG_HD int hyg_u192_is_zero(hyg_u192 a) { return (a.w0 | a.w1 | a.w2) == 0; }

/* exact integer image of an f32 mass m in [0, 1]: m * 2^149. */
HYG_HD hyg_u192 hyg_fix149f(float m) {
  /* branch-free: the 24-bit significand shifted left by E - 1 (0..126) */
  const uint32_t b = hyg_f32_bits(m);
  const int E = (int)((b >> 23) & 0xff);
  const uint64_t man = b & 0x7fffffu;
  const uint64_t v = (E == 0) ? man : (man | 0x800000u);
  const int sh = (E == 0) ? 0 : E - 1;
  const int s0 = sh & 63;
  const uint64_t lo = v << s0;
  const uint64_t hi = (v >> 1) >> (63 - s0); /* v >> (64 - s0), 0 for s0 = 0 */
  hyg_u192 r;
  r.w0 = (sh < 64) ? lo : 0;
  r.w1 = (sh < 64) ? hi : ((sh < 128) ? lo : 0);
  r.w2 = (sh < 64) ? 0 : ((sh < 128) ? hi : lo);
  const int zero = (b == 0) || (b >> 31);
  r.w0 = zero ? 0 : r.w0;
  r.w1 = zero ? 0 : r.w1;
  r.w2 = zero ? 0 : r.w2;
  return r;
}

/* hyg_fix149f for masses m < 2^-21 (image m 2^149 < 2^128): the two low words
 * of the same integer, the 24-bit significand shifted by E - 1 <= 105. Used by
 * the top-set resampling path for masses it has proved small (tg_kernels.hip);
 * tests/test_arith_carry.py checks it against hyg_fix149f. */
HYG_HD hyg_u128 hyg_fix149f_low128(float m) {
  const uint32_t b = hyg_f32_bits(m);
  const int E = (int)((b >> 23) & 0xff);
  const uint64_t man = b & 0x7fffffu;
  const uint64_t v = (E == 0) ? man : (man | 0x800000u);
  const int sh = (E == 0) ? 0 : E - 1;
  const int s0 = sh & 63;
  const uint64_t lo = v << s0;
  const uint64_t hi = (v >> 1) >> (63 - s0); /* v >> (64 - s0), 0 for s0 = 0 */
  const int zero = (b == 0) || (b >> 31);
  hyg_u128 r;
  r.lo = (zero || sh >= 64) ? 0 : lo;
  r.hi = zero ? 0 : ((sh < 64) ? hi : lo);
  return r;
}

/* value * 2^-149 as a double: top 53 bits (truncated), exactly scaled. */
HYG_HD double hyg_u192_to_f64(hyg_u192 a) {
  int p;
  if (a.w2) p = 191 - hyg_clz64(a.w2);
  else if (a.w1) p = 127 - hyg_clz64(a.w1);
  else if (a.w0) p = 63 - hyg_clz64(a.w0);
  else return 0.0;
  uint64_t top;
  int sh = p - 52;
  if (sh <= 0) {
    top = a.w0; /* p <= 52: value fits in w0 */
    sh = 0;
  } else if (sh < 64) {
    top = (a.w0 >> sh) | (a.w1 << (64 - sh));
  } else if (sh == 64) {
    top = a.w1;
  } else if (sh < 128) {
    top = (a.w1 >> (sh - 64)) | (a.w2 << (128 - sh));
  } else if (sh == 128) {
    top = a.w2;
  } else {
    top = a.w2 >> (sh - 128);
  }
  top &= 0x001fffffffffffffull;
  return (double)top * hyg_pow2(sh - 149);
}

/* ceil(T * R) for an f32 T in [0, 1] and R < 2^151 (R = value * 2^149 as
 * above): the smallest integer C with T <= C / R in exact arithmetic. The
 * systematic resampling comparison T_j <= Q_i = C_i / R
 * (resampling_functions.py:64) is evaluated as C_i >= ceil(T_j * R). */
HYG_HD hyg_u192 hyg_ceil_mul_f32(float T, hyg_u192 R) {
  const uint32_t b = hyg_f32_bits(T);
  hyg_u192 z = hyg_u192_zero();
  if (b == 0 || (b >> 31)) return z;
  const int E = (int)((b >> 23) & 0xff);
  const uint64_t m = (E == 0) ? (uint64_t)(b & 0x7fffffu) : (uint64_t)((b & 0x7fffffu) | 0x800000u);
  const int s = (E == 0) ? 149 : 150 - E; /* T = m * 2^-s, s >= 23 for T <= 1 */
  /* P = m * R (m < 2^24, R < 2^151: P < 2^175) */
  hyg_u192 P;
  const uint64_t l0 = m * R.w0, h0 = hyg_mulhi64(m, R.w0);
  const uint64_t l1 = m * R.w1, h1 = hyg_mulhi64(m, R.w1);
  const uint64_t l2 = m * R.w2;
  P.w0 = l0;
  P.w1 = h0 + l1;
  const uint64_t c1 = P.w1 < h0 ? 1u : 0u;
  P.w2 = h1 + l2 + c1;
  /* ceil(P / 2^s) = (P + 2^s - 1) >> s, s in [23, 149] */
  hyg_u192 bias = z;
  if (s < 64) bias.w0 = (1ull << s) - 1ull;
  else if (s < 128) { bias.w0 = ~0ull; bias.w1 = (s == 64) ? 0 : ((1ull << (s - 64)) - 1ull); }
  else { bias.w0 = ~0ull; bias.w1 = ~0ull; bias.w2 = (s == 128) ? 0 : ((1ull << (s - 128)) - 1ull); }
  const hyg_u192 Q = hyg_u192_add(P, bias);
  hyg_u192 r;
  if (s < 64) {
    r.w0 = (Q.w0 >> s) | (Q.w1 << (64 - s));
    r.w1 = (Q.w1 >> s) | (Q.w2 << (64 - s));
    r.w2 = Q.w2 >> s;
  } else if (s == 64) {
    r.w0 = Q.w1; r.w1 = Q.w2; r.w2 = 0;
  } else if (s < 128) {
    const int t = s - 64;
    r.w0 = (Q.w1 >> t) | (Q.w2 << (64 - t));
    r.w1 = Q.w2 >> t;
    r.w2 = 0;
  } else if (s == 128) {
    r.w0 = Q.w2; r.w1 = 0; r.w2 = 0;
  } else {
    r.w0 = Q.w2 >> (s - 128); r.w1 = 0; r.w2 = 0;
  }
  return r;
}

/* hyg_ceil_mul_f32 without branches (the same integer: tests/test_arith_carry.py):
 * the kernels evaluate it for a wave of systematic targets whose exponents
 * differ lane to lane, so the branch form runs several of its shift paths
 * one after another. m R from 24 x 32-bit partial products; the bias and the
 * shift by s = 64 q + sb by word selects and one funnel shift. */
HYG_HD hyg_u192 hyg_ceil_mul_f32_bf(float T, hyg_u192 R) {
  const uint32_t b = hyg_f32_bits(T);
  const int E = (int)((b >> 23) & 0xff);
  const uint64_t m = (E == 0) ? (uint64_t)(b & 0x7fffffu) : (uint64_t)((b & 0x7fffffu) | 0x800000u);
  const int s = (E == 0) ? 149 : 150 - E; /* in [23, 149] for 0 < T <= 1 */
  /* m w = (m w_lo) + (m w_hi) 2^32 for each 64-bit word w of R (m < 2^24) */
  const uint64_t a0 = m * (R.w0 & 0xffffffffu), b0 = m * (R.w0 >> 32);
  const uint64_t a1 = m * (R.w1 & 0xffffffffu), b1 = m * (R.w1 >> 32);
  const uint64_t a2 = m * (R.w2 & 0xffffffffu), b2 = m * (R.w2 >> 32);
  const uint64_t l0 = a0 + (b0 << 32), h0 = (b0 >> 32) + (l0 < a0 ? 1u : 0u);
  const uint64_t l1 = a1 + (b1 << 32), h1 = (b1 >> 32) + (l1 < a1 ? 1u : 0u);
  const uint64_t l2 = a2 + (b2 << 32);
  hyg_u192 P;
  P.w0 = l0;
  P.w1 = h0 + l1;
  P.w2 = h1 + l2 + (P.w1 < h0 ? 1u : 0u);
  /* ceil(P / 2^s) = (P + 2^s - 1) >> s */
  const int q = s >> 6, sb = s & 63;
  const uint64_t part = (sb == 0) ? 0 : ((1ull << (sb & 63)) - 1ull);
  hyg_u192 bias;
  bias.w0 = (q > 0) ? ~0ull : part;
  bias.w1 = (q > 1) ? ~0ull : ((q == 1) ? part : 0);
  bias.w2 = (q == 2) ? part : 0;
  const hyg_u192 Q = hyg_u192_add(P, bias);
  const uint64_t x0 = (q == 0) ? Q.w0 : ((q == 1) ? Q.w1 : Q.w2);
  const uint64_t x1 = (q == 0) ? Q.w1 : ((q == 1) ? Q.w2 : 0);
  const uint64_t x2 = (q == 0) ? Q.w2 : 0;
  const int rs = (64 - sb) & 63;
  hyg_u192 r;
  r.w0 = (sb == 0) ? x0 : ((x0 >> sb) | (x1 << rs));
  r.w1 = (sb == 0) ? x1 : ((x1 >> sb) | (x2 << rs));
  r.w2 = (sb == 0) ? x2 : (x2 >> sb);
  const int zero = (b == 0) || (b >> 31);
  r.w0 = zero ? 0 : r.w0;
  r.w1 = zero ? 0 : r.w1;
  r.w2 = zero ? 0 : r.w2;
  return r;
}

/* ------------------------------------------------------- Philox4x64-10 */
typedef struct { uint64_t v[4]; } hyg_ph4;

HYG_HD hyg_ph4 hyg_philox4x64(uint64_t c0, uint64_t c1, uint64_t c2, uint64_t c3,
                              uint64_t k0, uint64_t k1) {
  hyg_ph4 x;
  x.v[0] = c0; x.v[1] = c1; x.v[2] = c2; x.v[3] = c3;
  for (int round = 0; round < 10; ++round) {
    const uint64_t M0 = 0xD2E7470EE14C6C93ull, M1 = 0xCA5A826395121157ull;
    const uint64_t hi0 = hyg_mulhi64(M0, x.v[0]), lo0 = M0 * x.v[0];
    const uint64_t hi1 = hyg_mulhi64(M1, x.v[2]), lo1 = M1 * x.v[2];
    hyg_ph4 y;
    y.v[0] = hi1 ^ x.v[1] ^ k0;
    y.v[1] = lo1;
    y.v[2] = hi0 ^ x.v[3] ^ k1;
    y.v[3] = lo0;
    x = y;
    k0 += 0x9E3779B97F4A7C15ull;
    k1 += 0xBB67AE8584CAA73Bull;
  }
  return x;
}

/* Random streams (counter word 0). */
#define HYG_RNG_PHANTOM 1u     /* initial phantom regime (case_control_distributions.py:67-74) */
#define HYG_RNG_SYSTEMATIC 2u  /* systematic residual U (resampling_functions.py:58) */
#define HYG_RNG_MULTINOMIAL 3u /* unbiased-fallback categorical draws (resampling_functions.py:46) */
#define HYG_RNG_BACKWARD 4u    /* backward-simulation categorical draws (filter_and_smoother_algorithm.py:385,426) */

/* 64 random bits number `index` of (stream, step) for chain (seed, chain_id). */
HYG_HD uint64_t hyg_rand64(uint64_t seed, uint64_t chain_id, uint32_t stream, uint64_t step, uint64_t index) {
  const hyg_ph4 r = hyg_philox4x64((uint64_t)stream, step, index >> 2, 0, seed, chain_id);
  /* value selects, not r.v[index & 3]: a dynamic index would put r in GPU scratch memory */
  const unsigned q = (unsigned)(index & 3);
  const uint64_t lo = (q & 1) ? r.v[1] : r.v[0], hi = (q & 1) ? r.v[3] : r.v[2];
  return (q & 2) ? hi : lo;
}

/* f32 uniform on [0, 1) from 24 random bits (exact). */
HYG_HD float hyg_u01f(uint64_t r) { return (float)(r >> 40) * 5.9604644775390625e-08f; }

/* floor(r * total / 2^64): an integer uniform on [0, total) for total < 2^114. */
HYG_HD hyg_u128 hyg_scale_target(uint64_t r, hyg_u128 total) {
  hyg_u128 t;
  t.lo = r * total.hi;
  t.hi = hyg_mulhi64(r, total.hi);
  hyg_u128 add; add.lo = hyg_mulhi64(r, total.lo); add.hi = 0;
  return hyg_u128_add(t, add);
}

/* ------------------------------------------------------ packed particle */
/* bits [0,24) d_ctrl, [24,48) d_case, [48,54) r_ctrl, [54,60) r_case, [60] merged */
#define HYG_DMAX 0xffffff
HYG_HD uint64_t hyg_st_pack(int m, int dc, int rc, int dk, int rk) {
  return (uint64_t)(uint32_t)dc | ((uint64_t)(uint32_t)dk << 24) | ((uint64_t)rc << 48) |
         ((uint64_t)rk << 54) | ((uint64_t)m << 60);
}
HYG_HD int hyg_st_m(uint64_t s) { return (int)((s >> 60) & 1u); }
HYG_HD int hyg_st_dc(uint64_t s) { return (int)(s & 0xffffffu); }
HYG_HD int hyg_st_dk(uint64_t s) { return (int)((s >> 24) & 0xffffffu); }
HYG_HD int hyg_st_rc(uint64_t s) { return (int)((s >> 48) & 63u); }
HYG_HD int hyg_st_rk(uint64_t s) { return (int)((s >> 54) & 63u); }

#endif /* HYG_ARITH_H */
