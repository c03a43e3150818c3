/*
 * hyg_sg_pe.h -- single-group online parameter estimation:
 * the theta-dependent model quantities, rebuilt every time theta moves, and
 * the gradient-ascent / ADAM step. Shared, operation for operation, by the
 * CPU oracle (oracle/sg_oracle.c) and the chain kernel
 * (hygeia_amd/csrc/sg_kernels.hip), so the two stay bit-identical.
 *
 * Reference: src/single_group/src/cpp/
 *   singleGroup.h:197-270   setUnknownParameters (P rows = exp(normaliseExp(theta block)),
 *                           omega = inverseLogit)
 *   singleGroup.h:271-335   extendAuxiliaryQuantities (NegBin hazard rho(d), exit status,
 *                           d log rho / d theta_omega)
 *   singleGroup.h:641-717   evaluateGradThetaLogTransitionDensity
 *   misc/GradientAscent.h:62-155  ADAM / plain gradient ascent
 *   algorithms/OnlineParameterEstimation.h:42-176  phi recursion, update every c steps
 *   misc/misc.h:34-37,92-95,785-790  inverseLogit, gradLogitEvaluatedAtInverseLogit, normaliseExp
 *
 * Arithmetic contract: hyg_exp / hyg_log of include/hyg_arith.h, IEEE
 * + - * / sqrt, no FMA contraction; sums in the reference's sequential order.
 * The lgamma part of the NegBin log-pmf does not depend on theta (kappa is
 * fixed, the pipeline default --is_kappa_fixed TRUE, or estimated and then
 * never moved, see below) and is tabulated once on the host with libm lgamma
 * (hyg_sgpe_lgk_fill); the ADAM step sizes and bias corrections are libm pow
 * values tabulated once on the host (hyg_sgpe_steps_fill), as the reference
 * computes them.
 *
 * Estimated kappa (--is_kappa_fixed FALSE): theta gains K entries log kappa_r
 * (singleGroup.h:114-116,218-223, dim K (K + 1)). The reference's gradient
 * then writes d log rho / d theta_kappa into the OMEGA index
 * (singleGroup.h:664-668; its kappa index only ever receives
 * -grad(idxKappa) rho / (1 - rho) with grad(idxKappa) = 0, :688-692), and that
 * kappa derivative's bigH recursion adds the OMEGA gradient of bigH
 * (:329). Restated as written: the omega coordinate carries
 *   gK(d) = kappa (psi(x + kappa) - psi(kappa) - log(1 - omega))       (:328)
 *         + gKbigH(d - 1) / (1 - bigH(d - 1)),
 *   gKbigH(d) = gObigH(d - 1) + h(d) gK_h(d)                            (:329-330)
 * (x = d + 1 - u), and the kappa coordinates' score is exactly 0 at every
 * step, so ADAM / gradient ascent leave log kappa where it started (theta +
 * 0) and kappa = exp(theta_kappa) of the initial theta throughout. The digamma
 * differences psi(x + kappa) - psi(kappa) are theta-free and tabulated once
 * on the host (hyg_sgpe_dgk_fill, hyg_digamma below; the reference calls R's
 * digamma: parity at the last bits unpinned, tests check scipy to 1e-14).
 *
 * Hazard table semantics: rows d = d_prev - 1 = 0 .. L_r - 1 per regime, where
 * L_r = the exit onset + 1 (the first d with exitStatus) or the computed
 * length; lookups past the exit onset use the onset row. Past the onset the
 * reference's rows differ only in d log rho / d theta_omega, which only
 * particles of weight 0 (their continuation density is -inf) can reach, so
 * every weighted quantity is unchanged.
 */
#ifndef HYG_SG_PE_H
#define HYG_SG_PE_H

#include <math.h>
#include <stdint.h>

#include "hyg_arith.h"
#include "hygeia_amd.h"

#define HYG_SGPE_DCAP 65536 /* hazard rows per regime (longest sojourn a chain may reach) */
#define HYG_SGPE_EXIT_H 0.99999 /* bigH_[r][d-1] = 0.99999 at the exit onset (singleGroup.h:306) */

/* theta-dependent per-regime quantities (setUnknownParameters) */
typedef struct {
  double P[HYG_KMAX * HYG_KMAX];    /* P[r][r'], diagonal 0 */
  double logP[HYG_KMAX * HYG_KMAX]; /* log P, diagonal -inf */
  double omega[HYG_KMAX];
  double gl[HYG_KMAX];     /* gradLogitEvaluatedAtInverseLogit(omega_r) = 2 + e^-omega + e^omega */
  double log1mw[HYG_KMAX]; /* log(1 - omega_r) */
  double logw[HYG_KMAX];   /* log(omega_r) */
} hyg_sgpe_model;

/* one regime's row of P and its omega from theta (singleGroup.h:204-222) */
HYG_HD void hyg_sgpe_set_regime(const double* theta, int K, int r, hyg_sgpe_model* m) {
  const double* x = theta + r * (K - 1);
  double mx = HYG_NINF;
  for (int i = 0; i < K - 1; ++i) mx = (x[i] > mx) ? x[i] : mx;
  double s = 0.0;
  for (int i = 0; i < K - 1; ++i) s = s + hyg_exp(x[i] - mx);
  const double lz = mx + hyg_log(s);
  int i = 0;
  for (int r1 = 0; r1 < K; ++r1) {
    if (r1 == r) {
      m->P[r * K + r1] = 0.0;
      m->logP[r * K + r1] = HYG_NINF;
      continue;
    }
    const double p = hyg_exp(x[i++] - lz);
    m->P[r * K + r1] = p;
    m->logP[r * K + r1] = hyg_log(p);
  }
  const double w = 1.0 / (1.0 + hyg_exp(-1.0 * theta[K * (K - 1) + r]));
  m->omega[r] = w;
  m->gl[r] = (2.0 + hyg_exp(-w)) + hyg_exp(w);
  m->log1mw[r] = hyg_log(1.0 - w);
  m->logw[r] = hyg_log(w);
}

/* Hazard row inputs at d (parallel over d): h = NegBin pmf of x = d + 1 - u
 * (misc.h:673-693 evaluateLogNegativeBinomialDensity, lgk = lgamma(x + kappa)
 * - lgamma(kappa) - lgamma(x + 1)), g = d log h / d theta_omega
 * (singleGroup.h:322) and, when kappa is estimated (dgk != NULL: dgk[x] =
 * psi(x + kappa) - psi(kappa)), gk = d log h / d theta_kappa (:328). Rows
 * d < u - 1 are 0. */
HYG_HD void hyg_sgpe_hazard_point(const hyg_sgpe_model* m, int r, int d, int u, double kappa, const double* lgk,
                                  const double* dgk, double* h, double* g, double* gk) {
  if (d < u - 1) {
    *h = 0.0;
    *g = 0.0;
    if (dgk) *gk = 0.0;
    return;
  }
  const int x = d + 1 - u;
  const double w = m->omega[r];
  double lnb;
  if (w == 0.0) lnb = (x == 0) ? 0.0 : HYG_NINF;
  else lnb = (lgk[x] + kappa * m->log1mw[r]) + (double)x * m->logw[r];
  *h = hyg_exp(lnb);
  *g = ((double)x / w - kappa / (1.0 - w)) * m->gl[r];
  if (dgk) *gk = kappa * (dgk[x] - m->log1mw[r]);
}

/* Sequential part of extendAuxiliaryQuantities (singleGroup.h:298-331) for one
 * regime over rows 0 .. L-1: records per row the bigH[d-1] and gradBigH[d-1]
 * its rho and d log rho use, and the exit status. Stops at the exit onset.
 * With gk (kappa estimated) the recorded gradBigH[d-1] is the kappa one,
 * gradThetaKappaBigH[d] = gradThetaOmegaBigH[d-1] + h[d] gk[d] (:329), the
 * omega one still accumulated beside it. Returns L_r (rows valid). */
HYG_HD int hyg_sgpe_hazard_scan(const double* h, const double* g, const double* gk, int u, int L, double* Hm1s,
                                double* gm1s, uint8_t* ex) {
  double Hm1 = 0.0, gm1 = 0.0, gkm1 = 0.0;
  /* the inputs are read 16 rows ahead of the sequential recursion (on the GPU
   * one lane per regime runs it: the loads then overlap) */
  for (int d0 = 0; d0 < L; d0 += 16) {
    double hb[16], gb[16], kb[16];
    for (int i = 0; i < 16; ++i) {
      const int d = d0 + i;
      hb[i] = (d < L) ? h[d] : 0.0;
      gb[i] = (d < L) ? g[d] : 0.0;
      kb[i] = (gk && d < L) ? gk[d] : 0.0;
    }
    for (int i = 0; i < 16; ++i) {
      const int d = d0 + i;
      if (d >= L) break;
      if (d < u - 1) {
        Hm1s[d] = 0.0;
        gm1s[d] = 0.0;
        ex[d] = 0;
        continue;
      }
      if (Hm1 >= 1.0) { /* exit onset: bigH[d-1] is overwritten with 0.99999 */
        Hm1s[d] = HYG_SGPE_EXIT_H;
        gm1s[d] = gk ? gkm1 : gm1;
        ex[d] = 1;
        return d + 1;
      }
      Hm1s[d] = Hm1;
      gm1s[d] = gk ? gkm1 : gm1;
      ex[d] = 0;
      gkm1 = gm1 + hb[i] * kb[i];
      Hm1 = Hm1 + hb[i];
      gm1 = gm1 + hb[i] * gb[i];
    }
  }
  return L;
}

/* One finished hazard row (parallel over d), g / gm1 the omega (kappa fixed)
 * or the kappa (kappa estimated) derivative inputs:
 *   base  = log rho (the change-point density before log P), 0 after the exit
 *   cont  = log(1 - rho) if !exit && rho <= 1, else -inf   (singleGroup.h:569-608)
 *   gomg  = the omega coordinate's d log rho                (:324 / :330 via :664-668)
 *   gcont = the continuation's gradient entry -gomg rho / (1 - rho) if
 *           !exit && rho < 1, else 0                        (:683-699) */
typedef struct {
  double base, cont, gomg, gcont;
} hyg_sgpe_row;

HYG_HD hyg_sgpe_row hyg_sgpe_hazard_row(double h, double g, double Hm1, double gm1, int exd, int d, int u) {
  hyg_sgpe_row o;
  double rho, gomg;
  if (d < u - 1) {
    rho = 0.0;
    gomg = 0.0;
  } else {
    rho = exd ? 1.0 : h / (1.0 - Hm1);
    gomg = g + gm1 / (1.0 - Hm1);
  }
  o.base = exd ? 0.0 : hyg_log(rho);
  o.cont = (!exd && rho <= 1.0) ? hyg_log(1.0 - rho) : HYG_NINF;
  o.gomg = gomg;
  o.gcont = (!exd && rho < 1.0) ? ((-gomg) * rho) / (1.0 - rho) : 0.0;
  return o;
}

/* The fresh particle's phi (OnlineParameterEstimation.h:136-144) sums K_q(n)
 * (phi_n + grad_qn) over the previous particles n. The sum is taken in C
 * fixed chunks of 256 / C rows, each summed in n order, the chunk sums then
 * added left to right (C = 1: the reference's sequential order). C spreads
 * the K x K^2 sums over the threads of the chain's workgroup (512 threads
 * for K <= 8, 256 above): C = the largest power of two <= threads / K^3,
 * at most 8. */
HYG_HD int hyg_sgpe_fresh_chunks(int K) {
  const int nb = (K <= 8) ? 512 : 256;
  const int c = nb / (K * K * K);
  return c >= 8 ? 8 : (c >= 4 ? 4 : (c >= 2 ? 2 : 1));
}

/* ADAM / gradient-ascent step sizes (GradientAscent.h:124-127,147): per
 * iteration i = 0, 1, ...: lr_i = factor / (i + 1)^exponent, and the bias
 * corrections 1 - beta1^(i+1), 1 - beta2^(i+1). Host only (libm pow). */
typedef struct {
  double lr, c1, c2;
} hyg_sgpe_step;

typedef struct hyg_sgpe_consts {
  int32_t K, u, dim, every; /* dim = theta length: K^2 (kappa fixed) or K (K + 1); every = nStepsWithoutParameterUpdate */
  int32_t use_adam, normalise;
  int32_t kest, pad_;       /* kest: kappa estimated (is_kappa_fixed = 0) */
  double beta1, beta2, eps;
  double kappa[HYG_KMAX];
} hyg_sgpe_consts;

/* one coordinate of the update (GradientAscent.h:82-105,147): `grad` is
 * gradientCurr - gradientPrev of the filtered score, `l1` its L1 norm (used
 * when !use_adam && normalise), s the step sizes of this iteration. Scalars
 * only (no address of a kernel argument is taken on the device). Returns
 * the new theta_j. */
HYG_HD double hyg_sgpe_update(int use_adam, int normalise, double beta1, double beta2, double eps, double lr,
                              double c1, double c2, double theta, double grad, double l1, double* am, double* av) {
  if (use_adam) {
    const double m = beta1 * (*am) + (1.0 - beta1) * grad;
    const double v = beta2 * (*av) + ((1.0 - beta2) * grad) * grad;
    *am = m;
    *av = v;
    return theta + ((lr * m) * (1.0 / (sqrt(v / c2) + eps))) / c1;
  }
  if (normalise) return theta + lr * (grad / (l1 != 0.0 ? l1 : 1.0)); /* arma::normalise leaves a zero vector */
  return theta + lr * grad;
}

/* ---- host-only tables */
static inline void hyg_sgpe_steps_fill(const hyg_sg_pe_params* pe, int n, hyg_sgpe_step* s) {
  const double b1 = 0.9, b2 = 0.999;
  for (int i = 0; i < n; ++i) {
    s[i].lr = pe->learning_rate_factor / pow((double)i + 1.0, pe->learning_rate_exponent);
    s[i].c1 = 1.0 - pow(b1, (double)(i + 1));
    s[i].c2 = 1.0 - pow(b2, (double)(i + 1));
  }
}
/* lgk[r][x] = lgamma(x + kappa_r) - lgamma(kappa_r) - lgamma(x + 1), x < n */
static inline void hyg_sgpe_lgk_fill(const double* kappa, int K, int n, double* lgk) {
  for (int r = 0; r < K; ++r)
    for (int x = 0; x < n; ++x)
      lgk[(size_t)r * n + x] = (lgamma((double)x + kappa[r]) - lgamma(kappa[r])) - lgamma((double)x + 1.0);
}
/* psi(x), x > 0: the recurrence psi(x) = psi(x + 1) - 1/x up to x >= 10, then
 * the asymptotic series log x - 1/(2x) - sum_k B_2k / (2k x^2k) to k = 8
 * (truncation < 1e-17 relative at x >= 10). Host only. */
static inline double hyg_digamma(double x) {
  if (!(x > 0.0)) return NAN;
  double acc = 0.0;
  while (x < 10.0) {
    acc -= 1.0 / x;
    x += 1.0;
  }
  const double z = 1.0 / (x * x);
  /* B_2k / (2k): 1/12, -1/120, 1/252, -1/240, 1/132, -691/32760, 1/12, -3617/8160 */
  const double s = z * (1.0 / 12 - z * (1.0 / 120 - z * (1.0 / 252 - z * (1.0 / 240 - z * (1.0 / 132 -
                   z * (691.0 / 32760 - z * (1.0 / 12 - z * (3617.0 / 8160))))))));
  return acc + ((log(x) - 0.5 / x) - s);
}
/* dgk[r][x] = psi(x + kappa_r) - psi(kappa_r), x < n (singleGroup.h:328's digamma difference) */
static inline void hyg_sgpe_dgk_fill(const double* kappa, int K, int n, double* dgk) {
  for (int r = 0; r < K; ++r) {
    const double pk = hyg_digamma(kappa[r]);
    for (int x = 0; x < n; ++x) dgk[(size_t)r * n + x] = hyg_digamma((double)x + kappa[r]) - pk;
  }
}
static inline int hyg_sgpe_consts_make(const hyg_sg_params* p, const hyg_sg_pe_params* pe, hyg_sgpe_consts* c) {
  const int K = p->n_regimes;
  if (pe->n_steps_without_update < 1) return HYG_EINVAL;
  if (!(pe->learning_rate_factor == pe->learning_rate_factor) ||
      !(pe->learning_rate_exponent == pe->learning_rate_exponent))
    return HYG_EINVAL;
  c->K = K;
  c->u = p->minimum_duration;
  c->kest = p->is_kappa_fixed ? 0 : 1;
  c->dim = c->kest ? K * (K + 1) : K * K;
  c->every = pe->n_steps_without_update;
  c->use_adam = pe->use_adam ? 1 : 0;
  c->normalise = pe->normalise_gradients ? 1 : 0;
  c->beta1 = 0.9;
  c->beta2 = 0.999;
  c->eps = exp(-8.0 * log(10.0)); /* GradientAscent.h:60 */
  /* kappa_r = exp(theta_kappa_r) when estimated (singleGroup.h:218-223), as hyg_sg_derive */
  for (int r = 0; r < K; ++r) c->kappa[r] = c->kest ? exp(p->theta[K * K + r]) : p->kappa[r];
  for (int r = 0; r < K; ++r)
    if (!(c->kappa[r] > 0.0) || !isfinite(c->kappa[r])) return HYG_EINVAL;
  return HYG_OK;
}
/* number of theta rows a chain of T sites reports: the initial theta and
 * one row per update at t = every, 2 every, ... <= T - 1 */
static inline int64_t hyg_sgpe_theta_rows(int64_t T, int every) { return T >= 1 ? 1 + (T - 1) / every : 0; }

#endif /* HYG_SG_PE_H */
