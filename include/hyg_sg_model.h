/*
 * hyg_sg_model.h -- host-side model construction of the single-group engine,
 * shared by the CPU oracle (oracle/sg_oracle.c) and the C ABI (capi.cpp).
 *
 * Reference: src/single_group/src/cpp/singleGroup.h
 *   ModelParameters::setKnownParameters   :173-195  (vartheta: u, K, alpha, beta, isKappaFixed, kappa)
 *   ModelParameters::setUnknownParameters :197-270  (theta -> P rows by softmax, omega, kappa)
 *   extendAuxiliaryQuantities             :271-335  (NegBin hazard rho(d) with exit status)
 *   Model::evaluateLogTransitionDensity   :569-608
 *   misc.h:673-693 evaluateLogNegativeBinomialDensity (Wikipedia parametrisation)
 *
 * The tables are built in double on the host (libm lgamma/exp/log, as the
 * reference) and used unchanged by both the oracle and the GPU kernels.
 */
#ifndef HYG_SG_MODEL_H
#define HYG_SG_MODEL_H

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "hygeia_amd.h"

typedef struct {
  int32_t K, u, Nmax, is_kappa_fixed;
  double alpha[HYG_KMAX], beta[HYG_KMAX], kappa[HYG_KMAX], omega[HYG_KMAX];
  double logP[HYG_KMAX * HYG_KMAX]; /* log P[r_prev][r_curr], diagonal -inf */
  double log_K;                     /* log K: the initial density is -log K (singleGroup.h:556-565) */
  double epsilon;
} hyg_sg_consts;

/* softmax of a block in log space as misc.h normaliseExp: x - (max + log sum exp(x - max)) */
static inline void hyg__sg_normalise_exp(const double* x, int n, double* out) {
  double mx = -INFINITY;
  for (int i = 0; i < n; ++i) if (x[i] > mx) mx = x[i];
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += exp(x[i] - mx);
  const double lz = mx + log(s);
  for (int i = 0; i < n; ++i) out[i] = x[i] - lz;
}

static inline int hyg_sg_derive(const hyg_sg_params* p, hyg_sg_consts* c) {
  memset(c, 0, sizeof(*c));
  const int K = p->n_regimes;
  if (K < 2 || K > HYG_KMAX) return HYG_EINVAL;
  if (p->minimum_duration < 1 || p->num_particles_max <= K || p->num_particles_max > 1024) return HYG_EINVAL;
  if (p->resample_type != 2) return HYG_EUNSUPPORTED;
  const int need = K * (K - 1) + K + (p->is_kappa_fixed ? 0 : K);
  if (p->theta_len != need) return HYG_EINVAL;
  if (!(p->epsilon > 0.0)) return HYG_EINVAL;
  c->K = K;
  c->u = p->minimum_duration;
  c->Nmax = p->num_particles_max;
  c->is_kappa_fixed = p->is_kappa_fixed ? 1 : 0;
  c->epsilon = p->epsilon;
  c->log_K = log((double)K);
  for (int r = 0; r < K; ++r) {
    c->alpha[r] = p->alpha[r];
    c->beta[r] = p->beta[r];
    if (!(c->alpha[r] > 0.0) || !(c->beta[r] > 0.0) || !isfinite(c->alpha[r]) || !isfinite(c->beta[r]))
      return HYG_EINVAL;
  }
  /* P: row r = exp(normaliseExp(theta block r)) with 0 inserted at the diagonal (:204-214) */
  for (int r = 0; r < K; ++r) {
    double lz[HYG_KMAX];
    hyg__sg_normalise_exp(p->theta + r * (K - 1), K - 1, lz);
    int i = 0;
    for (int r1 = 0; r1 < K; ++r1) {
      if (r1 == r) { c->logP[r * K + r1] = -INFINITY; continue; }
      c->logP[r * K + r1] = log(exp(lz[i++]));
    }
  }
  for (int r = 0; r < K; ++r) {
    const double x = p->theta[K * (K - 1) + r];
    c->omega[r] = exp(x) / (1.0 + exp(x)); /* inverseLogit (misc.h) */
    if (!(c->omega[r] > 0.0 && c->omega[r] < 1.0)) return HYG_EINVAL;
    c->kappa[r] = p->is_kappa_fixed ? p->kappa[r] : exp(p->theta[K * K + r]);
    if (!(c->kappa[r] > 0.0)) return HYG_EINVAL;
  }
  return HYG_OK;
}

static inline double hyg_sg_lognb(double x, double size, double prob) {
  if (x == 0.0 && prob == 0.0) return 0.0;
  if (prob == 0.0) return -INFINITY;
  return lgamma(x + size) - lgamma(size) - lgamma(x + 1.0) + size * log(1.0 - prob) + x * log(prob);
}

/* Hazard rows for d_prev = 1 .. dcap (index d = d_prev - 1), per regime:
 *   hz[(r*dcap + d)*2 + 0] = log rho  (change point, before adding log P; used when !exit)
 *   hz[(r*dcap + d)*2 + 1] = log(1 - rho) if !exit && rho <= 1, else -inf (continuation)
 *   ex[r*dcap + d] = exit status (change point density = log P alone)
 * following extendAuxiliaryQuantities (:271-335). The rows are constant from
 * the first exit on, so lookups clamp d_prev to dcap. Returns dcap (>= 2) or
 * -1 if no exit is reached by max_duration (then dcap = max_duration + 1). */
static inline int hyg_sg_hazard_len(const hyg_sg_consts* c, int max_duration) {
  int dcap = 2;
  for (int r = 0; r < c->K; ++r) {
    double Hprev = 0.0;
    int exitp = 0, d;
    const int lim = max_duration + 1;
    for (d = c->u - 1; d < lim; ++d) {
      const double h = exp(hyg_sg_lognb((double)(d + 1 - c->u), c->kappa[r], c->omega[r]));
      if (exitp || Hprev >= 1.0) { exitp = 1; break; }
      Hprev = Hprev + h;
    }
    const int len = (d < lim ? d + 1 : lim);
    if (len + 1 > dcap) dcap = len + 1;
  }
  return dcap;
}
static inline void hyg_sg_hazard_fill(const hyg_sg_consts* c, int dcap, double* hz, uint8_t* ex) {
  const int K = c->K, u = c->u;
  for (int r = 0; r < K; ++r) {
    double* row = hz + (size_t)r * dcap * 2;
    uint8_t* er = ex + (size_t)r * dcap;
    double Hm1 = 0.0; /* bigH[d-1] */
    int exm1 = 0;     /* exitStatus[d-1] */
    for (int d = 0; d < dcap; ++d) {
      double rho;
      int exd;
      if (d < u - 1) {
        rho = 0.0;
        exd = 0;
        Hm1 = 0.0;
      } else {
        const double h = exp(hyg_sg_lognb((double)(d + 1 - u), c->kappa[r], c->omega[r]));
        if (exm1 || Hm1 >= 1.0) {
          rho = 1.0;
          exd = 1;
        } else {
          rho = h / (1.0 - Hm1);
          Hm1 = Hm1 + h;
          exd = 0;
        }
      }
      row[2 * d + 0] = log(rho);
      row[2 * d + 1] = (!exd && rho <= 1.0) ? log(1.0 - rho) : -INFINITY;
      er[d] = (uint8_t)exd;
      exm1 = exd;
    }
  }
}

/* Beta-Binomial lgamma tables (same layout as hyg_bb_tables of hyg_model.h) */
static inline void hyg_sg_bb_tables(const hyg_sg_consts* c, int nmax, double* lf, double* lg, double* cst) {
  const int L = nmax + 1;
  for (int j = 0; j < L; ++j) lf[j] = lgamma((double)j + 1.0);
  for (int r = 0; r < c->K; ++r) {
    const double a = c->alpha[r], b = c->beta[r];
    for (int j = 0; j < L; ++j) {
      lg[(size_t)(r * 3 + 0) * L + j] = lgamma((double)j + a);
      lg[(size_t)(r * 3 + 1) * L + j] = lgamma((double)j + b);
      lg[(size_t)(r * 3 + 2) * L + j] = lgamma((double)j + a + b);
    }
    cst[r] = lgamma(a + b) - lgamma(a) - lgamma(b);
  }
}

#endif /* HYG_SG_MODEL_H */
