#define _DEFAULT_SOURCE 1 /* lgamma_r */
/*
 * sg_oracle.c -- CPU oracle of the single-group engine (TEST INFRASTRUCTURE).
 *
 * Plain-C restatement of src/single_group/src/cpp (C++/Armadillo, R RNG):
 *   - SMC for the change-point model        algorithms/Smc.h:114-188 (initialise),
 *                                           :190-286 (iterate), :406-450 (resampleCp),
 *                                           :504-522 (sampleParticlesCp), :536-574
 *                                           (computeWeightsCp), :576-579 (selfNormalise)
 *   - optimal finite-state resampling        misc/resample.h:289-409, systematicBase :85-117
 *   - backward kernels                       algorithms/Smc.h:288-326
 *   - online marginal smoothing (epsilon)    algorithms/OnlineMarginalSmoothing.h:52-255
 *   - driver                                 algorithms/OnlineCombinedInference.h:48-118
 *   - model                                  singleGroup.h:556-627 (initial, transition,
 *                                            observation densities), include/hyg_sg_model.h
 * with the arithmetic contract of include/hyg_arith.h: every sum of weights,
 * masses or products is an exact fixed-point sum (u128, 2^-100 units), the
 * elementary functions are hyg_exp / hyg_log, the uniform of the systematic
 * draw comes from Philox (stream HYG_RNG_SG_SYSTEMATIC). Against the reference
 * (R RNG, sequential double sums, not buildable here: RcppArmadillo absent)
 * the results are "parity unpinned"; tests/test_sg_oracle.py pins the model
 * tables and the statistical behaviour. Only used by tests/ and bench.py.
 *
 * Online parameter estimation (oracle_sg_chain_pe): the phi
 * recursion of OnlineParameterEstimation.h:118-150 (continuing particle n:
 * phi_anc + grad; fresh particle (1, q): sum_n K_q(n) (phi_n + grad_qn) in n
 * order), the filtered score sum_n W_n phi_n (Smc.h:341-350) every
 * `every` steps, the ADAM / gradient step (GradientAscent.h:82-155) and the
 * rebuild of P, omega and the hazard tables from the new theta
 * (include/hyg_sg_pe.h, shared with the kernel). With kappa estimated the
 * K (K + 1) coordinates are carried literally, the kappa index's gradient
 * entries as singleGroup.h:664-692 write them (the kernel drops the
 * identically-zero kappa recursion; the GPU tests compare the two).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/hyg_arith.h"
#include "../include/hyg_sg_model.h"
#include "../include/hyg_sg_pe.h"

#define HYG_RNG_SG_SYSTEMATIC 5

typedef struct {
  hyg_sg_consts c;
  int dcap;
  double* hz;
  uint8_t* ex;
  /* online parameter estimation: theta-dependent model and hazard rows */
  int pe;
  hyg_sgpe_consts pc;
  hyg_sgpe_model pm;
  int rcap;              /* rows per regime: min(T + 1, HYG_SGPE_DCAP) */
  int Lr[HYG_KMAX], exited[HYG_KMAX];
  int overflow;          /* a lookup beyond the rows of a regime that has not exited */
  hyg_sgpe_row* rows;    /* [K][rcap] */
  double *lgk, *h, *g, *Hm1s, *gm1s; /* lgk [K][rcap], scratch [rcap] */
  double *dgk, *gk;      /* kappa estimated: digamma differences [K][rcap], scratch [rcap] */
  uint8_t* exs;
} sg_model;

/* rebuild of the theta-dependent model (setUnknownParameters, singleGroup.h:197-270,
 * extendAuxiliaryQuantities :271-335) with L rows per regime */
static void sgm_pe_rebuild(sg_model* m, const double* theta, int L) {
  const int K = m->c.K, u = m->c.u;
  if (L > m->rcap) L = m->rcap;
  for (int r = 0; r < K; ++r) hyg_sgpe_set_regime(theta, K, r, &m->pm);
  for (int r = 0; r < K; ++r) {
    const double* lgk = m->lgk + (size_t)r * m->rcap;
    const double* dgk = m->pc.kest ? m->dgk + (size_t)r * m->rcap : NULL;
    for (int d = 0; d < L; ++d)
      hyg_sgpe_hazard_point(&m->pm, r, d, u, m->pc.kappa[r], lgk, dgk, &m->h[d], &m->g[d], &m->gk[d]);
    const int Lr = hyg_sgpe_hazard_scan(m->h, m->g, dgk ? m->gk : NULL, u, L, m->Hm1s, m->gm1s, m->exs);
    m->Lr[r] = Lr;
    m->exited[r] = m->exs[Lr - 1];
    const double* gsel = dgk ? m->gk : m->g; /* the omega coordinate's derivative (hyg_sg_pe.h) */
    for (int d = 0; d < Lr; ++d)
      m->rows[(size_t)r * m->rcap + d] = hyg_sgpe_hazard_row(m->h[d], gsel[d], m->Hm1s[d], m->gm1s[d], m->exs[d], d, u);
  }
}
static const hyg_sgpe_row* sgm_pe_row(sg_model* m, int dp, int r) {
  int d = dp - 1;
  if (d >= m->Lr[r]) {
    if (!m->exited[r]) m->overflow = 1;
    d = m->Lr[r] - 1;
  }
  return m->rows + (size_t)r * m->rcap + d;
}

static int sgm_init(sg_model* m, const hyg_sg_params* p, int max_duration) {
  memset(m, 0, sizeof(*m));
  int rc = hyg_sg_derive(p, &m->c);
  if (rc) return rc;
  m->dcap = hyg_sg_hazard_len(&m->c, max_duration);
  m->hz = (double*)malloc(sizeof(double) * 2 * (size_t)m->c.K * m->dcap);
  m->ex = (uint8_t*)malloc((size_t)m->c.K * m->dcap);
  if (!m->hz || !m->ex) return HYG_ENOMEM;
  hyg_sg_hazard_fill(&m->c, m->dcap, m->hz, m->ex);
  return HYG_OK;
}
static void sgm_free(sg_model* m) {
  free(m->hz); free(m->ex);
  if (m->pe) {
    free(m->rows); free(m->lgk); free(m->h); free(m->g); free(m->Hm1s); free(m->gm1s); free(m->exs);
    free(m->dgk); free(m->gk);
  }
}

/* Model::evaluateLogTransitionDensity (singleGroup.h:569-608) for the two
 * cases the change-point SMC evaluates: (1, r') from (d, r) and (d+1, r) from (d, r). */
static double sg_trans(sg_model* m, int dc, int rc, int dp, int rp) {
  const int K = m->c.K;
  if (m->pe) {
    const hyg_sgpe_row* w = sgm_pe_row(m, dp, rp);
    if (dc == 1 && rc != rp && dp >= m->c.u) return w->base + m->pm.logP[rp * K + rc];
    if (dc > 1 && rc == rp) return w->cont;
    return -INFINITY;
  }
  int d = dp - 1;
  if (d >= m->dcap) d = m->dcap - 1;
  const double* h = m->hz + ((size_t)rp * m->dcap + d) * 2;
  const int ex = m->ex[(size_t)rp * m->dcap + d];
  if (dc == 1 && rc != rp && dp >= m->c.u) {
    const double lp = m->c.logP[rp * K + rc];
    return ex ? lp : (h[0] + lp);
  }
  if (dc > 1 && rc == rp) return h[1];
  return -INFINITY;
}

/* The particle-dependent part b of log f((1, r') | (d, r)) = b + log P[r][r']
 * (singleGroup.h:569-608): log rho_r(d), 0 once the hazard has exited, -inf
 * below the minimum sojourn u; as sg_trans forms it (b + log P). */
static double sg_bpart(sg_model* m, int dp, int rp) {
  if (dp < m->c.u) return -INFINITY;
  if (m->pe) return sgm_pe_row(m, dp, rp)->base;
  int d = dp - 1;
  if (d >= m->dcap) d = m->dcap - 1;
  return m->ex[(size_t)rp * m->dcap + d] ? 0.0 : m->hz[((size_t)rp * m->dcap + d) * 2];
}

/* exact log-sum-exp: max + log(sum fix100(exp(x - max))) */
static double lse(const double* x, int n) {
  double mx = -INFINITY;
  for (int i = 0; i < n; ++i) if (x[i] > mx) mx = x[i];
  if (!(mx > -INFINITY)) return -INFINITY;
  hyg_u128 s = hyg_u128_zero();
  for (int i = 0; i < n; ++i) s = hyg_u128_add(s, hyg_fix100(hyg_exp(x[i] - mx)));
  return mx + hyg_log(hyg_u128_to_f64(s, 100));
}
/* exact sum of non-negative doubles <= 1 (products of probabilities) */
static double xsum(const double* v, int n) {
  hyg_u128 s = hyg_u128_zero();
  for (int i = 0; i < n; ++i) s = hyg_u128_add(s, hyg_fix100(v[i]));
  return hyg_u128_to_f64(s, 100);
}

/* descending by value, ties by ascending index (arma::sort_index "descend").
 * The comparator's key array is thread-local: the tests and the CPU baselines
 * run several chains at once in threads (a shared pointer let one thread's
 * sort read another's weights). */
static _Thread_local const double* g_sort_v;
static int cmp_desc(const void* a, const void* b) {
  const int i = *(const int*)a, j = *(const int*)b;
  if (g_sort_v[i] > g_sort_v[j]) return -1;
  if (g_sort_v[i] < g_sort_v[j]) return 1;
  return (i < j) ? -1 : (i > j);
}
static void sort_desc(const double* v, int n, int* idx) {
  for (int i = 0; i < n; ++i) idx[i] = i;
  g_sort_v = v;
  qsort(idx, (size_t)n, sizeof(int), cmp_desc);
}

/* ceil(T * R) for a double T in [0, 1] and R < 2^127 (exact, via u192) */
static hyg_u128 ceil_mul_f64(double T, hyg_u128 R) {
  hyg_u128 z = hyg_u128_zero();
  if (!(T > 0.0)) return z;
  const uint64_t b = hyg_f64_bits(T);
  const int E = (int)((b >> 52) & 0x7ff);
  const uint64_t m = (E == 0) ? (b & 0x000fffffffffffffull) : ((b & 0x000fffffffffffffull) | 0x0010000000000000ull);
  const int s = (E == 0) ? 1074 : 1075 - E; /* T = m 2^-s, s >= 52 for T <= 1 */
  /* P = m * R (m < 2^53, R < 2^127: P < 2^180) as three 64-bit words */
  const uint64_t l0 = m * R.lo, h0 = hyg_mulhi64(m, R.lo);
  const uint64_t l1 = m * R.hi, h1 = hyg_mulhi64(m, R.hi);
  uint64_t w0 = l0, w1 = h0 + l1, w2 = h1 + (w1 < h0 ? 1u : 0u);
  if (s >= 192) return (w0 | w1 | w2) ? (hyg_u128){1, 0} : z;
  /* ceil(P / 2^s): add 2^s - 1 then shift */
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

typedef struct {
  int time;
  double* psi; /* [K][Nmax] */
} pending_t;

/* diagnostics: sum / max over steps of the number of pending smoothing times */
int64_t oracle_sg_pending_sum = 0;
int32_t oracle_sg_pending_max = 0;
int64_t oracle_sg_optimal_steps = 0; /* capped steps resampled by the optimal scheme (finite log c) */

/* One chain over T sites: E [T][K] emission table. Writes probs [T][K]
 * (the smoothed regime probabilities). Returns HYG_OK / HYG_ENUMERIC / HYG_ENOMEM. */
/* The reference's structure of the emission (singleGroup.h:611-627 through
 * misc.h:630-640, called from computeWeightsCp, Smc.h:563-573): every use
 * evaluates the Beta-Binomial log-density from the counts, 9 lgamma per sample,
 * the same expressions as the table of oracle_sg_emission (hyg_sg_bb_tables),
 * so the value is bit-identical. Used by oracle_sg_chain_refstruct, the CPU
 * baseline timed in the reference's cost structure. */
typedef struct {
  const uint16_t* meth;
  const uint16_t* tot;
  int S;
} sg_refcounts;
/* lgamma_r: the same values as lgamma without its write of the global signgam,
 * which made threads of the baseline contend for one cache line (the reference
 * runs one process per chain, so its lgamma calls never share it) */
static double lg_r(double x) {
  int sg;
  return lgamma_r(x, &sg);
}
static double sg_em_ref(const hyg_sg_consts* c, const sg_refcounts* rc, int64_t t, int r) {
  const double a = c->alpha[r], b = c->beta[r];
  double e = 0.0;
  for (int s = 0; s < rc->S; ++s) {
    const int n = rc->tot[t * rc->S + s], y = rc->meth[t * rc->S + s];
    if (y > n) return -INFINITY;
    double term = (lg_r((double)n + 1.0) - lg_r((double)y + 1.0)) - lg_r((double)(n - y) + 1.0);
    term = term + lg_r((double)y + a);
    term = term + lg_r((double)(n - y) + b);
    term = term - lg_r((double)n + a + b);
    term = term + (lg_r(a + b) - lg_r(a) - lg_r(b));
    e = e + term;
  }
  return e;
}

static int sg_chain_core(const hyg_sg_params* p, const hyg_sg_pe_params* pe, const double* E, int T, uint64_t seed,
                         uint64_t chain_id, double* probs, int32_t* nparts_out, double* theta_out,
                         const sg_refcounts* rcnt) {
  if (T < 1 || T >= HYG_DMAX - 2) return HYG_EINVAL;
  sg_model mo;
  int rc = sgm_init(&mo, p, T + 1);
  if (rc) return rc;
  const hyg_sg_consts* c = &mo.c;
  const int K = c->K, Nmax = c->Nmax;
  /* online parameter estimation state (OnlineParameterEstimation.h:42-176) */
  double *theta = NULL, *am = NULL, *av = NULL, *gprev = NULL, *gcur = NULL, *phiP = NULL, *phiC = NULL;
  hyg_sgpe_step* steps = NULL;
  int dim = 0, every = 1, iter = 0;
  if (pe) {
    rc = hyg_sgpe_consts_make(p, pe, &mo.pc);
    if (rc) { sgm_free(&mo); return rc; }
    mo.pe = 1;
    dim = mo.pc.dim;
    every = mo.pc.every;
    mo.rcap = (T + 1 < HYG_SGPE_DCAP) ? T + 1 : HYG_SGPE_DCAP;
    const int nst = (int)hyg_sgpe_theta_rows(T, every);
    mo.rows = malloc(sizeof(hyg_sgpe_row) * (size_t)K * mo.rcap);
    mo.lgk = malloc(sizeof(double) * (size_t)K * mo.rcap);
    mo.h = malloc(sizeof(double) * mo.rcap);
    mo.g = malloc(sizeof(double) * mo.rcap);
    mo.Hm1s = malloc(sizeof(double) * mo.rcap);
    mo.gm1s = malloc(sizeof(double) * mo.rcap);
    mo.exs = malloc(mo.rcap);
    mo.gk = malloc(sizeof(double) * mo.rcap);
    mo.dgk = mo.pc.kest ? malloc(sizeof(double) * (size_t)K * mo.rcap) : NULL;
    theta = malloc(sizeof(double) * dim);
    am = calloc(dim, sizeof(double));
    av = calloc(dim, sizeof(double));
    gprev = calloc(dim, sizeof(double));
    gcur = calloc(dim, sizeof(double));
    phiP = calloc((size_t)Nmax * dim, sizeof(double));
    phiC = calloc((size_t)Nmax * dim, sizeof(double));
    steps = malloc(sizeof(hyg_sgpe_step) * (nst + 1));
    if (!mo.rows || !mo.lgk || !mo.h || !mo.g || !mo.Hm1s || !mo.gm1s || !mo.exs || !mo.gk ||
        (mo.pc.kest && !mo.dgk) || !theta || !am || !av || !gprev || !gcur || !phiP || !phiC || !steps) {
      rc = HYG_ENOMEM;
      goto pe_fail;
    }
    hyg_sgpe_steps_fill(pe, nst + 1, steps);
    hyg_sgpe_lgk_fill(mo.pc.kappa, K, mo.rcap, mo.lgk);
    if (mo.pc.kest) hyg_sgpe_dgk_fill(mo.pc.kappa, K, mo.rcap, mo.dgk);
    memcpy(theta, p->theta, sizeof(double) * dim);
    sgm_pe_rebuild(&mo, theta, 1 + every + 1);
    if (theta_out) memcpy(theta_out, theta, sizeof(double) * dim);
  }
  int *dP = malloc(sizeof(int) * Nmax), *rP = malloc(sizeof(int) * Nmax), *dC = malloc(sizeof(int) * Nmax),
      *rC = malloc(sizeof(int) * Nmax), *anc = malloc(sizeof(int) * Nmax), *idx = malloc(sizeof(int) * Nmax);
  double *lwP = malloc(sizeof(double) * Nmax), *lwC = malloc(sizeof(double) * Nmax),
         *wP = malloc(sizeof(double) * Nmax), *wC = malloc(sizeof(double) * Nmax),
         *lwres = malloc(sizeof(double) * Nmax), *tmp = malloc(sizeof(double) * Nmax),
         *tmp2 = malloc(sizeof(double) * Nmax), *logq = malloc(sizeof(double) * Nmax),
         *BK = malloc(sizeof(double) * HYG_KMAX * Nmax);
  hyg_u128* cum = malloc(sizeof(hyg_u128) * (Nmax + 1));
  int cap = 64, npend = 0;
  pending_t* pend = malloc(sizeof(pending_t) * cap);
  if (!dP || !rP || !dC || !rC || !anc || !idx || !lwP || !lwC || !wP || !wC || !lwres || !tmp || !tmp2 || !logq ||
      !BK || !cum || !pend) {
    rc = HYG_ENOMEM;
    goto done;
  }
  for (int t = 0; t < T; ++t)
    for (int r = 0; r < K; ++r) probs[(size_t)t * K + r] = NAN;

  /* ---- t = 0 (Smc.h:114-188): N = K particles (1, r), w = -log K + log g_0 */
  int N = K;
  for (int n = 0; n < N; ++n) {
    dC[n] = 1;
    rC[n] = n;
    lwC[n] = -c->log_K + (rcnt ? sg_em_ref(c, rcnt, 0, n) : E[n]);
  }
  double logZ = lse(lwC, N);
  if (!(logZ > -INFINITY)) { rc = HYG_ENUMERIC; goto done; }
  for (int n = 0; n < N; ++n) wC[n] = hyg_exp(lwC[n] - logZ);
  if (nparts_out) nparts_out[0] = N;

  /* psi bookkeeping (OnlineMarginalSmoothing.h:132-150 initialisePsi, :199-253 storeEstimates) */
#define ADD_PENDING(tt)                                                              \
  do {                                                                               \
    if (npend == cap) {                                                              \
      cap *= 2;                                                                      \
      pending_t* np_ = realloc(pend, sizeof(pending_t) * cap);                       \
      if (!np_) { rc = HYG_ENOMEM; goto done; }                                      \
      pend = np_;                                                                    \
    }                                                                                \
    pend[npend].time = (tt);                                                         \
    pend[npend].psi = malloc(sizeof(double) * K * Nmax);                             \
    if (!pend[npend].psi) { rc = HYG_ENOMEM; goto done; }                            \
    for (int r_ = 0; r_ < K; ++r_)                                                   \
      for (int n_ = 0; n_ < N; ++n_) pend[npend].psi[r_ * Nmax + n_] = (rC[n_] == r_) ? 1.0 : 0.0; \
    ++npend;                                                                         \
  } while (0)

  ADD_PENDING(0);
  for (int t = 0; t < T; ++t) {
    const int final = (t == T - 1);
    if (t > 0) {
      /* ---- Smc::iterate (:190-286) */
      const int Np = N;
      memcpy(dP, dC, sizeof(int) * Np);
      memcpy(rP, rC, sizeof(int) * Np);
      memcpy(lwP, lwC, sizeof(double) * Np);
      memcpy(wP, wC, sizeof(double) * Np);
      const double logZp = logZ;
      N = (Np + K > Nmax) ? Nmax : Np + K;
      const int M = N - K;
      /* resampleCp (:406-450) */
      if (N < Np + K) {
        int fin = 0;
        for (int n = 0; n < Np; ++n) fin += hyg_isfinite(lwP[n]) ? 1 : 0;
        int keep_top = 1;
        if (fin > M) {
          /* optimalFiniteState (resample.h:289-409) on the self-normalised weights */
          sort_desc(wP, Np, idx);
          for (int q = 0; q < Np; ++q) logq[q] = hyg_log(wP[idx[q]]);
          cum[Np] = hyg_u128_zero(); /* reverse cumulative sums Q(k), exact */
          for (int q = Np - 1; q >= 0; --q) cum[q] = hyg_u128_add(cum[q + 1], hyg_fix100(wP[idx[q]]));
          int kOld = 1, kNew = 0;
          double logC = 0.0;
          while (kNew != kOld) {
            kOld = kNew;
            const double Qk = hyg_u128_to_f64(cum[kOld], 100);
            logC = hyg_log((double)(M - kOld)) - hyg_log(Qk);
            int cnt = 0;
            for (int q = kOld; q < Np; ++q) cnt += (logq[q] > -logC) ? 1 : 0;
            kNew = kOld + cnt;
          }
          if (hyg_isfinite(logC)) {
            keep_top = 0;
            ++oracle_sg_optimal_steps;
            const int Kk = kNew, L = M - Kk;
            for (int q = 0; q < Kk; ++q) {
              anc[q] = idx[q];
              lwres[q] = lwP[idx[q]];
            }
            if (L > 0) {
              /* residual systematic draw: normalised exp(logQ[K..N)) (:372-377),
               * systematicBase (:85-117) with T_j = (j + u) / L <= Q_i as exact
               * C_i >= ceil(T_j * R) */
              double rmax = -INFINITY;
              for (int q = Kk; q < Np; ++q) if (logq[q] > rmax) rmax = logq[q];
              hyg_u128 run = hyg_u128_zero();
              for (int q = Kk; q < Np; ++q) {
                run = hyg_u128_add(run, hyg_fix100(hyg_exp(logq[q] - rmax)));
                cum[q] = run;
              }
              const double uu =
                  (double)(hyg_rand64(seed, chain_id, HYG_RNG_SG_SYSTEMATIC, (uint64_t)t, 0) >> 11) *
                  1.1102230246251565404e-16;
              int i = Kk;
              for (int j = 0; j < L; ++j) {
                const double Tj = ((double)j + uu) / (double)L;
                const hyg_u128 thr = ceil_mul_f64(Tj, run);
                while (i < Np - 1 && hyg_u128_lt(cum[i], thr)) ++i;
                anc[Kk + j] = idx[i];
                lwres[Kk + j] = logZp - logC;
              }
            }
          }
        }
        if (keep_top) {
          /* keep the M largest weights (:432-441 and resample.h:379-384) */
          sort_desc(lwP, Np, idx);
          for (int n = 0; n < M; ++n) {
            anc[n] = idx[n];
            lwres[n] = lwP[idx[n]];
          }
        }
      } else {
        for (int n = 0; n < M; ++n) {
          anc[n] = n;
          lwres[n] = lwP[n];
        }
      }
      /* sampleParticlesCp (:504-522) + computeWeightsCp (:536-574) */
      const double* Et = rcnt ? NULL : E + (size_t)t * K;
      for (int n = 0; n < M; ++n) {
        dC[n] = dP[anc[n]] + 1;
        rC[n] = rP[anc[n]];
        const double gt = rcnt ? sg_em_ref(c, rcnt, t, rC[n]) : Et[rC[n]];
        lwC[n] = lwres[n] + (sg_trans(&mo, dC[n], rC[n], dP[anc[n]], rP[anc[n]]) + gt);
      }
      /* evaluateBackwardKernels (:288-326): K_q(n) = normalise_n(W_prev[n] + log f((1,q) | n)).
       * log f((1,q) | (d_n, r_n)) = b_n + log P[r_n][q] (b_n: the hazard part, sg_bpart;
       * log P[r][r] = -inf), so with a_n = W_prev[n] + b_n the rows factorise over the
       * regimes: A_r = max of a_n over the particles of regime r, m_q = max_r (A_r +
       * log P[r][q]) (= max_n (a_n + log P[r_n][q]): rounding is monotone),
       *   K_q(n) = (e_n G[r_n][q]) / S_q,  e_n = exp(a_n - A_{r_n}),
       *   G[r][q] = exp((A_r + log P[r][q]) - m_q),  S_q = sum_r G[r][q] E_r (FMA, r order),
       * E_r the exact sum of the F = 100 images of e_n over regime r: one exp per
       * particle and K^2 per step instead of one per (particle, row).
       * The fresh particle (1, q) has log weight m_q + log S_q + log g_t(q): the
       * reference's logsumexp_n(log f + log g + W_prev[n]) (computeWeightsCp :563-573)
       * with the n-independent log g taken out. */
      {
        double A[HYG_KMAX], Ef[HYG_KMAX];
        hyg_u128 Er[HYG_KMAX];
        for (int r = 0; r < K; ++r) {
          A[r] = -INFINITY;
          Er[r] = hyg_u128_zero();
        }
        for (int n = 0; n < Np; ++n) {
          tmp[n] = lwP[n] + sg_bpart(&mo, dP[n], rP[n]);
          if (tmp[n] > A[rP[n]]) A[rP[n]] = tmp[n];
        }
        for (int n = 0; n < Np; ++n) {
          tmp2[n] = (tmp[n] > -INFINITY) ? hyg_exp(tmp[n] - A[rP[n]]) : 0.0;
          Er[rP[n]] = hyg_u128_add(Er[rP[n]], hyg_fix100(tmp2[n]));
        }
        for (int r = 0; r < K; ++r) Ef[r] = hyg_u128_to_f64(Er[r], 100);
        const double* lP = mo.pe ? mo.pm.logP : c->logP;
        for (int q = 0; q < K; ++q) {
          dC[M + q] = 1;
          rC[M + q] = q;
          double mq = -INFINITY;
          for (int r = 0; r < K; ++r) {
            const double v = A[r] + lP[r * K + q];
            if (v > mq) mq = v;
          }
          if (mq > -INFINITY) {
            double G[HYG_KMAX], S = 0.0;
            for (int r = 0; r < K; ++r) {
              G[r] = hyg_exp((A[r] + lP[r * K + q]) - mq);
              S = HYG_FMA(G[r], Ef[r], S);
            }
            const double inv = 1.0 / S;
            for (int n = 0; n < Np; ++n) BK[q * Nmax + n] = (tmp2[n] * G[rP[n]]) * inv;
            double gq;
            if (rcnt) {  /* the reference evaluates log g inside its loop over the previous particles */
              volatile double sink = 0.0;
              for (int n = 0; n < Np; ++n) sink = sg_em_ref(c, rcnt, t, q);
              gq = sink;
            } else {
              gq = Et[q];
            }
            lwC[M + q] = (mq + hyg_log(S)) + gq;
          } else {
            for (int n = 0; n < Np; ++n) BK[q * Nmax + n] = 0.0;
            lwC[M + q] = -INFINITY;
          }
        }
      }
      logZ = lse(lwC, N); /* selfNormaliseWeights (:576-579) */
      if (!(logZ > -INFINITY)) { rc = HYG_ENUMERIC; goto done; }
      for (int n = 0; n < N; ++n) wC[n] = hyg_exp(lwC[n] - logZ);
      if (nparts_out) nparts_out[t] = N;
      if (mo.pe) {
        /* updatePhi (OnlineParameterEstimation.h:118-150): phiCurr from phiPrev
         * (gradients of the log transition density, singleGroup.h:641-717) */
        const int jw = K * (K - 1), jk = K * K; /* omega / kappa blocks of theta */
        for (int n = 0; n < M; ++n) {
          const int a = anc[n];
          const hyg_sgpe_row* w = sgm_pe_row(&mo, dP[a], rP[a]);
          /* the kappa index of a continuation (:688-692): -grad(idxKappa) rho / (1 - rho)
           * with grad(idxKappa) = 0 never written, i.e. -0.0 where that branch runs
           * (!exit && rho < 1, i.e. a finite log(1 - rho)), else the zeroed vector */
          const double gkap = (w->cont > -INFINITY) ? -0.0 : 0.0;
          for (int j = 0; j < dim; ++j) {
            const double g = (j == jw + rC[n]) ? w->gcont : (j == jk + rC[n]) ? gkap : 0.0;
            phiC[(size_t)n * dim + j] = phiP[(size_t)a * dim + j] + g;
          }
        }
        const int nch = hyg_sgpe_fresh_chunks(K), rows = 256 / nch;
        for (int q = 0; q < K; ++q) {
          for (int j = 0; j < dim; ++j) {
            double acc = 0.0;
            for (int ck = 0; ck < nch; ++ck) {
            double part = 0.0;
            const int n1 = (ck + 1) * rows < Np ? (ck + 1) * rows : Np;
            for (int n = ck * rows; n < n1; ++n) {
              const int rp = rP[n];
              double g = 0.0;
              if (q != rp && dP[n] >= c->u) {
                if (j == jw + rp) {
                  g = sgm_pe_row(&mo, dP[n], rp)->gomg;
                } else if (j >= rp * (K - 1) && j < (rp + 1) * (K - 1)) {
                  const int i = j - rp * (K - 1), jj = (i < rp) ? i : i + 1;
                  g = -mo.pm.P[rp * K + jj];
                  if (jj == q) g = g + 1.0;
                }
              }
              part = part + BK[q * Nmax + n] * (phiP[(size_t)n * dim + j] + g);
            }
            acc = (ck == 0) ? part : acc + part;
            }
            phiC[(size_t)(M + q) * dim + j] = acc;
          }
        }
        if (t % every == 0) {
          /* updateGradients (:151-156) + GradientAscent::iterate (GradientAscent.h:82-105) */
          double l1 = 0.0;
          for (int j = 0; j < dim; ++j) {
            double est = 0.0;
            for (int n = 0; n < N; ++n) est = est + wC[n] * phiC[(size_t)n * dim + j];
            gcur[j] = est - gprev[j];
            gprev[j] = est;
            l1 = l1 + fabs(gcur[j]);
          }
          for (int j = 0; j < dim; ++j) theta[j] = hyg_sgpe_update(mo.pc.use_adam, mo.pc.normalise, mo.pc.beta1, mo.pc.beta2, mo.pc.eps,
                                       steps[iter].lr, steps[iter].c1, steps[iter].c2, theta[j], gcur[j], l1,
                                       &am[j], &av[j]);
          ++iter;
          int maxd = 0;
          for (int n = 0; n < N; ++n) maxd = dC[n] > maxd ? dC[n] : maxd;
          sgm_pe_rebuild(&mo, theta, maxd + every + 1);
          if (theta_out) memcpy(theta_out + (size_t)(t / every) * dim, theta, sizeof(double) * dim);
        }
        double* sw = phiP;
        phiP = phiC;
        phiC = sw;
        if (mo.overflow) { rc = HYG_ENOMEM; goto done; }
      }
      /* updatePsi (:152-197) for every pending time */
      for (int s = 0; s < npend; ++s) {
        double* ps = pend[s].psi;
        for (int r = 0; r < K; ++r) {
          double* row = ps + r * Nmax;
          memcpy(tmp2, row, sizeof(double) * Np);
          for (int n = 0; n < M; ++n) row[n] = tmp2[anc[n]];
          for (int q = 0; q < K; ++q) {
            for (int n = 0; n < Np; ++n) tmp[n] = BK[q * Nmax + n] * tmp2[n];
            row[M + q] = xsum(tmp, Np);
          }
        }
      }
      ADD_PENDING(t);
    }
    /* storeEstimates (:199-253): finalise a time once every regime's filtered
     * variance is below epsilon (or at the final step) */
    int keep = 0;
    for (int s = 0; s < npend; ++s) {
      double* ps = pend[s].psi;
      double mean[HYG_KMAX];
      int ok = 1;
      for (int r = 0; r < K; ++r) {
        const double* row = ps + r * Nmax;
        for (int n = 0; n < N; ++n) tmp[n] = wC[n] * row[n];
        mean[r] = xsum(tmp, N);
        if (!final && ok) {
          for (int n = 0; n < N; ++n) {
            const double v = row[n] - mean[r];
            tmp[n] = wC[n] * (v * v);
          }
          if (!(xsum(tmp, N) < c->epsilon)) ok = 0;
        }
      }
      if (final || ok) {
        for (int r = 0; r < K; ++r) probs[(size_t)pend[s].time * K + r] = mean[r];
        free(ps);
      } else {
        pend[keep++] = pend[s];
      }
    }
    npend = keep;
    oracle_sg_pending_sum += npend;
    if (npend > oracle_sg_pending_max) oracle_sg_pending_max = npend;
  }
  rc = HYG_OK;
done:
  for (int s = 0; s < npend; ++s) free(pend[s].psi);
  free(pend);
  free(dP); free(rP); free(dC); free(rC); free(anc); free(idx);
  free(lwP); free(lwC); free(wP); free(wC); free(lwres); free(tmp); free(tmp2); free(logq); free(BK); free(cum);
pe_fail:
  free(theta); free(am); free(av); free(gprev); free(gcur); free(phiP); free(phiC); free(steps);
  sgm_free(&mo);
  return rc;
#undef ADD_PENDING
}

int oracle_sg_chain(const hyg_sg_params* p, const double* E, int T, uint64_t seed, uint64_t chain_id,
                    double* probs, int32_t* nparts_out) {
  return sg_chain_core(p, NULL, E, T, seed, chain_id, probs, nparts_out, NULL, NULL);
}
/* oracle_sg_chain with the emission evaluated from the counts at every use
 * (the reference's cost structure, sg_em_ref): the same outputs bit for bit */
int oracle_sg_chain_refstruct(const hyg_sg_params* p, const uint16_t* meth, const uint16_t* tot, int S, int T,
                              uint64_t seed, uint64_t chain_id, double* probs, int32_t* nparts_out) {
  sg_refcounts rc = {meth, tot, S};
  return sg_chain_core(p, NULL, NULL, T, seed, chain_id, probs, nparts_out, NULL, &rc);
}
/* theta_out [1 + (T - 1) / every][K^2, or K (K + 1) with kappa estimated] */
int oracle_sg_chain_pe(const hyg_sg_params* p, const hyg_sg_pe_params* pe, const double* E, int T, uint64_t seed,
                       uint64_t chain_id, double* probs, double* theta_out) {
  return sg_chain_core(p, pe, E, T, seed, chain_id, probs, NULL, theta_out, NULL);
}
double oracle_sg_digamma(double x) { return hyg_digamma(x); }
int oracle_sg_pe_hazard(const hyg_sg_params* p, const double* theta, int L, hyg_sgpe_row* rows, int32_t* Lr) {
  /* hazard rows of the estimation path for tests: rows [K][L] */
  hyg_sg_pe_params pe = {1, 0, 200, 0, 0.1, 0.01};
  sg_model mo;
  int rc = sgm_init(&mo, p, L + 1);
  if (rc) return rc;
  rc = hyg_sgpe_consts_make(p, &pe, &mo.pc);
  if (rc) { sgm_free(&mo); return rc; }
  mo.pe = 1;
  mo.rcap = L;
  const int K = mo.c.K;
  mo.rows = malloc(sizeof(hyg_sgpe_row) * (size_t)K * L);
  mo.lgk = malloc(sizeof(double) * (size_t)K * L);
  mo.h = malloc(sizeof(double) * L); mo.g = malloc(sizeof(double) * L);
  mo.Hm1s = malloc(sizeof(double) * L); mo.gm1s = malloc(sizeof(double) * L);
  mo.exs = malloc(L);
  mo.gk = malloc(sizeof(double) * L);
  mo.dgk = mo.pc.kest ? malloc(sizeof(double) * (size_t)K * L) : NULL;
  if (!mo.rows || !mo.lgk || !mo.h || !mo.g || !mo.Hm1s || !mo.gm1s || !mo.exs || !mo.gk || (mo.pc.kest && !mo.dgk)) {
    sgm_free(&mo);
    return HYG_ENOMEM;
  }
  hyg_sgpe_lgk_fill(mo.pc.kappa, K, L, mo.lgk);
  if (mo.pc.kest) hyg_sgpe_dgk_fill(mo.pc.kappa, K, L, mo.dgk);
  sgm_pe_rebuild(&mo, theta, L);
  memcpy(rows, mo.rows, sizeof(hyg_sgpe_row) * (size_t)K * L);
  for (int r = 0; r < K; ++r) Lr[r] = mo.Lr[r];
  sgm_free(&mo);
  return HYG_OK;
}

/* E[t][r] = sum_s BB(y | n, alpha_r, beta_r) (singleGroup.h:611-627, misc.h:630-640),
 * every sample included (n = 0 adds the lgamma round-off, as the reference) */
int oracle_sg_emission(const hyg_sg_params* p, const uint16_t* meth, const uint16_t* tot, int S, int64_t T,
                       double* E) {
  hyg_sg_consts c;
  int rc = hyg_sg_derive(p, &c);
  if (rc) return rc;
  int nmax = 0;
  for (int64_t i = 0; i < T * S; ++i) if (tot[i] > nmax) nmax = tot[i];
  const int L = nmax + 1, K = c.K;
  double* lf = malloc(sizeof(double) * L);
  double* lg = malloc(sizeof(double) * 3 * K * L);
  double cst[HYG_KMAX];
  if (!lf || !lg) { free(lf); free(lg); return HYG_ENOMEM; }
  hyg_sg_bb_tables(&c, nmax, lf, lg, cst);
  for (int64_t t = 0; t < T; ++t) {
    for (int r = 0; r < K; ++r) {
      double e = 0.0;
      for (int s = 0; s < S; ++s) {
        const int n = tot[t * S + s], y = meth[t * S + s];
        if (y > n) { e = -INFINITY; break; }
        double term = (lf[n] - lf[y]) - lf[n - y];
        term = term + lg[(size_t)(r * 3 + 0) * L + y];
        term = term + lg[(size_t)(r * 3 + 1) * L + (n - y)];
        term = term - lg[(size_t)(r * 3 + 2) * L + n];
        term = term + cst[r];
        e = e + term;
      }
      E[t * K + r] = e;
    }
  }
  free(lf);
  free(lg);
  return HYG_OK;
}

/* tables for tests */
int oracle_sg_hazard(const hyg_sg_params* p, int r, int n, double* out, uint8_t* ex, int32_t* dcap) {
  sg_model mo;
  int rc = sgm_init(&mo, p, n + 2);
  if (rc) return rc;
  *dcap = mo.dcap;
  for (int dp = 1; dp <= n; ++dp) {
    int d = dp - 1;
    if (d >= mo.dcap) d = mo.dcap - 1;
    out[2 * (dp - 1) + 0] = mo.hz[((size_t)r * mo.dcap + d) * 2 + 0];
    out[2 * (dp - 1) + 1] = mo.hz[((size_t)r * mo.dcap + d) * 2 + 1];
    ex[dp - 1] = mo.ex[(size_t)r * mo.dcap + d];
  }
  sgm_free(&mo);
  return HYG_OK;
}
int oracle_sg_consts(const hyg_sg_params* p, hyg_sg_consts* out) { return hyg_sg_derive(p, out); }
int oracle_sizeof_sg_params(void) { return (int)sizeof(hyg_sg_params); }
int oracle_sizeof_sg_consts(void) { return (int)sizeof(hyg_sg_consts); }
