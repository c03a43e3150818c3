/*
 * hygeia_amd.h -- C ABI of the MI355X-native Hygeia change-point inference path.
 *
 * Drop-in boundary for the two-group (case/control) inference engine of
 * ucl-medical-genomics/hygeia. The reference exposes this path as
 *
 *   filter_and_smoother_algorithm.run(observations, initial_state_prior,
 *       initial_proposal, transition_fn, observation_fn, num_particles,
 *       proposal_fn, num_resampled_ancestors, optimal_resampling,
 *       multinomial_resampling, num_simulations)
 *     -> (BackwardSimulationResults(particle={merged_state [T,B],
 *          control_state [T,B,2], case_state [T,B,2]}),
 *         final_unnormalized_log_weights [N_max])
 *   (src/two_group/hygeia/filter_and_smoother_algorithm.py:38-138)
 *
 * with the model (CaseControlRegimeModel, case_control_regime_model.py:41-244)
 * and the proposal (CaseControlProposal, case_control_proposal_mappings.py:3-216)
 * passed in as Python callables, driven by
 * src/two_group/run_inference_two_groups.py:92-322 ("hygeia infer"). Here the
 * model is fixed (it is the only one the CLI builds) and given by its
 * parameters; everything else is plain pointers and sizes.
 *
 * Conventions: every entry point returns HYG_OK (0) or a negative HYG_E* code
 * and never throws; hyg_last_error() gives a thread-local message. The caller
 * owns every buffer. Functions taking a `stream` argument enqueue work on that
 * hipStream_t (NULL = the default stream) and take DEVICE pointers; functions
 * named *_host take host pointers and synchronise. There is no CPU fallback:
 * without a HIP device every compute entry point returns HYG_EDEVICE.
 *
 * Threading: a model handle (hyg_tg_model / hyg_sg_model) is read-only after
 * creation except for its per-stream pinned staging buffers, which are
 * mutex-guarded; several host threads may launch with one model, each on its
 * own stream, without waiting for each other's kernels. hyg_set_kernel_timing /
 * hyg_tg_last_kernel_ms are a process-wide diagnostic and are not thread-safe.
 * The single-group chain launches need two workgroups per chain resident at
 * once; they stay correct on a shared GPU (a chain's pair then waits for a
 * free CU) but are sized for a GPU they have to themselves.
 */
#ifndef HYGEIA_AMD_H
#define HYGEIA_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HYG_KMAX 16

#define HYG_OK 0
#define HYG_EINVAL (-1)
#define HYG_ENUMERIC (-2) /* all particle weights became -inf */
#define HYG_EDEVICE (-3)
#define HYG_ENOMEM (-4)
#define HYG_EUNSUPPORTED (-5)

/* Parameters of the two-group model as "hygeia infer" receives them
 * (absl flags at run_inference_two_groups.py:19-72, theta file at :76-89,
 * fixed kappa at :158-161). */
typedef struct hyg_tg_params {
  int32_t n_regimes;               /* K = len(--mu) (:126)                        */
  int32_t minimum_duration;        /* u, --minimum_duration, default 3 (:25-27)   */
  int32_t num_resampled_ancestors; /* M, --num_resampled_particles, default 50     */
  int32_t num_samples_backward;    /* B, --num_samples_backward, default 25       */
  int32_t optimal_resampling;      /* 1 on the CLI path (:274)                    */
  int32_t multinomial;             /* --multinomial; used only when optimal == 0  */
  int32_t theta_len;               /* number of values in theta (K^2 on the CLI)  */
  int32_t _pad;
  double mu[HYG_KMAX];             /* --mu (float32 in the reference)             */
  double sigma[HYG_KMAX];          /* --sigma                                     */
  double theta[HYG_KMAX * HYG_KMAX]; /* theta_{chrom}.csv.gz 'data': K(K-1) log-p
                                        blocks, then K logit-omega (:76-89)       */
  double omega_case;               /* --omega_case, default 0.8 (:28-30)          */
  double merge_log_prob;           /* --merge_log_prob, default log(0.1) (:31-33) */
  double split_prob;               /* --split_prob, default 0.01 (:34-36)         */
  double kappa_control;            /* 2 (:158-159)                                */
  double kappa_case;               /* 2 (:160-161)                                */
} hyg_tg_params;

/* Fills p with the reference's flag defaults (K = 6, uniform theta). */
void hyg_tg_params_default(hyg_tg_params* p);

/* One chain = one (chromosome, segment, seed) task of modules/two_group/4_infer.nf,
 * i.e. one run_inference_two_groups.py process. */
typedef struct hyg_tg_chain {
  int64_t site_begin; /* first site of the chain in the site-major input arrays  */
  int32_t n_sites;    /* T (segment + buffers, run_inference_two_groups.py:199-200) */
  int32_t _pad;
  uint64_t seed;      /* --seed                                                  */
  uint64_t chain_id;  /* RNG stream id of the chain (e.g. chrom*2^32 + batch)    */
  int64_t out_begin;  /* first output row of the chain in the output arrays      */
} hyg_tg_chain;

typedef struct hyg_tg_model hyg_tg_model; /* opaque: derived constants + tables */

/* Builds the model: derived constants (T2/T4 of SURVEY 8a), Beta-Binomial
 * log-gamma tables for read counts <= max_total_reads, and the hazard tables
 * (case_control_regime_model.py:111-168) for durations <= max_duration.
 * Uploads the tables to the current HIP device when one is present. */
int hyg_tg_model_create(const hyg_tg_params* params, int32_t max_total_reads,
                        int32_t max_duration, hyg_tg_model** out);
void hyg_tg_model_destroy(hyg_tg_model* model);

/* Derived sizes: I = 2K + K^2 proposal slots, N_max = M * I particles
 * (run_inference_two_groups.py:263,285). */
int32_t hyg_tg_num_particles(const hyg_tg_model* model);

/* Threads per chain workgroup of the forward kernel for a launch of n_chains
 * chains on the current device: 256 (up to three chains per CU) or, at most
 * one chain per CU, the low-occupancy width 512, whose extra waves shorten the
 * parallel phases of each step of the sequential chain (512 also for the
 * K = 12 stress shape, one chain per CU by its LDS). Diagnostic: the launch
 * functions choose it themselves. No reference counterpart (the reference
 * runs one chain per CPU process, modules/two_group/4_infer.nf:28). */
int32_t hyg_tg_threads_per_chain(const hyg_tg_model* model, int32_t n_chains);

/* Forward-kernel workgroups (chains) one CU holds at the width a launch of
 * n_chains uses (the HIP occupancy query with the kernel's LDS): 3 for the
 * pipeline shape at 256 threads, 1 at the low-occupancy width. 0 without a
 * device. Diagnostic. */
int32_t hyg_tg_chains_per_cu(const hyg_tg_model* model, int32_t n_chains);

/* LDS bytes of one chain workgroup of the forward (backward = 0) or backward
 * kernel at `threads` (64, 128, 256, 512 or 768; 0 for another width). No
 * device needed. Diagnostic: C3 on one GPU needs three 256-thread forward
 * chains per CU, and the hardware's LDS allocation leaves the pipeline shape
 * little room (53 520 B holds three per CU; 53 776 B held two while the
 * occupancy query still reported three); tests pin it. */
size_t hyg_tg_lds_bytes(const hyg_tg_model* model, int32_t threads, int32_t backward);

/* Test / tuning override of the chain workgroup sizes for every later launch
 * in the process: forward and backward threads (64, 128, 256, 512 or 768;
 * 0 = the automatic choice above). Not thread-safe. The results do not depend
 * on it: every width computes the same bits. */
int hyg_tg_force_threads(int32_t forward, int32_t backward);

/* Tail overlap of hyg_tg_run_chains (on = 1, the default; 0 = off) for every
 * later launch in the process. When the forward holds one chain per CU and
 * the chains fill more than one round of CUs with a partial last round (the
 * K = 12 stress shape: 1 164 chains on 256 CUs), the launch runs the forward
 * of the full rounds, then the rest's forward on the launch stream while the
 * full rounds' backward runs on a second stream of the library's, on the CUs
 * the last round leaves idle; the call's stream waits for both. The results
 * do not depend on it (GPU test). Not thread-safe. No reference counterpart. */
int hyg_tg_set_tail_overlap(int32_t on);

/* Compute units of `device` as the two-group launcher sees them: the width
 * choice (one chain per CU or more) and the tail overlap depend on it. Cached
 * per device, so a process that switches devices (hyg_set_device) uses each
 * device's own count. 0 if unknown (no such device, no HIP). No reference
 * counterpart. */
int32_t hyg_tg_device_cus(int32_t device);

/* Test override of that count for device (0 <= device < 64); cus = 0 drops
 * the override (the next use queries the device). The results do not depend
 * on it (every width computes the same bits); launches after it are shaped as
 * on a device with that many CUs. */
int hyg_tg_set_device_cus(int32_t device, int32_t cus);

/* Test override of the single-group chain's log-weight sort for every later
 * launch in the process. The sort orders one 64-bit word per particle: the
 * order key's top 64 - bits bits and the particle index (bits = 8, or 0 for
 * the default). Wherever keys that agree on those bits disagree below them,
 * the kernel detects it and re-sorts exactly, so the results do not depend on
 * it; larger values (up to 60) make that path run often. Not thread-safe. */
int hyg_sg_force_key_drop(int32_t bits);

/* Per-site emission table E[t][g*K + r] = log g_t for group g (0 control,
 * 1 case) and regime r: sum over samples of BetaBinomial(meth | total,
 * alpha_r, beta_r) (case_control_regime_model.py:197-231). Counts are
 * site-major uint16 [T][S]. Device pointers. */
int hyg_tg_emission(const hyg_tg_model* model, const uint16_t* meth_ctrl, const uint16_t* tot_ctrl,
                    int32_t s_ctrl, const uint16_t* meth_case, const uint16_t* tot_case, int32_t s_case,
                    int64_t n_sites, double* emission, void* stream);

/* Workspace bytes for the forward->backward ancestor history of `n_chains`
 * chains totalling `total_steps` filter steps. For the K = 12 stress shape the
 * bound also holds a full-N weight scratch per chain (Nmax f64, 67 KB), which
 * only the 256-thread backward of a launch with more chains than CUs uses; it
 * is charged whatever the width, so the size does not depend on the launch
 * width or hyg_tg_force_threads (a conservative bound: under 0.04 % of a
 * full-length chain's history). */
size_t hyg_tg_workspace_bytes(const hyg_tg_model* model, int32_t n_chains, int64_t total_steps);

/* Outputs of hyg_tg_run_chains, all device pointers indexed by out_begin + t:
 * trajectories as the reference saves them (run_inference_two_groups.py:299-314):
 *   merged [T][B] int16, control [T][B][2] int16 (d, r), case [T][B][2] int16,
 *   split_probs [T] f32, regime_probs [T][2K] f32 (test_function means, :233-240,294-296),
 * per chain: log_z [n_chains] f64 (logsumexp of the final weights, :289-290) and
 * optionally final_log_weights [n_chains][N_max] f64 (the second return value
 * of run(), -inf padded; may be NULL), status [n_chains] int32 (HYG_OK or
 * HYG_ENUMERIC per chain; may be NULL). */
typedef struct hyg_tg_outputs {
  int16_t* merged;
  int16_t* control;
  int16_t* kase;
  float* split_probs;
  float* regime_probs;
  double* log_z;
  double* final_log_weights;
  int32_t* status;
} hyg_tg_outputs;

/* Runs the particle filter with optimal finite-state resampling followed by
 * backward simulation (filter_and_smoother_algorithm.py:38-138, 141-288,
 * 368-447) for `n_chains` independent chains, one workgroup per chain.
 * `chains` is a HOST array; `emission` is the device table of
 * hyg_tg_emission; `workspace` has hyg_tg_workspace_bytes bytes. */
int hyg_tg_run_chains(const hyg_tg_model* model, const hyg_tg_chain* chains, int32_t n_chains,
                      const double* emission, void* workspace, size_t workspace_bytes,
                      const hyg_tg_outputs* outputs, void* stream);

/* Host-pointer convenience: one chain of T sites (the whole of one
 * run_inference_two_groups.py invocation). Outputs are host arrays sized as
 * above for one chain; final_log_weights may be NULL. */
int hyg_tg_run_chain_host(const hyg_tg_model* model, const uint16_t* meth_ctrl, const uint16_t* tot_ctrl,
                          int32_t s_ctrl, const uint16_t* meth_case, const uint16_t* tot_case, int32_t s_case,
                          int32_t n_sites, uint64_t seed, uint64_t chain_id, int16_t* merged, int16_t* control,
                          int16_t* kase, float* split_probs, float* regime_probs, double* log_z,
                          double* final_log_weights);

/* Host-pointer form of hyg_tg_run_chains (round 4): the counts of n_sites
 * sites (host, site-major) are copied in, the emission table is formed, the
 * n_chains chains (host array: site_begin into the counts, out_begin into the
 * output rows) run in one launch, and the outputs come back into host arrays
 * of out_rows rows (layouts as above), log_z and status [n_chains]
 * (final_log_weights [n_chains][N_max], may be NULL). Returns HYG_OK when the
 * launch ran; a chain whose weights all became -inf has HYG_ENUMERIC in its
 * status. `hygeia infer_many` (every task that modules/two_group/4_infer.nf:42-48
 * fans out, in one launch) runs through it without torch. */
int hyg_tg_run_chains_host(const hyg_tg_model* model, const uint16_t* meth_ctrl, const uint16_t* tot_ctrl,
                           int32_t s_ctrl, const uint16_t* meth_case, const uint16_t* tot_case, int32_t s_case,
                           int64_t n_sites, const hyg_tg_chain* chains, int32_t n_chains, int64_t out_rows,
                           int16_t* merged, int16_t* control, int16_t* kase, float* split_probs,
                           float* regime_probs, double* log_z, double* final_log_weights, int32_t* status);

/* Kernel timing for benchmarks: when enabled, HIP events are recorded on the
 * launch stream around the emission, forward and backward kernels;
 * hyg_tg_last_kernel_ms waits for the last ones and returns their durations
 * in ms (-1 for a kernel not launched since timing was enabled). */
void hyg_set_kernel_timing(int enable);
int hyg_tg_last_kernel_ms(float* ms3);

/* ======================================================== single group
 * The single-group engine (src/single_group/src/cpp): SMC over the semi-Markov
 * state (d, r) with up to N_max particles, optimal finite-state resampling and
 * online marginal smoothing of the regime indicators (Alenlov & Olsson 2019),
 * as exported to R by
 *   runOnlineCombinedInferenceCpp(vartheta, thetaInit, genomicPositions,
 *       nTotalReads [S x T], nMethylatedReads [S x T], nParticlesMax,
 *       smcProposalType = 1, smcResampleType = 2, useOnlineMarginalSmoothing,
 *       epsilon, useOnlineParameterEstimation = false, ...)
 *     -> regimeProbabilityEstimates [T][1 + K] (position, P(r = 1..K))
 *   (singleGroup.cpp:76-189; called by bin/estimate_parameters_and_regimes:303-322).
 * Online parameter estimation (useOnlineParameterEstimation = TRUE, the
 * pipeline's --estimate_parameters) is the hyg_sg_*_pe family below. */
typedef struct hyg_sg_params {
  int32_t n_regimes;          /* K = vartheta[1] (model_functions.R:36-59)          */
  int32_t minimum_duration;   /* u = vartheta[0]                                    */
  int32_t num_particles_max;  /* nParticlesMax, 250 in the pipeline                 */
  int32_t resample_type;      /* smcResampleType: 2 = optimal finite state (only)    */
  int32_t is_kappa_fixed;     /* vartheta[2K+2]                                     */
  int32_t theta_len;          /* K(K-1) + K (+ K if kappa is estimated)             */
  double alpha[HYG_KMAX];     /* vartheta[2 .. K+1]                                  */
  double beta[HYG_KMAX];      /* vartheta[K+2 .. 2K+1]                               */
  double kappa[HYG_KMAX];     /* vartheta[2K+3 ..] when fixed                        */
  double theta[HYG_KMAX * (HYG_KMAX + 1)]; /* K rows of K-1 log-weights of P, K logit(omega), (K log kappa) */
  double epsilon;             /* smoothing variance threshold, 0.01                  */
} hyg_sg_params;

typedef struct hyg_sg_model hyg_sg_model;

/* One chain: the sites [site_begin, site_begin + n_sites) of the site-major
 * count arrays (one sample group on one chromosome). */
typedef struct hyg_sg_chain {
  int64_t site_begin;
  int32_t n_sites;
  int32_t _pad;
  uint64_t seed;
  uint64_t chain_id;
  int64_t out_begin;
} hyg_sg_chain;

void hyg_sg_params_default(hyg_sg_params* p);
/* Derived quantities of ModelParameters::setKnownParameters/setUnknownParameters
 * (singleGroup.h:173-335): P, omega, kappa and the hazard tables rho(d, r)
 * with the exit status, Beta-Binomial lgamma tables for counts <= max_total_reads. */
int hyg_sg_model_create(const hyg_sg_params* params, int32_t max_total_reads, int32_t max_duration,
                        hyg_sg_model** out);
void hyg_sg_model_destroy(hyg_sg_model* model);
/* E[t][r] = sum_s log BetaBinomial(meth_ts | tot_ts, alpha_r, beta_r)
 * (Model::evaluateLogObservationDensity, singleGroup.h:611-627). Device pointers, [T][S]. */
int hyg_sg_emission(const hyg_sg_model* model, const uint16_t* meth, const uint16_t* tot, int32_t n_samples,
                    int64_t n_sites, double* emission, void* stream);
/* Workspace for n_chains chains with room for `psi_capacity` pending smoothing
 * times per chain (the online-smoothing state; 0 = default 4096). */
size_t hyg_sg_workspace_bytes(const hyg_sg_model* model, int32_t n_chains, int32_t psi_capacity);
/* Runs SMC + online marginal smoothing for n_chains chains (one workgroup
 * each). regime_probs [rows][K] f64 receives the smoothed P(r_t = r) of every
 * site (OnlineCombinedInference.h:106-117), status [n_chains] HYG_OK /
 * HYG_ENUMERIC / HYG_ENOMEM (pending smoothing times exceeded psi_capacity). */
int hyg_sg_run_chains(const hyg_sg_model* model, const hyg_sg_chain* chains, int32_t n_chains,
                      const double* emission, void* workspace, size_t workspace_bytes, int32_t psi_capacity,
                      double* regime_probs, int32_t* status, void* stream);
/* Host-pointer convenience for one chain: counts [T][S]. */
int hyg_sg_run_chain_host(const hyg_sg_model* model, const uint16_t* meth, const uint16_t* tot,
                          int32_t n_samples, int32_t n_sites, uint64_t seed, uint64_t chain_id,
                          double* regime_probs);

/* ---- online parameter estimation
 * runOnlineCombinedInferenceCpp(..., useOnlineParameterEstimation = TRUE,
 *     normaliseGradients, useAdam, nStepsWithoutParameterUpdate,
 *     learningRateExponent, learningRateFactor, ...) -> thetaEstimates
 * (singleGroup.cpp:76-189, OnlineCombinedInference.h:48-118,
 * OnlineParameterEstimation.h:42-176, GradientAscent.h:62-155), run by the
 * two-group pipeline's `hygeia estimate_parameters_and_regimes ...
 * --estimate_regime_probabilities --estimate_parameters`
 * (modules/two_group/2_estimate_parameters_and_regimes.nf:38-52). The
 * regime probabilities are smoothed under the moving theta, as the reference.
 * With is_kappa_fixed = 0 theta holds K more entries log kappa_r and the
 * gradient is the reference's as written (singleGroup.h:664-692: the omega
 * coordinate takes d log rho / d theta_kappa, the kappa coordinates stay put;
 * include/hyg_sg_pe.h). */
typedef struct hyg_sg_pe_params {
  int32_t use_adam;               /* --use_adam, TRUE                          */
  int32_t normalise_gradients;    /* --normalise_gradients, FALSE              */
  int32_t n_steps_without_update; /* --n_steps_without_parameter_update, 200   */
  int32_t _pad;
  double learning_rate_exponent;  /* --learning_rate_exponent, 0.1             */
  double learning_rate_factor;    /* --learning_rate_factor, 0.01              */
} hyg_sg_pe_params;

void hyg_sg_pe_params_default(hyg_sg_pe_params* pe);
/* Rows of theta the chains report: per chain 1 + (n_sites - 1) / every (the
 * initial theta, then theta after each update at t = every, 2 every, ...);
 * chain i's rows follow chain i-1's. The reference's thetaEstimates row t
 * (t = 0 .. T-1) is row t / every of its chain. */
int64_t hyg_sg_pe_theta_rows(const hyg_sg_chain* chains, int32_t n_chains, int32_t every);
size_t hyg_sg_pe_workspace_bytes(const hyg_sg_model* model, const hyg_sg_chain* chains, int32_t n_chains,
                                 int32_t psi_capacity);
/* As hyg_sg_run_chains, with theta updated online; theta_out [rows][theta_len]
 * f64 (device; theta_len = K^2, or K (K + 1) with kappa estimated). status may also be HYG_ENOMEM when a sojourn outgrows the
 * hazard table (HYG_SGPE_DCAP rows) before the hazard's exit. */
int hyg_sg_run_chains_pe(const hyg_sg_model* model, const hyg_sg_pe_params* pe, const hyg_sg_chain* chains,
                         int32_t n_chains, const double* emission, void* workspace, size_t workspace_bytes,
                         int32_t psi_capacity, double* regime_probs, double* theta_out, int32_t* status,
                         void* stream);
/* Host-pointer convenience for one chain: regime_probs [T][K], theta_out
 * [1 + (T - 1) / every][K^2]. */
int hyg_sg_run_chain_host_pe(const hyg_sg_model* model, const hyg_sg_pe_params* pe, const uint16_t* meth,
                             const uint16_t* tot, int32_t n_samples, int32_t n_sites, uint64_t seed,
                             uint64_t chain_id, double* regime_probs, double* theta_out);

/* ================================================ aggregation and DMPs
 * The consumers of the two-group trajectories:
 *   aggregate_results.py:71-206  per-site means over every seed's trajectories
 *                                (split_probs = mean(merged == 0), regimes)
 *   get_dmps.py:46-180           test statistics 1 - #(r_ctrl != r_case) / P
 *                                (and 1 - #(r_ctrl = i, r_case = j) / P), FDR
 *                                and weighted-FDR selection, regime frequencies
 *   multiple_testing.py:3-22     FDR_procedure, weighted_FDR_procedure
 * on trajectories resident in HBM (the outputs of hyg_tg_run_chains). */

/* The job's gather of per-site posterior counts over trajectories and seeds
 * (what aggregate_results.py:129,181 averages; bench.py's step ends with it):
 * for every segment (out_row, site, n_rows) of the device array segments
 * [n_segments][3] int64 and every i < n_rows,
 *   counts[site + i][0]     += round(B * split[out_row + i])
 *   counts[site + i][1 + j] += round(B * regime[out_row + i][j]),  j < 2K,
 * round half to even (torch.round). split / regime are hyg_tg_outputs'
 * split_probs / regime_probs, means over the B trajectories, so B p is an
 * integer. counts [n_sites][1 + 2K] int32 (device) is added to, not cleared.
 * exclusive = 1: the caller guarantees that the call's segments cover disjoint
 * sites (e.g. the chains of one seed), and each count is a plain read-add-write
 * (coalesced; the C3 job's 56 M rows in about 2 ms per seed); exclusive = 0:
 * segments may share sites (several seeds in one call) and every add is an
 * integer atomic (the same sums, about 22 ms for the C3 job). The caller keeps
 * every row and site in range; max_rows (>= every n_rows) sizes the grid.
 * Asynchronous on stream. Replaces a torch gather / round / index_add chain
 * (parallel.posterior_counts, kept as the tests' reference). */
int hyg_tg_posterior_counts(const float* split, const float* regime, int32_t K, int32_t B,
                            const int64_t* segments, int32_t n_segments, int64_t max_rows, int32_t exclusive,
                            int32_t* counts, void* stream);

/* One chromosome segment: the same reported (trimmed) rows in every seed's
 * trajectory block. */
typedef struct hyg_dmp_group {
  int64_t site_begin; /* global site index of the first reported row */
  int64_t n_rows;     /* reported rows */
} hyg_dmp_group;

/* Per-site counts over the P = B * n_seeds trajectories of a site (device
 * pointers; host arrays `groups` [n_groups] and `block_rows`
 * [n_groups][n_seeds] = output row, in merged/control/kase, of the first
 * reported row of each seed's block):
 *   counts [n_sites][2 + 2K] int32 = (#(merged == 0), #(r_ctrl != r_case),
 *                                     #(r_ctrl == r) for r < K, #(r_case == r) for r < K)
 *   pairs  [n_sites][K][K]   int32 = #(r_ctrl == i and r_case == j), or NULL.
 * merged [rows][B], control/kase [rows][B][2] (d, r) int16 as hyg_tg_outputs.
 * Rows of sites outside every group are not written. */
int hyg_dmp_site_counts(const int16_t* merged, const int16_t* control, const int16_t* kase, int32_t B,
                        int32_t K, const hyg_dmp_group* groups, const int64_t* block_rows, int32_t n_groups,
                        int32_t n_seeds, int64_t n_sites, int32_t* counts, int32_t* pairs, void* stream);

/* FDR_procedure(t, fdr_threshold) (multiple_testing.py:3-12) for the
 * statistics t_i = 1 - c_i / P, c_i = counts[i * stride + column] (device),
 * 0 <= c_i <= P: the ascending sort is a counting sort by c (device), the
 * float64 running means np.cumsum(sorted) / (i + 1) are replayed exactly in
 * numpy's sequential order on the host. Outputs the reference's (k, Q_k,
 * threshold): (0, 0, 0) when fdr_threshold < min t; (n, Q_n, 1.01) when every
 * Q_i <= fdr_threshold (the reference's `s == shape` branch). Synchronises. */
int hyg_dmp_fdr(const int32_t* counts, int32_t stride, int32_t column, int64_t n, int32_t n_particles,
                double fdr_threshold, int64_t* k, double* q_k, double* threshold, void* stream);

/* weighted_FDR_procedure(t, fdr_threshold, w_fp, w_fn) (multiple_testing.py:14-22)
 * for the same statistics: ranking computed and sorted on the device (stable
 * LSD radix sort; the reference's np.argsort is not stable, so ties of the
 * ranking keep ascending site order here), Nsums = np.cumsum of the ranked
 * excess error rates replayed exactly on the host. ranked [n] (device,
 * int64) receives ranking_indices; *s the number selected (ranked[0:s]),
 * *n_sum = Nsums[s - 1] (Python indexing: the last sum when s = 0).
 * Synchronises. */
int hyg_dmp_weighted_fdr(const int32_t* counts, int32_t stride, int32_t column, int64_t n, int32_t n_particles,
                         double fdr_threshold, const double* w_fp, const double* w_fn, int64_t* ranked,
                         int64_t* s, double* n_sum, void* stream);

/* ================================================ regime BED tracks
 * make_bed_file (src/single_group/bin/make_bed_file:19-66)
 * on regime probabilities resident in HBM. */

/* Per site of regime_probs [n_sites][K] f64 (device): score = the largest
 * probability, label = the first regime attaining it, or -1 ("equiprobable")
 * when more than one does (data.table pmax / rowSums(.SD == score) / max.col
 * ties.method "first"). label [n_sites] int8, score [n_sites] f64 (device). */
int hyg_bed_labels(const double* regime_probs, int32_t K, int64_t n_sites, int8_t* label, double* score,
                   void* stream);
/* Host: the BED lines of fwrite(bed, sep = "\t", col.names = FALSE, scipen = 999)
 *   chrom  pos-1  pos+1  name  score  .  pos-1  pos+1  itemRgb
 * for sites already in output order (setkey(bed, chr, start)); names[K + 1]
 * = the regime column names then "equiprobable", rgb[K + 1] likewise; score
 * with at most 15 significant digits, trailing zeros dropped. Writes at most
 * out_bytes bytes; returns the bytes needed (call with out = NULL to size the
 * buffer) or a negative HYG_E* code. */
int64_t hyg_bed_format(const char* chrom, const int64_t* positions, const int8_t* label, const double* score,
                       int64_t n_sites, int32_t K, const char* const* names, const char* const* rgb, char* out,
                       int64_t out_bytes);

/* ================================================ preprocess (BED -> counts)
 * `hygeia preprocess` (src/two_group/preprocess_bed.py), the
 * device part for one sample on one chromosome: the strand collapse
 * (collapse_strands :183-259: "+" rows joined to "-" rows on end == start,
 * missing strand 0, key = start+ or start- - 1, rows with coverage > 0) and its
 * counts on the CpG grid (:298-336: meth = round(total avg / 100), unmeth =
 * round(total (100 - avg) / 100), half away from zero as polars; sites without
 * a collapsed row NaN, the reference's null). Device pointers; each strand's records sorted by start
 * with unique starts (the caller checks); coverage and percent as f64.
 * Writes counts[t * stride + column] = meth, [.. + 1] = unmeth for every site
 * (stride 2: one sample's contiguous [n_sites][2] block, the fastest layout);
 * plus_single_base != 0 promises end = start + 1 for every "+" record (the
 * pairing then needs no marking pass and no scratch); else scratch [n_minus]
 * bytes; *conflicts (device int, caller-zeroed) counts sites
 * that two collapsed rows claim (records longer than one base). */
int hyg_pre_collapse(const int64_t* cpg_pos0, int64_t n_sites, const int64_t* plus_start, const int64_t* plus_end,
                     const double* plus_coverage, const double* plus_percent, int64_t n_plus,
                     const int64_t* minus_start, const double* minus_coverage, const double* minus_percent,
                     int64_t n_minus, int32_t plus_single_base, uint8_t* scratch, double* counts, int32_t stride,
                     int32_t column, int32_t* conflicts, void* stream);

/* Number of visible HIP devices (0 when none: compute calls then fail). */
int hyg_device_count(void);

/* Device policy of concurrent task processes. The reference runs one CPU
 * process per (chrom, batch, seed) task (modules/two_group/4_infer.nf:28,42-48),
 * all at once under Nextflow's local executor (nextflow.config:17-21), and a
 * task never names a device; without a policy every task of an 8-GPU node
 * would land on device 0.
 *
 * hyg_device_slot_acquire takes the first free slot in the order
 * (slot 0 of device 0, 1, ..., n_devices - 1, slot 1 of device 0, ...), a slot
 * being an exclusive flock(2) on `<lock_dir>/hygeia_amd.gpu<d>.slot<j>.lock`
 * held until hyg_device_slot_release or the process exits (a crashed task
 * frees its slot), so concurrent tasks spread evenly over the devices: 16
 * tasks on 8 devices hold two slots each. No HIP call (n_devices is the
 * caller's: tests fake it). HYG_EINVAL when lock_dir is not usable or all
 * max_per_device slots of every device are held; one slot per process (a
 * second call returns the held one). hyg_set_device makes `device` the
 * calling thread's current HIP device (hipSetDevice): models created and
 * chains launched after it use that device. */
int hyg_device_slot_acquire(const char* lock_dir, int32_t n_devices, int32_t max_per_device, int32_t* device,
                            int32_t* slot);
int hyg_device_slot_release(void);
int hyg_set_device(int32_t device);
int hyg_get_device(void);
const char* hyg_last_error(void);
const char* hyg_version(void);

#ifdef __cplusplus
}
#endif
#endif /* HYGEIA_AMD_H */
