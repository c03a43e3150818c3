"""The two-group oracle against an EXACT enumeration of the model (CPU only).

The reference ships no fixtures and TF 2.3 cannot run here, so
the chain is pinned by an independent numpy/scipy restatement of the model
(tests/tg_exact_model.py) on tiny chains whose state space can be enumerated:

(i)   keep-all regime (M large: filter_and_smoother_algorithm.py:207-209 at every
      step): the particle filter enumerates every path, so the oracle's log Z
      must equal the exact log marginal likelihood given the phantom regime,
      and its normalised final weights, pooled by state, the exact filter
      marginal -- both to 1e-12;
(ii)  the backward simulation (filter_and_smoother_algorithm.py:368-447) draws
      i.i.d. from the exact smoothing distribution in that regime: chi-square
      tests of the per-site state marginals and of the (t, t+1) pair marginals
      pooled over seeds;
(iii) with M = 2-3 the optimal finite-state resampling (resampling_functions.py:
      7-52, systematic :56-69) and the weight correction -min(0, log c + W -
      lse) (filter_and_smoother_algorithm.py:238-270) are active; the estimate
      Z_hat must stay unbiased: the seed average of Z_hat / Z(r_ph) is 1 within
      its standard error.
"""
import math
import os
import sys
from collections import Counter

import numpy as np
import pytest
from scipy import stats

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tg_exact_model import ExactModel, phantom_regime, unpack  # noqa: E402

MODE_KEEP, MODE_OPTIMAL, MODE_UNBIASED = 0, 1, 2
KEEP_ALL_M = 64  # above the largest finite particle count of these chains (53)
# (K, T, data seed, u). u = 3 is the pipeline's min_cpg_sites_between_change_points
# (run_inference_two_groups.py:25-27, case_control_regime_model.py:80-87,111-168);
# with T >= 6 the minimum-duration gate binds (no change point and no merge
# switch before a duration reaches u).
KEEP_ALL_CASES = [(2, 5, 1, 2), (3, 4, 2, 2), (3, 3, 3, 2), (2, 6, 4, 2), (2, 1, 5, 2), (3, 2, 6, 2),
                  (2, 8, 7, 3), (3, 6, 8, 3), (2, 9, 9, 4), (3, 6, 10, 4)]
BACKWARD_CASES = [(2, 5, 11, 2), (3, 4, 12, 2), (2, 7, 13, 3), (3, 6, 14, 3), (2, 8, 15, 4)]
RESAMPLING_CASES = [(3, 8, 3, 24, 2), (3, 5, 3, 22, 2), (2, 7, 2, 23, 2), (3, 8, 3, 25, 3), (2, 9, 2, 26, 3),
                    (3, 8, 3, 27, 4)]


def _problem(oracle, K, T, seed, M, B, cov=12, p_random=True, u=2, S=1):
    rng = np.random.default_rng(seed)
    mu = [(i + 0.5) / K for i in range(K)]
    sg = [0.08 + 0.04 * (i % 2) for i in range(K)]
    if p_random:  # a non-uniform control transition matrix and omegas
        P = rng.dirichlet(np.ones(K - 1) * 2.0, size=K)
        Pm = np.zeros((K, K))
        for r in range(K):
            Pm[r, [c for c in range(K) if c != r]] = P[r]
        om = rng.uniform(0.6, 0.9, size=K)
        theta = oracle.theta_from(Pm, om)
    else:
        theta = None
    p = oracle.make_params(K=K, M=M, B=B, mu=mu, sigma=sg, theta=theta, u=u)
    theta = np.array(p.theta[: p.theta_len])
    tot = rng.poisson(cov, size=(T, 2 * S)).astype(np.uint16)
    # methylation levels drawn from the regimes, with a change in the case group
    lev = np.where(np.arange(T)[:, None] < T // 2, 0.2, 0.8) * np.repeat(np.array([[1.0, 0.5]]), S, 1) + \
        np.repeat(np.array([[0.1, 0.3]]), S, 1)
    meth = rng.binomial(tot.astype(np.int64), np.clip(lev, 0.01, 0.99)).astype(np.uint16)
    d = {"meth_control": meth[:, :S].copy(), "tot_control": tot[:, :S].copy(),
         "meth_case": meth[:, S:].copy(), "tot_case": tot[:, S:].copy()}
    ex = ExactModel(K, mu, sg, theta, u=u)
    E = oracle.emission(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
    E_ex = ex.emission(d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
    return p, ex, E, E_ex


@pytest.mark.parametrize("K,T,dseed", [(2, 5, 1), (3, 4, 2), (3, 3, 3), (2, 6, 4)])
def test_emission_matches_scipy(oracle, K, T, dseed):
    _, _, E, E_ex = _problem(oracle, K, T, dseed, M=10, B=5)
    np.testing.assert_allclose(E, E_ex, rtol=0, atol=1e-12)


@pytest.mark.parametrize("K,T,dseed,u", KEEP_ALL_CASES)
def test_keep_all_log_z_and_filter_marginal(oracle, K, T, dseed, u):
    M = KEEP_ALL_M
    p, ex, E, E_ex = _problem(oracle, K, T, dseed, M=M, B=4, u=u)
    seen = set()
    for seed in range(12):
        cid = 40 + seed
        out = oracle.chain(p, E, seed, cid, want_modes=True)
        assert out["status"] == 0
        assert np.all(out["modes"][1:] // 65536 == MODE_KEEP), "M too small for the keep-all regime"
        r_ph = phantom_regime(oracle, seed, cid, K)
        seen.add(r_ph)
        log_z, alphas, _, _ = ex.forward_backward(E_ex, r_ph)
        assert abs(out["log_z"] - log_z) < 1e-12 * max(1.0, abs(log_z)), (out["log_z"], log_z)
        # final weights pooled by state = exact filter marginal
        w, st = out["final_log_weights"], out["final_states"]
        fin = np.isfinite(w)
        pooled = Counter()
        for s, lw in zip(st[fin], w[fin]):
            pooled[unpack(s)] += math.exp(lw - out["log_z"])
        exact = {x: math.exp(a - log_z) for x, a in alphas[-1].items()}
        assert set(pooled) == set(exact)
        for x in exact:
            assert abs(pooled[x] - exact[x]) < 1e-12, (x, pooled[x], exact[x])
    assert len(seen) >= 2  # the phantom regime varies over seeds


def _chi2_pvalue(counts: Counter, probs: dict, n: int) -> float:
    """Pearson chi-square of observed counts against exact probabilities, bins
    with expectation < 5 pooled."""
    obs, exp, o_rest, e_rest = [], [], 0, 0.0
    for k, pk in probs.items():
        e = n * pk
        if e >= 5:
            obs.append(counts.get(k, 0))
            exp.append(e)
        else:
            o_rest += counts.get(k, 0)
            e_rest += e
    assert sum(counts.values()) == n
    assert all(k in probs for k in counts), "a drawn state has probability 0"
    if e_rest >= 5:
        obs.append(o_rest)
        exp.append(e_rest)
    if len(obs) < 2:
        return None
    obs, exp = np.array(obs, float), np.array(exp)
    exp *= obs.sum() / exp.sum()
    return float(stats.chisquare(obs, exp).pvalue)


def check_draws_follow_exact_smoother(oracle, ex, E_ex, K, T, u, B, seeds, cid, paths_of):
    """Pool the backward draws of every seed by phantom regime and chi-square
    them against the exact smoother: per-site and (t, t+1) pair marginals.
    paths_of(i, seed) -> (merged [T, B], control [T, B, 2], case [T, B, 2])."""
    exact = {}
    draws = {}
    for i, seed in enumerate(seeds):
        r_ph = phantom_regime(oracle, seed, cid, K)
        if r_ph not in exact:
            exact[r_ph] = ex.forward_backward(E_ex, r_ph)
            draws[r_ph] = [Counter() for _ in range(T)], [Counter() for _ in range(T - 1)]
        m, c, k = (a.astype(int) for a in paths_of(i, seed))
        for b in range(B):
            path = [(m[t, b], c[t, b, 0], c[t, b, 1], k[t, b, 0], k[t, b, 1]) for t in range(T)]
            for t in range(T):
                draws[r_ph][0][t][path[t]] += 1
            for t in range(T - 1):
                draws[r_ph][1][t][(path[t], path[t + 1])] += 1
    pvals = []
    for r_ph, (single, pair) in draws.items():
        _, _, smooth, pairs = exact[r_ph]
        n = sum(single[0].values())
        for t in range(T):
            pvals.append(_chi2_pvalue(single[t], smooth[t], n))
        for t in range(T - 1):
            pvals.append(_chi2_pvalue(pair[t], pairs[t], n))
    assert len(draws) >= 2
    pvals = [q for q in pvals if q is not None]
    # enough bins with mass to test (a longer minimum duration u leaves fewer
    # uncertain sites: no change point is possible before a duration reaches u)
    assert len(pvals) >= (2 * T if u <= 2 else T), len(pvals)
    # deterministic seeds: a fixed set of p-values; each must be unremarkable
    assert min(pvals) > 1e-4, sorted(pvals)[:5]
    # and, pooled, they must look uniform (no systematic bias). Where a site's
    # state fixes the next one (durations below u only continue), the single and
    # pair tests of those sites test the same draws and repeat one p-value: keep
    # one of each.
    distinct = sorted({round(q, 12) for q in pvals})
    assert stats.kstest(distinct, "uniform").pvalue > 1e-3, distinct


@pytest.mark.parametrize("K,T,dseed,u", BACKWARD_CASES)
def test_backward_draws_follow_exact_smoother(oracle, K, T, dseed, u):
    M, B, nseeds = KEEP_ALL_M, 60, 300
    p, ex, E, E_ex = _problem(oracle, K, T, dseed, M=M, B=B, cov=2, u=u)  # weak data: a spread-out posterior

    def paths_of(i, seed):
        out = oracle.chain(p, E, seed, 7)
        assert out["status"] == 0
        return out["merged"], out["control"], out["case"]

    check_draws_follow_exact_smoother(oracle, ex, E_ex, K, T, u, B, range(nseeds), 7, paths_of)


@pytest.mark.parametrize("K,T,M,dseed,u", RESAMPLING_CASES)
def test_resampling_keeps_z_unbiased(oracle, K, T, M, dseed, u):
    nseeds = 20000
    p, ex, E, E_ex = _problem(oracle, K, T, dseed, M=M, B=2, u=u)
    zex = {}
    ratios = []
    modes = Counter()
    for seed in range(nseeds):
        cid = 3
        r_ph = phantom_regime(oracle, seed, cid, K)
        if r_ph not in zex:
            zex[r_ph] = ex.forward_backward(E_ex, r_ph)[0]
        out = oracle.chain(p, E, seed, cid, want_modes=True)
        assert out["status"] == 0
        modes.update((out["modes"][1:] // 65536).tolist())
        ratios.append(math.exp(out["log_z"] - zex[r_ph]))
    assert modes[MODE_OPTIMAL] > nseeds  # the optimal resampling ran on most steps
    r = np.array(ratios)
    se = r.std() / math.sqrt(len(r))
    assert abs(r.mean() - 1.0) < 4 * se + 1e-3, (r.mean(), se, dict(modes))
    # the estimate is not degenerate: resampling actually adds variance
    assert r.std() > 1e-3


# ---------------------------------------------------------------------------
# The pipeline's K. K = 6 is the shape every BASELINE configuration but C5 runs
# (K = 12); K = 4 sits between. These are the first shapes at which the three
# uniform regime draws of the case transition (case_control_distributions.py:
# 246-291) have normalisers other than 1 and 1/2: branch 2 (a merged ancestor
# splits, the control continues) draws r_k' over K - 1 regimes, branch 3 over
# K - 1, branch 4 (the case changes while the control changed or moved
# elsewhere) over K - 2 -- at K = 6: 1/5, 1/5 and 1/4. u = 3 (the pipeline's
# min_cpg_sites_between_change_points) and 2 + 2 samples.
#
# Keep-all regime: at step t the filter keeps every finite particle of step
# t - 1, so M must cover the finite count of step T - 2: K = 6 has 5, 5, 5,
# 180, 680 paths at t = 0..4; K = 4 has 3, 3, 3, 48, 156. The GPU holds
# M <= 165 at K = 6 in LDS (N = 48 M candidates), so K = 6, T = 5 (M = 192)
# is a CPU (oracle) case only; the GPU runs K = 6 up to T = 4 and K = 4 up to
# T = 6 in the keep-all regime, and K = 6, T = 7 with resampling.
# (K, T, data seed, u, samples per group, M, gpu)
#
# Round 5 adds the stress shape K = 12 (BASELINE.json configs[4]): branch 2 and
# branch 3 draw over K - 1 = 11 regimes, a branch-4 change over K - 2 = 10.
# K = 12 has 11, 11, 11, 1584, 6908 finite paths at t = 0..4 (397 and 1047
# distinct states at t = 3, 4), so M = 16 keeps every path up to T = 4 (a GPU
# case: N = 168 M candidates fit the kernel's LDS up to M of about 58) and
# M = 1600 up to T = 5 (CPU only).
PIPELINE_KEEP_ALL = [(6, 4, 71, 3, 2, 64, True), (4, 5, 72, 3, 2, 64, True), (4, 6, 73, 3, 2, 160, True),
                     (6, 5, 74, 3, 2, 192, False), (12, 4, 101, 3, 2, 16, True), (12, 5, 102, 3, 2, 1600, False)]
PIPELINE_BACKWARD = [(6, 4, 81, 3, 2, 64, True), (4, 5, 82, 3, 2, 64, True), (6, 5, 83, 3, 2, 192, False),
                     (12, 4, 111, 3, 2, 16, True)]
# (K, T, M, data seed, u, samples per group): optimal finite-state resampling active
PIPELINE_RESAMPLING = [(6, 7, 4, 91, 3, 2), (6, 6, 10, 92, 3, 2), (4, 8, 6, 93, 3, 2),
                       (12, 5, 4, 121, 3, 2), (12, 5, 8, 122, 3, 2)]


def backward_seeds(K: int) -> int:
    """Seeds of the backward chi-square cases: at K = 12 a branch-4 change is
    rare enough (~1e-4 of the draws at T = 4) that 300 seeds x 60 draws would
    show it about once; 1000 show it a few times."""
    return 1000 if K == 12 else 300


def branch_mass(ex, pair):
    """Posterior mass of the case transition's branches over the sites of a
    chain, from the exact pairwise smoothing marginals: {(branch, change):
    expected number of such transitions}, change = the case regime is redrawn
    (d_k' = 1 outside branch 1)."""
    out = Counter()
    for d in pair:
        for (x, y), pr in d.items():
            b = ex.case_branch(x, y)
            out[(b, b != 1 and y[3] == 1)] += pr
    return out


@pytest.mark.parametrize("K", [6, 12])
def test_pipeline_k_visits_every_case_branch(oracle, K):
    """The K = 6 and K = 12 cases exercise the case transition's K-dependent
    normalisers: the exact smoother puts mass on branch 2 (1/(K-1): 1/5, 1/11),
    branch 3 (1/(K-1)) and a branch-4 change (1/(K-2): 1/4, 1/10), and replacing
    any of those normalisers by its neighbour moves the exact log Z by far more
    than the 1e-12 the keep-all tests allow -- so those tests pin them."""
    for K, T, dseed, u, S, M, _ in [c for c in PIPELINE_KEEP_ALL if c[0] == K]:
        p, ex, E, E_ex = _problem(oracle, K, T, dseed, M=M, B=4, u=u, S=S)
        r_ph = phantom_regime(oracle, 0, 40, K)
        log_z, _, _, pair = ex.forward_backward(E_ex, r_ph)
        mass = branch_mass(ex, pair)
        assert mass[(2, True)] > 1e-6, dict(mass)
        assert mass[(4, True)] > 1e-6, dict(mass)
        if T >= 5:  # a split ancestor whose control moves onto the case regime needs t >= u + 1
            assert mass[(3, True)] > 1e-9, dict(mass)
        for branch, size in ((2, K - 2), (4, K - 1)) + (((3, K - 2),) if T >= 5 else ()):
            wrong = ExactModel(K, [p.mu[i] for i in range(K)], [p.sigma[i] for i in range(K)],
                               np.array(p.theta[: p.theta_len]), u=u, case_uniform_sizes={branch: size})
            lz_wrong = wrong.forward_backward(E_ex, r_ph)[0]
            # at least 100 x the keep-all tolerance (1e-12 relative)
            assert abs(lz_wrong - log_z) > 1e-10 * abs(log_z), (branch, lz_wrong, log_z)


@pytest.mark.parametrize("K,T,dseed,u,S,M,gpu", PIPELINE_KEEP_ALL)
def test_pipeline_k_keep_all_log_z_and_filter_marginal(oracle, K, T, dseed, u, S, M, gpu):
    p, ex, E, E_ex = _problem(oracle, K, T, dseed, M=M, B=4, u=u, S=S)
    seen = set()
    for seed in range(8):
        cid = 40 + seed
        out = oracle.chain(p, E, seed, cid, want_modes=True)
        assert out["status"] == 0
        assert np.all(out["modes"][1:] // 65536 == MODE_KEEP), "M too small for the keep-all regime"
        r_ph = phantom_regime(oracle, seed, cid, K)
        seen.add(r_ph)
        log_z, alphas, _, _ = ex.forward_backward(E_ex, r_ph)
        assert abs(out["log_z"] - log_z) < 1e-12 * max(1.0, abs(log_z)), (out["log_z"], log_z)
        w, st = out["final_log_weights"], out["final_states"]
        fin = np.isfinite(w)
        pooled = Counter()
        for s, lw in zip(st[fin], w[fin]):
            pooled[unpack(s)] += math.exp(lw - out["log_z"])
        exact = {x: math.exp(a - log_z) for x, a in alphas[-1].items()}
        assert set(pooled) == set(exact)
        for x in exact:
            assert abs(pooled[x] - exact[x]) < 1e-12, (x, pooled[x], exact[x])
    assert len(seen) >= 2


def draws_branch_counts(ex, paths):
    """Case-branch transitions in drawn trajectories: {(branch, change): n}."""
    out = Counter()
    for path in paths:
        for x, y in zip(path[:-1], path[1:]):
            b = ex.case_branch(x, y)
            out[(b, b != 1 and y[3] == 1)] += 1
    return out


@pytest.mark.parametrize("K,T,dseed,u,S,M,gpu", PIPELINE_BACKWARD)
def test_pipeline_k_backward_draws_follow_exact_smoother(oracle, K, T, dseed, u, S, M, gpu):
    B, nseeds = 60, backward_seeds(K)
    p, ex, E, E_ex = _problem(oracle, K, T, dseed, M=M, B=B, cov=2, u=u, S=S)
    outs = {}

    def paths_of(i, seed):
        out = oracle.chain(p, E, seed, 7)
        assert out["status"] == 0
        outs[seed] = out
        return out["merged"], out["control"], out["case"]

    check_draws_follow_exact_smoother(oracle, ex, E_ex, K, T, u, B, range(nseeds), 7, paths_of)
    # the draws themselves take the K-dependent branches
    paths = []
    for out in outs.values():
        m, c, k = (a.astype(int) for a in (out["merged"], out["control"], out["case"]))
        paths += [[(m[t, b], c[t, b, 0], c[t, b, 1], k[t, b, 0], k[t, b, 1]) for t in range(T)] for b in range(B)]
    n = draws_branch_counts(ex, paths)
    assert n[(2, True)] > 0 and n[(4, True)] > 0, dict(n)


@pytest.mark.parametrize("K,T,M,dseed,u,S", PIPELINE_RESAMPLING)
def test_pipeline_k_resampling_keeps_z_unbiased(oracle, K, T, M, dseed, u, S):
    nseeds = 6000 if K == 12 else 12000  # K = 12: the GPU test runs 8192 seeds of the same chains
    p, ex, E, E_ex = _problem(oracle, K, T, dseed, M=M, B=2, u=u, S=S)
    zex = {}
    ratios = []
    modes = Counter()
    for seed in range(nseeds):
        cid = 3
        r_ph = phantom_regime(oracle, seed, cid, K)
        if r_ph not in zex:
            zex[r_ph] = ex.log_z(E_ex, r_ph)
        out = oracle.chain(p, E, seed, cid, want_modes=True)
        assert out["status"] == 0
        modes.update((out["modes"][1:] // 65536).tolist())
        ratios.append(math.exp(out["log_z"] - zex[r_ph]))
    assert modes[MODE_OPTIMAL] > nseeds
    r = np.array(ratios)
    se = r.std() / math.sqrt(len(r))
    assert abs(r.mean() - 1.0) < 4 * se + 1e-3, (r.mean(), se, dict(modes))
    assert r.std() > 1e-3


# The pipeline's M = 50 (run_inference_two_groups.py:37-39) with optimal
# finite-state resampling active: K = 6, T = 8, weak data (coverage 3) so that
# the resampling matters (Z_hat / Z spreads by ~1.5e-3). With M <= 64 the GPU
# resamples these steps by its top-set path (A <= 256 of the N = 2 400
# candidates, the cutoffs, the counting-sort fallback), so the GPU twin of this
# test checks that path against the exact Z, not only against the oracle.
# (K, T, M, data seed, u, samples per group, coverage)
PIPELINE_M50 = [(6, 8, 50, 134, 3, 2, 3)]


@pytest.mark.parametrize("K,T,M,dseed,u,S,cov", PIPELINE_M50)
def test_pipeline_m50_resampling_keeps_z_unbiased(oracle, K, T, M, dseed, u, S, cov):
    nseeds = 3000
    p, ex, E, E_ex = _problem(oracle, K, T, dseed, M=M, B=2, u=u, S=S, cov=cov)
    zex = {r: ex.log_z(E_ex, r) for r in range(K)}
    ratios, modes = [], Counter()
    for seed in range(nseeds):
        out = oracle.chain(p, E, seed, 3, want_modes=True)
        assert out["status"] == 0
        modes.update((out["modes"][1:] // 65536).tolist())
        ratios.append(math.exp(out["log_z"] - zex[phantom_regime(oracle, seed, 3, K)]))
    assert modes[MODE_OPTIMAL] >= 3 * nseeds  # every chain resamples optimally on several steps
    r = np.array(ratios)
    se = r.std() / math.sqrt(len(r))
    assert abs(r.mean() - 1.0) < 4 * se + 1e-6, (r.mean(), se, dict(modes))
    assert r.std() > 5e-4  # the resampling adds variance: the test can see a bias
