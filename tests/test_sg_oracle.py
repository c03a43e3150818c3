"""The CPU oracle of the single-group engine (oracle/sg_oracle.c), CPU only.

Pins, independently of the C code:
* the hazard tables against SURVEY.md Appendix C's known answers and a scipy
  NegBin restatement (row S2), the Beta-Binomial emission against
  scipy.stats.betabinom and Appendix C (row S4), P / omega from theta (S1);
* the whole SMC + online marginal smoothing (S5-S10) against an exact
  forward-backward smoother of the semi-Markov model written here in numpy:
  with N_max >= K T no particle is ever resampled, the particle system
  enumerates every (d, r) state and the smoothed probabilities must equal the
  exact ones (epsilon ~ 0 stores every time at the final step);
* the resampled filter (S7) statistically: the seed-average of smoothed
  probabilities with a small N_max approaches the exact smoother;
* golden fixture (tests/golden/make_golden.py) and seed determinism.
Against the reference binary itself parity is unpinned (RcppArmadillo absent).
"""
import math
import os

import numpy as np
import pytest
from scipy import stats

from hygeia_amd import synthetic as syn

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def sg():
    from oracle import sg_binding

    sg_binding.lib()
    return sg_binding


def _P_uniform(K):
    P = np.full((K, K), 1.0 / (K - 1))
    np.fill_diagonal(P, 0.0)
    return P


# ---------------------------------------------------------------- tables
@pytest.mark.parametrize("omega,expect", [
    (0.8, [0, 0, 0.04, 0.0666666667, 0.0857142857, 0.1, 0.1111111111, 0.12]),
    (0.9, [0, 0, 0.01, 0.0181818182, 0.025, 0.0307692308, 0.0357142857, 0.04]),
    (0.995, [0, 0, 2.5e-05, 4.9751243781e-05, 7.4257425743e-05, 9.8522167488e-05]),
])
def test_hazard_known_answers(sg, omega, expect):
    p = sg.make_params(K=2, omega=(omega, omega), u=3, kappa=2.0)
    hz, ex, _ = sg.hazard(p, 0, len(expect))
    rho = np.exp(hz[:, 0])
    np.testing.assert_allclose(rho, expect, rtol=1e-9, atol=1e-15)
    assert not ex.any()
    # continuation log(1 - rho)
    np.testing.assert_allclose(hz[:, 1], np.log1p(-rho), rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("u,kappa,omega", [(1, 2.0, 0.9), (3, 2.0, 0.995), (5, 3.5, 0.7), (2, 1.0, 0.5)])
def test_hazard_vs_scipy_negbin(sg, u, kappa, omega):
    """rho(d) = h(d) / (1 - H(d - 1)), h(d) = NB(d - u; kappa, omega), 0 below u."""
    n = 400
    p = sg.make_params(K=2, omega=(omega, omega), u=u, kappa=kappa)
    hz, ex, _ = sg.hazard(p, 1, n)
    d = np.arange(1, n + 1)
    h = np.where(d >= u, stats.nbinom.pmf(d - u, kappa, 1.0 - omega), 0.0)
    Hm1 = np.concatenate([[0.0], np.cumsum(h)[:-1]])
    live = (~ex.astype(bool)) & (1.0 - Hm1 > 1e-6)
    rho = np.where(d >= u, h / np.maximum(1.0 - Hm1, 1e-300), 0.0)
    np.testing.assert_allclose(np.exp(hz[live, 0]), rho[live], rtol=1e-7, atol=1e-300)
    # once the cumulative mass reaches one the row exits: rho = 1, no continuation
    if ex.any():
        first = int(np.argmax(ex))
        assert np.all(ex[first:]) and np.all(hz[first:, 0] == 0.0) and np.all(hz[first:, 1] == -np.inf)


def test_emission_vs_scipy_and_known_answers(sg):
    p = sg.make_params(K=6)
    a, b = sg.beta_params(sg.DEFAULT_MU, sg.DEFAULT_SIGMA)
    np.testing.assert_allclose(a, [17.1, 0.9, 12, 3, 12, 1], rtol=1e-6)
    np.testing.assert_allclose(b, [0.9, 17.1, 3, 12, 12, 1], rtol=1e-6)
    E = sg.emission(p, np.array([[27]]), np.array([[30]]))
    np.testing.assert_allclose(E[0], [-2.4295459334, -22.1441119005, -2.2568763832, -13.5643065905,
                                      -7.2607102908, -3.4339873230], atol=2e-9)
    E = sg.emission(p, np.array([[15]]), np.array([[30]]))
    np.testing.assert_allclose(E[0], [-9.3939673419, -9.3939673419, -4.6950362008, -4.6950362008,
                                      -2.3459712375, -3.4339869953], atol=2e-9)
    rng = np.random.default_rng(5)
    tot = rng.integers(0, 200, size=(300, 3))
    meth = rng.integers(0, 201, size=(300, 3)) % (tot + 1)
    E = sg.emission(p, meth, tot)
    ref = sum(stats.betabinom.logpmf(meth[:, s, None], tot[:, s, None], a[None], b[None]) for s in range(3))
    np.testing.assert_allclose(E, ref, rtol=1e-9, atol=1e-9)
    # n = 0 contributes the lgamma round-off, not exactly 0 (Appendix C)
    E0 = sg.emission(p, np.array([[0]]), np.array([[0]]))
    assert abs(E0[0, 0]) < 1e-12
    # y > n: density -inf
    assert np.all(sg.emission(p, np.array([[5]]), np.array([[3]])) == -np.inf)


def test_consts_from_theta(sg):
    K = 4
    rng = np.random.default_rng(2)
    P = rng.random((K, K))
    np.fill_diagonal(P, 0.0)
    P /= P.sum(axis=1, keepdims=True)
    om = np.array([0.9, 0.8, 0.95, 0.7])
    c = sg.consts(sg.make_params(K=K, P=P, omega=om))
    logP = np.array(c.logP[:K * K]).reshape(K, K)
    with np.errstate(divide="ignore"):
        np.testing.assert_allclose(np.exp(logP), P, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(np.array(c.omega[:K]), om, rtol=1e-12)
    assert np.all(np.isneginf(np.diag(logP)))


# --------------------------------------------- exact semi-Markov smoother
def exact_smoother(sg, p, E, T):
    """Forward-backward over the states (d, r), d = 1..T, of the model of row S3."""
    K = p.n_regimes
    c = sg.consts(p)
    logP = np.array(c.logP[:K * K]).reshape(K, K)
    with np.errstate(divide="ignore"):
        Pm = np.exp(logP)
    rho = np.zeros((K, T + 1))
    for r in range(K):
        hz, ex, _ = sg.hazard(p, r, T + 1)
        rho[r] = np.where(ex.astype(bool), 1.0, np.exp(hz[:, 0]))
    cont = np.zeros((K, T + 1))
    for r in range(K):
        hz, ex, _ = sg.hazard(p, r, T + 1)
        cont[r] = np.exp(hz[:, 1])
    n = T * K  # state index (d - 1) * K + r
    A = np.zeros((n, n))
    for d in range(1, T + 1):
        for r in range(K):
            i = (d - 1) * K + r
            if d < T:
                A[i, d * K + r] = cont[r, d - 1]
            for r1 in range(K):
                if r1 != r and d >= p.minimum_duration:
                    A[i, r1] += rho[r, d - 1] * Pm[r, r1]
    g = np.exp(E - E.max(axis=1, keepdims=True))
    alpha = np.zeros((T, n))
    alpha[0, :K] = g[0] / K
    alpha[0] /= alpha[0].sum()
    for t in range(1, T):
        a = alpha[t - 1] @ A
        a *= np.tile(g[t], T)
        alpha[t] = a / a.sum()
    beta = np.ones(n)
    post = np.zeros((T, K))
    for t in range(T - 1, -1, -1):
        if t < T - 1:
            beta = A @ (np.tile(g[t + 1], T) * beta)
            beta /= beta.max()
        m = alpha[t] * beta
        post[t] = m.reshape(T, K).sum(axis=0) / m.sum()
    return post


def _data(K, T, S=2, seed=3, cov=8.0, omega=0.8):
    mu, sgm = syn.regime_params(K)
    d = syn.simulate(T, S, 1, K=K, seed=seed, coverage=cov, omega=omega, mu=mu, sigma=sgm)
    return d["meth_control"], d["tot_control"], d["regime_control"], mu, sgm


@pytest.mark.parametrize("K,T,u,seed", [(3, 60, 3, 1), (2, 100, 2, 2), (4, 45, 1, 3), (3, 70, 5, 4)])
def test_smc_without_resampling_is_exact_smoother(sg, K, T, u, seed):
    meth, tot, _, mu, sgm = _data(K, T, seed=seed)
    p = sg.make_params(K=K, mu=mu, sigma=sgm, P=_P_uniform(K), omega=[0.8] * K, u=u, Nmax=250, epsilon=1e-300)
    assert K * T <= 250
    E = sg.emission(p, meth, tot)
    out = sg.chain(p, E, seed=7, chain_id=1, want_nparts=True)
    assert out["status"] == 0
    np.testing.assert_array_equal(out["nparts"], K * np.arange(1, T + 1))
    ref = exact_smoother(sg, p, E, T)
    np.testing.assert_allclose(out["regime_probs"], ref, atol=1e-10)


def test_epsilon_rule_gives_filtered_lag_estimates(sg):
    """With epsilon = 0.01 each time is emitted once its filtered variance is
    small: the estimates stay close to the exact smoother (here <= 0.2)."""
    K, T = 3, 70
    meth, tot, _, mu, sgm = _data(K, T, seed=11, cov=20.0)
    p = sg.make_params(K=K, mu=mu, sigma=sgm, P=_P_uniform(K), omega=[0.8] * K, Nmax=250, epsilon=0.01)
    E = sg.emission(p, meth, tot)
    out = sg.chain(p, E, seed=1)
    ref = exact_smoother(sg, p, E, T)
    assert np.max(np.abs(out["regime_probs"] - ref)) < 0.2
    assert np.allclose(out["regime_probs"].sum(axis=1), 1.0, atol=1e-12)


def test_resampled_filter_is_close_to_exact_on_average(sg):
    K, T = 3, 60
    meth, tot, _, mu, sgm = _data(K, T, seed=21, cov=6.0)
    p = sg.make_params(K=K, mu=mu, sigma=sgm, P=_P_uniform(K), omega=[0.8] * K, Nmax=15, epsilon=1e-300)
    E = sg.emission(p, meth, tot)
    ref = exact_smoother(sg, p, E, T)
    runs = [sg.chain(p, E, seed=s, chain_id=2, want_nparts=True) for s in range(40)]
    assert all(r["status"] == 0 for r in runs)
    assert all(r["nparts"].max() == 15 for r in runs)
    avg = np.mean([r["regime_probs"] for r in runs], axis=0)
    assert np.mean(np.abs(avg - ref)) < 0.03
    assert np.max(np.abs(avg - ref)) < 0.25


def test_pipeline_config_recovers_regimes(sg):
    meth, tot, truth, mu, sgm = _data(6, 4000, S=2, seed=5, cov=15.0, omega=0.95)
    p = sg.make_params(K=6)
    E = sg.emission(p, meth, tot)
    out = sg.chain(p, E, seed=3, want_nparts=True)
    assert out["status"] == 0
    pr = out["regime_probs"]
    assert np.all(np.isfinite(pr)) and np.all(pr >= 0) and np.all(pr <= 1 + 1e-12)
    np.testing.assert_allclose(pr.sum(axis=1), 1.0, atol=1e-12)
    assert out["nparts"].max() == 250
    # regimes 5 and 6 (mu 0.5, sd 0.1 vs uniform) are hard to tell apart
    hard = np.isin(truth, [4, 5])
    acc = np.mean(pr.argmax(axis=1)[~hard] == truth[~hard])
    assert acc > 0.9, acc


def test_determinism_and_seed_dependence(sg):
    meth, tot, _, _, _ = _data(6, 1500, seed=8, cov=10.0)
    p = sg.make_params(K=6)
    E = sg.emission(p, meth, tot)
    a = sg.chain(p, E, seed=5, chain_id=9)["regime_probs"]
    b = sg.chain(p, E, seed=5, chain_id=9)["regime_probs"]
    assert np.array_equal(a, b)
    # at N_max = 250 the six dropped particles are negligible ones whatever the
    # uniform; with a small N_max the residual draw matters
    p30 = sg.make_params(K=6, Nmax=30)
    a = sg.chain(p30, E, seed=5, chain_id=9)["regime_probs"]
    c = sg.chain(p30, E, seed=6, chain_id=9)["regime_probs"]
    d = sg.chain(p30, E, seed=5, chain_id=10)["regime_probs"]
    assert not np.array_equal(a, c) and not np.array_equal(a, d)
    assert np.mean(np.abs(a - c)) < 0.05


def test_edge_cases(sg):
    p = sg.make_params(K=6)
    # one site: the prior-weighted posterior of site 0
    E = sg.emission(p, np.array([[3, 1]]), np.array([[10, 4]]))
    out = sg.chain(p, E, seed=0)
    w = np.exp(E[0] - E[0].max())
    np.testing.assert_allclose(out["regime_probs"][0], w / w.sum(), rtol=1e-12)
    # zero coverage everywhere with exchangeable regimes: the uniform prior
    # (exact while N < N_max; afterwards the resampling breaks the symmetry a little)
    ps = sg.make_params(K=6, omega=[0.9] * 6)
    z = np.zeros((80, 2), np.uint16)
    out = sg.chain(ps, sg.emission(ps, z[:40], z[:40]), seed=0)
    assert out["status"] == 0
    np.testing.assert_allclose(out["regime_probs"], 1.0 / 6.0, atol=1e-9)
    out = sg.chain(ps, sg.emission(ps, z, z), seed=0)
    np.testing.assert_allclose(out["regime_probs"], 1.0 / 6.0, atol=0.03)
    # an impossible site (y > n) makes every weight -inf
    meth = np.array([[1], [5], [1]])
    tot = np.array([[2], [3], [2]])
    out = sg.chain(p, sg.emission(p, meth, tot), seed=0)
    assert out["status"] == -2


@pytest.mark.parametrize("name", ["sg_chain_k6", "sg_chain_k3"])
def test_golden_chain(sg, name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    K = int(g["K"])
    p = sg.make_params(K=K, mu=g["mu"], sigma=g["sigma"], P=g["P"], omega=g["omega"], u=int(g["u"]),
                       Nmax=int(g["Nmax"]), epsilon=float(g["epsilon"]))
    E = sg.emission(p, g["meth"], g["tot"])
    assert np.array_equal(E, g["E"])
    out = sg.chain(p, E, int(g["seed"]), int(g["chain_id"]))
    assert out["status"] == 0
    assert np.array_equal(out["regime_probs"], g["regime_probs"])


def test_concurrent_chains_equal_sequential_runs():
    """The oracle runs chains in threads (the GPU config tests, the CPU
    baselines): concurrent chains must not share sort state. A shared qsort key
    pointer made concurrently sorted chains read each other's weights."""
    import concurrent.futures as cf

    from hygeia_amd import synthetic as syn
    from oracle import sg_binding as sgb

    p = sgb.make_params(K=6)
    runs = []
    for i in range(4):
        d = syn.simulate(6000, 2, 1, K=6, seed=300 + i, coverage=100.0, omega=syn.SG_OMEGA)
        runs.append(sgb.emission(p, d["meth_control"], d["tot_control"]))
    seq = [sgb.chain(p, E, seed=i, chain_id=9) for i, E in enumerate(runs)]
    with cf.ThreadPoolExecutor(max_workers=4) as ex:
        par = list(ex.map(lambda a: sgb.chain(p, a[1], seed=a[0], chain_id=9), enumerate(runs)))
    for a, b in zip(seq, par):
        assert a["status"] == b["status"] == 0
        np.testing.assert_array_equal(a["regime_probs"], b["regime_probs"])


@pytest.mark.parametrize("S,Nmax", [(1, 250), (4, 250), (2, 30)])
def test_reference_structure_variant_equals_oracle(sg, S, Nmax):
    # the CPU baseline's variant evaluates the Beta-Binomial from the counts at
    # every use (9 lgamma per sample, inside the loop over previous particles
    # for the fresh ones, as computeWeightsCp does): the same chain, bit for bit
    meth, tot, _, _, _ = _data(6, 700, S=S, seed=11 + S, cov=12.0)
    p = sg.make_params(K=6, Nmax=Nmax)
    a = sg.chain(p, sg.emission(p, meth, tot), seed=3, chain_id=4)
    b = sg.chain_refstruct(p, meth, tot, seed=3, chain_id=4)
    assert a["status"] == b["status"] == 0
    assert np.array_equal(a["regime_probs"], b["regime_probs"], equal_nan=True)
