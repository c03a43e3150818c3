"""CPU oracle of single-group online parameter estimation (SURVEY.md 8f-1,
oracle/sg_oracle.c:oracle_sg_chain_pe + include/hyg_sg_pe.h), CPU only.

Pins, independently of the C code:
* the score recursion (OnlineParameterEstimation.h:118-156, gradients of
  singleGroup.h:641-717): with N_max >= K T nothing is resampled, the particle
  system is the exact filter and the filtered mean of phi is the exact score.
  One plain gradient step with learning rate 1 (GradientAscent.h:94-103)
  therefore moves theta by d log p(y_0:T-1) / d theta, checked against central
  finite differences of an exact semi-Markov forward recursion written here
  with scipy's NegBin. The P-block entries are the true gradient; the omega
  entries carry the reference's gradLogitEvaluatedAtInverseLogit(omega)
  = 2 + e^-omega + e^omega (misc.h:92-95) in place of d omega / d theta =
  omega (1 - omega), so they equal the true derivative times
  (2 + e^-omega + e^omega) / (omega (1 - omega));
* the hazard rows of the estimation path against scipy and against the
  fixed-theta tables (row S2);
* the ADAM step (GradientAscent.h:124-147) from the same score;
* learning rate 0: the estimation path reproduces the exact smoother;
* determinism, the committed golden fixture, and the unsupported kappa case.
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


def _data(K, T, S=2, seed=3, cov=8.0, omega=0.8):
    mu, sgm = syn.regime_params(K)
    d = syn.simulate(T, S, 1, K=K, seed=seed, coverage=cov, omega=omega, mu=mu, sigma=sgm)
    return d["meth_control"], d["tot_control"], mu, sgm


def loglik(theta, K, u, kappa, E):
    """log p(y_0:T-1 | theta) of the change-point model (singleGroup.h:556-627)
    by the exact forward recursion over states (d, r), d = 1..T."""
    T = E.shape[0]
    th = np.asarray(theta, float)
    P = np.zeros((K, K))
    for r in range(K):
        x = th[r * (K - 1):(r + 1) * (K - 1)]
        p = np.exp(x - x.max())
        p /= p.sum()
        P[r, [j for j in range(K) if j != r]] = p
    omega = 1.0 / (1.0 + np.exp(-th[K * (K - 1):K * K]))
    rho = np.zeros((K, T + 1))  # rho[r, d], d = sojourn 1..T
    for r in range(K):
        nb = stats.nbinom(kappa, 1.0 - omega[r])
        for d in range(u, T + 1):
            rho[r, d] = nb.pmf(d - u) / nb.sf(d - u - 1)
    g = np.exp(E - E.max(axis=1, keepdims=True))
    ll = float(E.max(axis=1).sum())
    a = np.zeros((T + 1, K))  # a[d, r]
    a[1] = g[0] / K
    s = a.sum()
    ll += math.log(s)
    a /= s
    for t in range(1, T):
        na = np.zeros_like(a)
        na[2:] = a[1:-1] * (1.0 - rho[:, 1:-1].T)
        cp = (a * rho.T).sum(axis=0)  # mass leaving each regime
        na[1] = cp @ P
        na *= g[t]
        s = na.sum()
        ll += math.log(s)
        a = na / s
    return ll


@pytest.mark.parametrize("K,T,u,seed", [(3, 50, 3, 1), (2, 90, 2, 2), (4, 40, 2, 3)])
def test_score_equals_finite_difference_gradient(sg, K, T, u, seed):
    meth, tot, mu, sgm = _data(K, T, seed=seed)
    p = sg.make_params(K=K, mu=mu, sigma=sgm, P=_P_uniform(K), omega=[0.8] * K, u=u, Nmax=250, epsilon=1e-300)
    assert K * T <= 250
    E = sg.emission(p, meth, tot)
    theta0 = np.array(p.theta[:K * K])
    # one plain step at t = T - 1 with learning rate 1: theta_1 - theta_0 = score
    pe = sg.make_pe(use_adam=False, every=T - 1, lr_exponent=0.0, lr_factor=1.0)
    out = sg.chain_pe(p, pe, E, seed=5, chain_id=1)
    assert out["status"] == 0
    np.testing.assert_array_equal(out["theta"][0], theta0)
    score = out["theta"][1] - theta0
    h = 1e-5
    fd = np.empty(K * K)
    for j in range(K * K):
        tp, tm = theta0.copy(), theta0.copy()
        tp[j] += h
        tm[j] -= h
        fd[j] = (loglik(tp, K, u, 2.0, E) - loglik(tm, K, u, 2.0, E)) / (2 * h)
    w = 1.0 / (1.0 + np.exp(-theta0[K * (K - 1):]))
    quirk = (2.0 + np.exp(-w) + np.exp(w)) / (w * (1.0 - w))  # gradLogit(omega) / (d omega / d theta)
    expect = fd.copy()
    expect[K * (K - 1):] *= quirk
    np.testing.assert_allclose(score, expect, rtol=2e-5, atol=2e-6)


def test_adam_step_from_the_score(sg):
    K, T, u = 3, 50, 3
    meth, tot, mu, sgm = _data(K, T, seed=1)
    p = sg.make_params(K=K, mu=mu, sigma=sgm, P=_P_uniform(K), omega=[0.8] * K, u=u, Nmax=250, epsilon=1e-300)
    E = sg.emission(p, meth, tot)
    theta0 = np.array(p.theta[:K * K])
    plain = sg.chain_pe(p, sg.make_pe(use_adam=False, every=T - 1, lr_exponent=0.0, lr_factor=1.0), E, 5, 1)
    g = plain["theta"][1] - theta0
    adam = sg.chain_pe(p, sg.make_pe(use_adam=True, every=T - 1, lr_exponent=0.1, lr_factor=0.01), E, 5, 1)
    b1, b2, eps, lr = 0.9, 0.999, math.exp(-8 * math.log(10)), 0.01 / 1.0 ** 0.1
    m, v = (1 - b1) * g, (1 - b2) * g * g
    expect = theta0 + lr * m / (np.sqrt(v / (1 - b2)) + eps) / (1 - b1)
    np.testing.assert_allclose(adam["theta"][1], expect, rtol=1e-9, atol=1e-12)
    # normalised plain step: g / |g|_1
    nrm = sg.chain_pe(p, sg.make_pe(use_adam=False, normalise_gradients=True, every=T - 1, lr_exponent=0.0,
                                    lr_factor=1.0), E, 5, 1)
    np.testing.assert_allclose(nrm["theta"][1] - theta0, g / np.abs(g).sum(), rtol=1e-9, atol=1e-12)


def test_learning_rate_zero_reproduces_exact_smoother(sg):
    from tests.test_sg_oracle import exact_smoother

    K, T, u = 3, 60, 3
    meth, tot, mu, sgm = _data(K, T, seed=1)
    p = sg.make_params(K=K, mu=mu, sigma=sgm, P=_P_uniform(K), omega=[0.8] * K, u=u, Nmax=250, epsilon=1e-300)
    E = sg.emission(p, meth, tot)
    out = sg.chain_pe(p, sg.make_pe(every=7, lr_factor=0.0), E, 3, 1)
    assert out["status"] == 0
    np.testing.assert_array_equal(out["theta"], np.tile(np.array(p.theta[:K * K]), (out["theta"].shape[0], 1)))
    np.testing.assert_allclose(out["regime_probs"], exact_smoother(sg, p, E, T), atol=1e-10)


@pytest.mark.parametrize("omega", [0.8, 0.9, 0.995])
def test_pe_hazard_rows_vs_scipy_and_fixed_tables(sg, omega):
    K, u, kappa, L = 2, 3, 2.0, 400
    p = sg.make_params(K=K, omega=(omega, omega), u=u, kappa=kappa)
    rows, Lr = sg.pe_hazard(p, np.array(p.theta[:K * K]), L)
    nb = stats.nbinom(kappa, 1.0 - omega)
    # the reference's rho = h / (1 - sum h) (sequential bigH) loses digits where the
    # survival probability is tiny: compare while it is above 1e-6
    n = min(Lr[0], 200, int(np.argmax(nb.sf(np.arange(400)) < 1e-6)) + u)
    d = np.arange(1, n + 1)  # sojourn d_prev, row d_prev - 1
    rho = np.where(d >= u, nb.pmf(d - u) / nb.sf(d - u - 1), 0.0)
    got = np.exp(rows[0, :n, 0])
    np.testing.assert_allclose(got[u - 1:], rho[u - 1:], rtol=1e-9)
    np.testing.assert_allclose(rows[0, :n, 1], np.log1p(-rho), rtol=1e-9, atol=1e-15)
    hz, _, _ = sg.hazard(p, 0, n)  # fixed-theta tables (libm) agree to rounding
    np.testing.assert_allclose(rows[0, u - 1:n, 0], hz[u - 1:, 0], rtol=1e-9)
    # d log rho / d theta_omega: finite difference of log rho in theta_omega, times the quirk ratio
    th = np.array(p.theta[:K * K])
    hstep = 1e-6
    tp, tm = th.copy(), th.copy()
    tp[K * (K - 1)] += hstep
    tm[K * (K - 1)] -= hstep
    rp, _ = sg.pe_hazard(p, tp, L)
    rm, _ = sg.pe_hazard(p, tm, L)
    m = min(n, 60)
    fd = (rp[0, u - 1:m, 0] - rm[0, u - 1:m, 0]) / (2 * hstep)
    quirk = (2.0 + math.exp(-omega) + math.exp(omega)) / (omega * (1.0 - omega))
    np.testing.assert_allclose(rows[0, u - 1:m, 2], fd * quirk, rtol=1e-4, atol=1e-6)
    # continuation entry: d log(1 - rho) = -rho / (1 - rho) d log rho
    r = np.exp(rows[0, u - 1:m, 0])
    np.testing.assert_allclose(rows[0, u - 1:m, 3], -rows[0, u - 1:m, 2] * r / (1 - r), rtol=1e-12, atol=1e-300)


def test_exit_onset_row(sg):
    """omega = 0.5: bigH reaches 1 in double; the onset row has rho = 1
    (base 0: log P alone), no continuation, and d log rho uses bigH = 0.99999
    (singleGroup.h:304-320)."""
    K = 2
    p = sg.make_params(K=K, omega=(0.5, 0.5), u=3, kappa=2.0)
    rows, Lr = sg.pe_hazard(p, np.array(p.theta[:K * K]), 2000)
    assert Lr[0] < 2000
    onset = rows[0, Lr[0] - 1]
    assert onset[0] == 0.0 and onset[1] == -np.inf and onset[3] == 0.0
    assert np.isfinite(rows[0, :Lr[0] - 1, 1]).all()


def test_determinism_golden_and_unsupported(sg):
    path = os.path.join(GOLDEN, "sg_pe_chain.npz")
    g = np.load(path)
    p = sg.make_params(K=6)
    E = sg.emission(p, g["meth"], g["tot"])
    pe = sg.make_pe(every=int(g["every"]))
    a = sg.chain_pe(p, pe, E, seed=int(g["seed"]), chain_id=int(g["chain_id"]))
    b = sg.chain_pe(p, pe, E, seed=int(g["seed"]), chain_id=int(g["chain_id"]))
    assert a["status"] == 0
    np.testing.assert_array_equal(a["regime_probs"], b["regime_probs"])
    np.testing.assert_array_equal(a["regime_probs"], g["regime_probs"])
    np.testing.assert_array_equal(a["theta"], g["theta"])
    # theta moved, P rows stay on the simplex, omega in (0, 1)
    assert not np.array_equal(a["theta"][0], a["theta"][-1])
    p.is_kappa_fixed = 0
    p.theta_len = 40  # kappa estimated needs K (K + 1) = 42 entries
    assert sg.chain_pe(p, pe, E[:10], 0, 0)["status"] == -1  # HYG_EINVAL


def test_digamma_vs_scipy(sg):
    from scipy import special

    for x in [1e-3, 0.01, 0.1, 0.5, 1.0, 1.4616321449683623, 2.0, 3.7, 9.99, 10.0, 10.5, 50.0, 1e3, 65537.25]:
        assert sg.digamma(x) == pytest.approx(float(special.digamma(x)), rel=1e-14, abs=1e-14), x
    assert math.isnan(sg.digamma(0.0)) and math.isnan(sg.digamma(-1.0))


def _ref_rows_kappa(K, u, kappa, omega, L):
    """extendAuxiliaryQuantities (singleGroup.h:271-335) with isKappaFixed_
    false, restated literally for one regime, and the omega coordinate of the
    gradient it then feeds (:657-668: the kappa derivative, written into the
    omega index): rows (log rho, log(1 - rho), gomg, gcont) up to the exit
    onset, with scipy's gammaln / digamma in place of libm / R's."""
    from scipy import special

    w, k = omega, kappa
    gl = 2.0 + math.exp(-w) + math.exp(w)  # gradLogitEvaluatedAtInverseLogit (misc.h:92-95)
    bigH, gOB, gKB = {}, {}, {}
    ex_prev = False
    out = []
    for d in range(L):
        if d < u - 1:
            bigH[d] = gOB[d] = gKB[d] = 0.0
            out.append((-np.inf, 0.0, 0.0, 0.0))
            continue
        x = d + 1 - u
        lh = math.exp(special.gammaln(x + k) - special.gammaln(k) - special.gammaln(x + 1.0)
                      + k * math.log(1.0 - w) + x * math.log(w))
        Hm1 = bigH.get(d - 1, 0.0)
        if ex_prev or Hm1 >= 1.0:
            bigH[d - 1] = Hm1 = 0.99999
            rho, exd = 1.0, True
        else:
            bigH[d] = Hm1 + lh
            rho, exd = lh / (1.0 - Hm1), False
        gO = (x / w - k / (1.0 - w)) * gl
        gOB[d] = gOB.get(d - 1, 0.0) + lh * gO
        gK = k * (special.digamma(x + k) - special.digamma(k) - math.log(1.0 - w))
        gKB[d] = gOB.get(d - 1, 0.0) + lh * gK  # the omega bigH gradient (:329)
        gomg = gK + gKB.get(d - 1, 0.0) / (1.0 - Hm1)
        base = 0.0 if exd else math.log(rho)
        cont = math.log(1.0 - rho) if (not exd and rho <= 1.0) else -np.inf
        gcont = (-gomg * rho) / (1.0 - rho) if (not exd and rho < 1.0) else 0.0
        out.append((base, cont, gomg, gcont))
        if exd:
            break
        ex_prev = exd
    return np.array(out)


@pytest.mark.parametrize("omega,kappa", [(0.8, 2.0), (0.95, 0.6), (0.99, 4.5)])
def test_kappa_estimated_hazard_rows_literal(sg, omega, kappa):
    K, u, L = 2, 3, 300
    p = sg.make_params(K=K, omega=(omega, omega), u=u, kappa=(kappa, kappa), kappa_fixed=False)
    rows, Lr = sg.pe_hazard(p, np.array(p.theta[:K * (K + 1)]), L)
    ref = _ref_rows_kappa(K, u, kappa, omega, L)
    # compare while the survival prod(1 - rho) stays above 1e-6 (the sequential
    # bigH sums lose digits where 1 - bigH is tiny)
    n = min(Lr[0], ref.shape[0])
    rho = np.where(np.arange(n) >= u - 1, np.exp(ref[:n, 0]), 0.0)
    alive = np.cumprod(1.0 - rho)
    m = max(int(np.argmax(alive < 1e-6)) if np.any(alive < 1e-6) else n, u + 5)
    np.testing.assert_allclose(rows[0, u - 1:m, 0], ref[u - 1:m, 0], rtol=1e-10)
    np.testing.assert_allclose(rows[0, u - 1:m, 2], ref[u - 1:m, 2], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(rows[0, u - 1:m, 3], ref[u - 1:m, 3], rtol=1e-9, atol=1e-12)
    # the kappa derivative differs from the omega one the fixed path carries
    pf = sg.make_params(K=K, omega=(omega, omega), u=u, kappa=kappa)
    rf, _ = sg.pe_hazard(pf, np.array(pf.theta[:K * K]), L)
    np.testing.assert_array_equal(rf[0, :m, 0], rows[0, :m, 0])
    assert not np.allclose(rf[0, u - 1:m, 2], rows[0, u - 1:m, 2])


def test_kappa_estimated_chain(sg):
    """Estimated kappa: log kappa never moves (its score is identically 0, the
    reference's gradient never writing the kappa index, singleGroup.h:664-692);
    with learning rate 0 the chain is the fixed-kappa chain at kappa =
    exp(log kappa); with ADAM theta's P / omega entries move along a different
    path from the fixed-kappa run (the omega coordinate follows d log rho /
    d theta_kappa)."""
    K, T, u = 3, 400, 3
    kappa = (1.5, 2.0, 3.0)
    meth, tot, mu, sgm = _data(K, T, seed=4)
    pk = sg.make_params(K=K, mu=mu, sigma=sgm, P=_P_uniform(K), omega=[0.9] * K, u=u, kappa=kappa, kappa_fixed=False)
    kap = np.exp(np.log(np.asarray(kappa)))
    pf = sg.make_params(K=K, mu=mu, sigma=sgm, P=_P_uniform(K), omega=[0.9] * K, u=u, kappa=kap)
    E = sg.emission(pk, meth, tot)
    pe = sg.make_pe(every=20)
    a = sg.chain_pe(pk, pe, E, 3, 1)
    assert a["status"] == 0 and a["theta"].shape == (1 + (T - 1) // 20, K * (K + 1))
    np.testing.assert_array_equal(a["theta"][:, K * K:], np.tile(np.log(np.asarray(kappa)), (a["theta"].shape[0], 1)))
    b = sg.chain_pe(pf, pe, E, 3, 1)
    assert b["status"] == 0
    np.testing.assert_array_equal(a["theta"][:, :K * (K - 1)][0], b["theta"][:, :K * (K - 1)][0])
    assert not np.array_equal(a["theta"][-1, :K * K], b["theta"][-1])
    z = sg.make_pe(every=20, lr_factor=0.0)
    a0, b0 = sg.chain_pe(pk, z, E, 3, 1), sg.chain_pe(pf, z, E, 3, 1)
    np.testing.assert_array_equal(a0["regime_probs"], b0["regime_probs"])
    np.testing.assert_array_equal(a0["theta"][:, :K * K], b0["theta"])
