"""Model tables of the two-group path against scipy and SURVEY.md Appendix C.

These pin the parts of the oracle that restate third-party arithmetic the
reference calls (tfp 0.11 BetaBinomial / NegativeBinomial, absent here):
case_control_regime_model.py:19-23 (alpha/beta), :111-168 (hazard),
:197-231 (emission); run_inference_two_groups.py:76-89, 110-167 (theta and the
merge/split matrix).
"""
import math

import numpy as np
import pytest
from scipy import special, stats

# Appendix C known answers (scipy, float64)
ALPHA = (17.1, 0.9, 12, 3, 12, 1)
BETA = (0.9, 17.1, 3, 12, 12, 1)
BB_27_30 = (-2.4295459334, -22.1441119005, -2.2568763832, -13.5643065905, -7.2607102908, -3.4339873230)
BB_15_30 = (-9.3939673419, -9.3939673419, -4.6950362008, -4.6950362008, -2.3459712375, -3.4339869953)
RHO = {
    0.8: (0, 0, 0.04, 0.0666666667, 0.0857142857, 0.1, 0.1111111111, 0.12),
    0.9: (0, 0, 0.01, 0.0181818182, 0.025, 0.0307692308, 0.0357142857, 0.04),
    0.995: (0, 0, 2.5e-05, 4.9751243781e-05, 7.4257425743e-05, 9.8522167488e-05),
}


def test_beta_params_appendix_c(oracle):
    c = oracle.consts(oracle.make_params(K=6))
    # mu/sigma are float32 in the reference (run_inference_two_groups.py:110-113)
    np.testing.assert_allclose([c.alpha[i] for i in range(6)], ALPHA, rtol=1e-5)
    np.testing.assert_allclose([c.beta[i] for i in range(6)], BETA, rtol=1e-5)
    assert (c.K, c.u, c.M, c.B, c.I, c.Nmax) == (6, 3, 50, 25, 48, 2400)
    c12 = oracle.consts(oracle.make_params(K=12))
    assert (c12.I, c12.Nmax) == (168, 8400)


def _emission_one(oracle, p, y, n):
    z = np.zeros((1, 1), np.uint16)
    E = oracle.emission(p, np.array([[y]], np.uint16), np.array([[n]], np.uint16), z, z)
    return E[0]


@pytest.mark.parametrize("y,n,want", [(27, 30, BB_27_30), (15, 30, BB_15_30)])
def test_betabinomial_known_answers(oracle, y, n, want):
    p = oracle.make_params(K=6)
    E = _emission_one(oracle, p, y, n)
    np.testing.assert_allclose(E[:6], want, rtol=0, atol=2e-6)  # float32 mu/sigma
    assert np.all(E[6:] == 0.0)  # case group has n = 0: contributes exactly 0


def test_betabinomial_grid_vs_scipy(oracle):
    p = oracle.make_params(K=6)
    c = oracle.consts(p)
    a = np.array([c.alpha[i] for i in range(6)])
    b = np.array([c.beta[i] for i in range(6)])
    rng = np.random.default_rng(5)
    T, S = 400, 3
    tot = rng.integers(0, 600, size=(T, S)).astype(np.uint16)
    tot[:5] = 0
    tot[5:10] = 65535
    meth = (rng.uniform(size=(T, S)) * (tot.astype(np.float64) + 1)).astype(np.int64)
    meth = np.minimum(meth, tot).astype(np.uint16)
    tk = rng.integers(0, 100, size=(T, 2)).astype(np.uint16)
    mk = (tk * rng.uniform(size=(T, 2))).astype(np.uint16)
    E = oracle.emission(p, meth, tot, mk, tk)
    for g, (y, n) in enumerate(((meth, tot), (mk, tk))):
        want = np.zeros((T, 6))
        for r in range(6):
            lp = stats.betabinom.logpmf(y.astype(np.int64), n.astype(np.int64), a[r], b[r])
            want[:, r] = np.where(n > 0, lp, 0.0).sum(axis=1)
        np.testing.assert_allclose(E[:, 6 * g:6 * g + 6], want, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("p_succ", sorted(RHO))
def test_hazard_known_answers(oracle, p_succ):
    """rho(d) for u=3, kappa=2 (Appendix C): the control row of regime 0 with
    omega_ctrl = p_succ; the case row with omega_case = p_succ."""
    p = oracle.make_params(K=6, omega_ctrl=p_succ, omega_case=p_succ)
    want = RHO[p_succ]
    for g in (0, 1):
        h = oracle.hazard(p, g, 0, len(want) + 1)
        rho = np.exp(h[1:, 0])
        # omega is float32 in the reference: 1 - f32(0.995) is 2e-6 off relative
        np.testing.assert_allclose(rho, want, rtol=5e-6, atol=0)
        om = float(np.float32(p_succ))
        nb = stats.nbinom(2, 1 - om)
        exact = [0.0 if d < 3 else nb.pmf(d - 3) / (1.0 - float(np.float32(nb.cdf(d - 4))))
                 for d in range(1, len(want) + 1)]  # survival from the float32 cdf
        np.testing.assert_allclose(rho, exact, rtol=1e-9, atol=0)
        np.testing.assert_allclose(np.exp(h[1:, 1]), 1.0 - np.asarray(want), rtol=1e-7)


def test_hazard_vs_scipy_and_f32_saturation(oracle):
    """h/S with the float32 cdf: where the f32 cdf rounds to 1 the reference's
    rho is inf/nan and is replaced by 0.1 (case_control_regime_model.py:120-124)."""
    p = oracle.make_params(K=6, omega_ctrl=0.8)
    h = oracle.hazard(p, 0, 0, 600)
    om = float(np.float32(0.8))
    nb = stats.nbinom(2, 1.0 - om)  # scipy's p = failure prob of tfp's probs
    sat = None
    for d in range(3, 600):
        x = d - 3
        cdf32 = np.float32(nb.cdf(x - 1)) if x > 0 else np.float32(0.0)
        if cdf32 == np.float32(1.0):
            sat = d
            break
        want = nb.pmf(x) / (1.0 - float(cdf32))
        assert math.isclose(math.exp(h[d, 0]), want, rel_tol=1e-9), d
    assert sat is not None and sat < 150
    assert np.all(np.exp(h[sat:, 0]) == pytest.approx(0.1, rel=1e-15))
    assert np.all(h[:3, 0] == -np.inf) and np.all(h[:3, 1] == 0.0)


def test_theta_softmax_and_merge_matrix(oracle):
    """theta -> log P_ctrl: each row a softmax of the K-1 off-diagonal entries
    (run_inference_two_groups.py:76-89); the merged-state matrix
    [[log(1-q_m), log q_m], [log q_s, log(1-q_s)]] (:164-167)."""
    K = 4
    rng = np.random.default_rng(6)
    P = rng.uniform(0.1, 1.0, (K, K))
    np.fill_diagonal(P, 0)
    P /= P.sum(1, keepdims=True)
    om = rng.uniform(0.5, 0.95, K)
    p = oracle.make_params(K=K, theta=oracle.theta_from(P, om), merge_log_prob=math.log(0.1), split_prob=0.01)
    c = oracle.consts(p)
    lPc = np.array([c.lPc[i] for i in range(K * K)]).reshape(K, K)
    assert np.all(np.diag(lPc) == -np.inf)
    off = ~np.eye(K, dtype=bool)
    np.testing.assert_allclose(np.exp(lPc[off]), P[off], rtol=1e-6)
    np.testing.assert_allclose([c.p_ctrl[i] for i in range(K)], om, rtol=1e-6)
    q_m, q_s = 0.1, 0.01
    np.testing.assert_allclose([c.lPm[i] for i in range(4)],
                               [math.log(1 - q_m), math.log(q_m), math.log(q_s), math.log(1 - q_s)], rtol=1e-6)
    assert c.log_M == pytest.approx(math.log(50))
    assert c.lU1 == pytest.approx(-math.log(K - 1))
    assert c.lU2 == pytest.approx(-math.log(K - 2))


def test_proposal_slots(oracle):
    """CaseControlProposal (case_control_proposal_mappings.py:11-216): the
    I = 2K + K^2 children of one ancestor; every child must be reachable
    (finite transition) from the ancestor, and the slot table is exhaustive:
    each finite-transition successor state appears at exactly one slot."""
    K = 4
    p = oracle.make_params(K=K)
    L = oracle.lib()
    I = 2 * K + K * K
    for anc in [(1, 5, 2, 5, 2), (0, 7, 1, 4, 3), (0, 2, 0, 9, 1), (1, 3, 3, 3, 3), (0, 3, 1, 3, 2)]:
        a = oracle.pack(*anc)
        kids = [L.oracle_tg_xi(K, a, s) for s in range(I)]
        finite = {k for k in kids if oracle.trans(p, a, k) > -math.inf}
        # brute force: every successor with finite density is some slot's child
        m, dc, rc, dk, rk = anc
        for m2 in (0, 1):
            for rc2 in range(K):
                for rk2 in range(K):
                    for dc2 in {1, dc + 1}:
                        for dk2 in {1, dk + 1, 0, dc2}:
                            s = oracle.pack(m2, dc2, rc2, dk2, rk2)
                            if oracle.trans(p, a, s) > -math.inf:
                                assert s in finite, (anc, oracle.unpack(s))


def test_zero_coverage_emission_is_zero(oracle):
    p = oracle.make_params(K=6)
    z = np.zeros((7, 4), np.uint16)
    E = oracle.emission(p, z, z, z, z)
    assert np.all(E == 0.0)


def test_lgamma_tables_match_special(oracle):
    """BB via log-factorial and lgamma(j + alpha) tables equals the direct
    lgamma formula of tfd.BetaBinomial.log_prob for large counts too."""
    p = oracle.make_params(K=6)
    c = oracle.consts(p)
    a, b = c.alpha[4], c.beta[4]
    n = np.array([[60000]], np.uint16)
    y = np.array([[31234]], np.uint16)
    z = np.zeros((1, 1), np.uint16)
    E = oracle.emission(p, y, n, z, z)
    want = (special.gammaln(60001) - special.gammaln(31235) - special.gammaln(60000 - 31234 + 1)
            + special.betaln(31234 + a, 60000 - 31234 + b) - special.betaln(a, b))
    assert E[0, 4] == pytest.approx(want, rel=1e-10)
