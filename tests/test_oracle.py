"""The CPU oracle (oracle/tg_oracle.c) of the two-group chain, CPU only.

* bit-identical to the independent pure-Python restatement (oracle/tg_oracle_np.py)
  on small chains (trajectories, probabilities, final weights, log Z);
* reproduces the committed golden fixtures (tests/golden/make_golden.py);
* statistical behaviour the reference's own simulation study checks
  (simulate_two_groups.py:273-319: recovered regimes / split probabilities);
* edge cases: T = 1, 2, zero coverage, K = 2 and 3, long saturated durations.
"""
import os

import numpy as np
import pytest

from hygeia_amd import synthetic as syn
from oracle import tg_oracle_np as onp

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
OUT_KEYS = ("merged", "control", "case", "split_probs", "regime_probs")


def _setup(oracle, K, M, B, T, S=2, cov=30.0, dseed=1):
    d = syn.simulate(T, S, S, K=K, seed=dseed, coverage=cov)
    mu, sg = syn.regime_params(K)
    p = oracle.make_params(K=K, M=M, B=B, mu=mu, sigma=sg)
    E = oracle.emission(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
    return d, p, E


@pytest.mark.parametrize("K,M,B,T,seed,cov", [(6, 8, 5, 120, 0, 30.0), (4, 6, 4, 150, 1, 30.0),
                                              (3, 5, 6, 200, 2, 10.0), (2, 4, 3, 90, 3, 30.0),
                                              (6, 12, 7, 60, 4, 100.0)])
def test_c_oracle_equals_python_restatement(oracle, K, M, B, T, seed, cov):
    d, p, E = _setup(oracle, K, M, B, T, cov=cov, dseed=seed + 1)
    c = oracle.consts(p)
    hz = {(g, r): oracle.hazard(p, g, r, T + 2) for g in range(2) for r in range(K)}
    model = onp.Model(c, hz, T + 2)
    a = oracle.chain(p, E, seed, 3)
    b = onp.run_chain(model, E, seed, 3)
    assert a["status"] == 0
    for k in OUT_KEYS:
        assert np.array_equal(a[k], b[k]), k
    fw = np.asarray(b["final_log_weights"])
    assert np.array_equal(a["final_log_weights"][:len(fw)], fw)
    assert np.all(a["final_log_weights"][len(fw):] == -np.inf)
    assert a["log_z"] == b["log_z"]


@pytest.mark.parametrize("name", ["tg_chain_k6", "tg_chain_k4"])
def test_golden_chain(oracle, name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    K, M, B = int(g["K"]), int(g["M"]), int(g["B"])
    p = oracle.make_params(K=K, M=M, B=B, mu=g["mu"], sigma=g["sigma"])
    E = oracle.emission(p, g["meth_control"], g["tot_control"], g["meth_case"], g["tot_case"])
    assert np.array_equal(E, g["E"])
    out = oracle.chain(p, E, int(g["seed"]), int(g["chain_id"]))
    assert out["status"] == 0
    for k in OUT_KEYS:
        assert np.array_equal(out[k], g[k]), k
    assert out["log_z"] == float(g["log_z"])
    assert np.array_equal(out["final_log_weights"], g["final_log_weights"])


def test_golden_tables(oracle):
    g = np.load(os.path.join(GOLDEN, "tg_tables.npz"))
    p = oracle.make_params(K=6)
    z = np.zeros((g["tot"].shape[0], 1), np.uint16)
    assert np.array_equal(oracle.emission(p, g["meth"], g["tot"], z, z), g["E"])
    for gi in range(2):
        for r in range(6):
            assert np.array_equal(oracle.hazard(p, gi, r, 200), g["hazard"][gi, r])


def test_trajectory_invariants(oracle):
    """Every sampled trajectory is a feasible path of the semi-Markov model:
    durations count up by one or restart at 1, regimes only change at a
    restart, merged steps have identical control/case states, and
    split/regime probabilities are the means over the B trajectories."""
    K, B = 6, 10
    _, p, E = _setup(oracle, K, 20, B, 800, cov=50.0, dseed=9)
    out = oracle.chain(p, E, 1, 77)
    m, ctl, cas = out["merged"].astype(int), out["control"].astype(int), out["case"].astype(int)
    # a merge (split -> merged) makes the case group take the control state
    # (merged_state_case_cp, case_control_proposal_mappings.py:88-103)
    merge = (m[1:] == 1) & (m[:-1] == 0)
    for g, arr in enumerate((ctl, cas)):
        d, r = arr[..., 0], arr[..., 1]
        assert np.all(d[0] == 1)
        step = d[1:] - d[:-1]
        ok = (d[1:] == 1) | (step == 1)
        if g == 1:
            ok |= merge
        assert np.all(ok)
        assert np.all((d[1:] == 1) | (r[1:] == r[:-1]) | (merge if g == 1 else False))
        assert np.all((r >= 0) & (r < K))
    mm = m == 1
    assert np.all(ctl[..., 0][mm] == cas[..., 0][mm]) and np.all(ctl[..., 1][mm] == cas[..., 1][mm])
    np.testing.assert_array_equal(out["split_probs"], (m == 0).mean(1).astype(np.float32))
    for r in range(K):
        np.testing.assert_array_equal(out["regime_probs"][:, r], (ctl[..., 1] == r).mean(1).astype(np.float32))
        np.testing.assert_array_equal(out["regime_probs"][:, K + r], (cas[..., 1] == r).mean(1).astype(np.float32))


def test_statistical_recovery(oracle):
    """simulate_two_groups.py:273-319 style: on simulated data the posterior
    regimes match the truth and split stretches get high split probability."""
    K = 6
    d, p, E = _setup(oracle, K, 50, 25, 3000, S=4, cov=100.0, dseed=21)
    out = oracle.chain(p, E, 0, 1)
    map_ctrl = out["regime_probs"][:, :K].argmax(1)
    assert (map_ctrl == d["regime_control"]).mean() > 0.9
    sp = out["split_probs"]
    split = d["split"]
    if split.any() and (~split).any():
        assert sp[split].mean() > sp[~split].mean() + 0.3


def test_determinism_and_seed_dependence(oracle):
    _, p, E = _setup(oracle, 6, 10, 5, 300, dseed=5)
    a = oracle.chain(p, E, 7, 11)
    b = oracle.chain(p, E, 7, 11)
    c = oracle.chain(p, E, 8, 11)
    for k in OUT_KEYS:
        assert np.array_equal(a[k], b[k])
    assert a["log_z"] == b["log_z"]
    assert not all(np.array_equal(a[k], c[k]) for k in OUT_KEYS)


@pytest.mark.parametrize("T", [1, 2, 3])
def test_tiny_chains(oracle, T):
    _, p, E = _setup(oracle, 6, 10, 5, T, dseed=6)
    out = oracle.chain(p, E, 0, 0)
    assert out["status"] == 0
    assert out["merged"].shape == (T, 5)
    assert np.all(out["merged"][0] == 1)  # t = 0 keeps only i == j candidates
    assert np.isfinite(out["log_z"])


def test_zero_coverage_is_prior_only(oracle):
    """With no reads the emission is exactly 0 and the chain is a draw from
    the prior; the run must still succeed and produce feasible paths."""
    K = 4
    p = oracle.make_params(K=K, M=10, B=6)
    E = np.zeros((500, 2 * K))
    out = oracle.chain(p, E, 3, 4)
    assert out["status"] == 0
    # the prior normalises to 1 up to the float32 model tables (500 steps)
    assert abs(out["log_z"]) < 1e-3


@pytest.mark.parametrize("K,M,B,T,S,seed", [(6, 50, 25, 300, 4, 0), (4, 8, 5, 200, 2, 1), (12, 20, 6, 60, 3, 2)])
def test_reference_structure_variant_equals_oracle(oracle, K, M, B, T, S, seed):
    """bench.py's reference-structure CPU baseline (per-particle Beta-Binomial,
    full-N history, [B, N] backward rows) computes the same chain."""
    d, p, E = _setup(oracle, K, M, B, T, S=S, cov=60.0, dseed=seed + 30)
    a = oracle.chain(p, E, seed, 5)
    b = oracle.chain_refstruct(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"], seed, 5)
    assert a["status"] == 0 and b["status"] == 0
    for k in OUT_KEYS:
        assert np.array_equal(a[k], b[k]), k
    assert a["log_z"] == b["log_z"]
