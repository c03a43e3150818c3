"""CPU tests of the DMP-calling oracle (oracle/dmp_oracle.py) against the
reference's own multiple_testing.py outputs (tests/golden/dmp_fdr.npz, made by
tests/golden/make_dmp_golden.py), and of the get_dmps weight formula."""
import os

import numpy as np
import pytest

from oracle import dmp_oracle as od

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "dmp_fdr.npz")


def _cases():
    z = np.load(GOLD)
    return [(i, z) for i in range(int(z["n_cases"]))]


@pytest.mark.parametrize("i", range(8))
def test_fdr_matches_reference_golden(i):
    z = np.load(GOLD)
    t = od.statistics_from_counts(z[f"case_{i}_counts"], int(z[f"case_{i}_P"]))
    k, q, th = od.fdr_procedure(t, float(z[f"case_{i}_thr"]))
    g = z[f"case_{i}_fdr"]
    assert (k, q, th) == (int(g[0]), g[1], g[2])  # bit-exact


@pytest.mark.parametrize("i", range(8))
def test_weighted_fdr_matches_reference_golden(i):
    z = np.load(GOLD)
    t = od.statistics_from_counts(z[f"case_{i}_counts"], int(z[f"case_{i}_P"]))
    idx, ns = od.weighted_fdr_procedure(t, float(z[f"case_{i}_thr"]), np.ones(t.shape[0]), z[f"case_{i}_wfn"])
    np.testing.assert_array_equal(np.sort(idx), z[f"case_{i}_widx"])
    assert ns == z[f"case_{i}_wsum"]


def test_false_negative_weights_match_pandas_formula():
    """get_dmps.py:79-80,101 in pandas, against the numpy restatement."""
    pd = pytest.importorskip("pandas")
    z = np.load(GOLD)
    pos = z["case_0_pos"]
    idx = pd.DataFrame(pos)
    diffs = 1 / 3 * (idx.diff(1) + idx.diff(2) + idx.diff(3))
    ref = np.squeeze(1. / (diffs.fillna(1e+5).to_numpy()), -1)
    np.testing.assert_array_equal(od.false_negative_weights(pos), ref)
    np.testing.assert_array_equal(od.false_negative_weights(pos), z["case_0_wfn"])


def test_site_counts_definitions():
    rng = np.random.default_rng(3)
    T, P, K = 50, 40, 6
    m = rng.integers(0, 2, (T, P))
    c = rng.integers(0, K, (T, P))
    k = rng.integers(0, K, (T, P))
    out, pairs = od.site_counts(m, c, k, K)
    assert np.array_equal(out[:, 0], (m == 0).sum(1))
    assert np.array_equal(out[:, 1], P - np.trace(pairs, axis1=1, axis2=2))
    assert np.array_equal(out[:, 2:2 + K], pairs.sum(2))
    assert np.array_equal(out[:, 2 + K:], pairs.sum(1))
