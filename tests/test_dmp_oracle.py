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


def tie_boundary_check(idx, ns, z):
    """A weighted-FDR cutoff inside a ranking tie group (golden tie_* case).
    The reference selects ranking_indices[:s] of an UNSTABLE np.argsort, so
    which tied sites it takes at the boundary is numpy's accident; the
    restatement (and the GPU radix sort) is stable and takes the lowest site
    indices of the group. Required: the same s and Nsums[s-1], the same sites
    outside the boundary tie group, and the same number from inside it."""
    c, P, thr, wfn = z["tie_counts"], int(z["tie_P"]), float(z["tie_thr"]), z["tie_wfn"]
    t = od.statistics_from_counts(c, P)
    rk = (t - thr) / (wfn * (1 - t) + np.abs(t - thr))
    ref = z["tie_widx"]
    assert len(idx) == len(ref) and ns == z["tie_wsum"]
    edge = rk[ref].max()
    group = rk == edge
    assert group.sum() > 1 and (~group[ref]).sum() < len(ref)  # the cutoff is inside a tie group
    sel = np.zeros(len(c), bool)
    sel[idx] = True
    want = np.zeros(len(c), bool)
    want[ref] = True
    np.testing.assert_array_equal(sel[~group], want[~group])
    assert sel[group].sum() == want[group].sum()
    return sel, want


def test_weighted_fdr_tie_at_cutoff_vs_reference_golden():
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "dmp_fdr.npz"))
    t = od.statistics_from_counts(z["tie_counts"], int(z["tie_P"]))
    idx, ns = od.weighted_fdr_procedure(t, float(z["tie_thr"]), np.ones(t.shape[0]), z["tie_wfn"])
    sel, want = tie_boundary_check(idx, ns, z)
    assert not np.array_equal(sel, want)  # the accident is real: the sets differ inside the group
