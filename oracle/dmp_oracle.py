"""CPU restatement of the aggregation / DMP-calling stage (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench tooling import this module; the
product package (hygeia_amd/) never does. It restates, in numpy:

  multiple_testing.py:3-12   FDR_procedure
  multiple_testing.py:14-22  weighted_FDR_procedure (argsort made stable: the
                             reference's default np.argsort is not, so only
                             tie-free rankings are order-defined there)
  get_dmps.py:46-101         test statistics and false-negative weights
  aggregate_results.py:129   split probabilities

Pinned against the reference's own multiple_testing.py, run in the build
container on the inputs of tests/golden/make_dmp_golden.py (the vectors are
committed in tests/golden/dmp_fdr.npz).
"""
from __future__ import annotations

import numpy as np


def fdr_procedure(t: np.ndarray, fdr_threshold: float):
    """(k, Q_k, threshold) of multiple_testing.py:3-12."""
    o = np.sort(np.asarray(t, dtype=np.float64))
    q = (1.0 / np.arange(1, o.shape[0] + 1, dtype=np.float64)) * np.cumsum(o)
    s = int(np.count_nonzero(q <= fdr_threshold))
    if fdr_threshold < o[0]:
        return 0, 0.0, 0.0
    if s == o.shape[0]:  # the reference's `s == test_statistics.shape` branch
        return s, float(q[s - 1]), 1.01
    return s, float(q[s - 1]), float(o[s])


def weighted_fdr_procedure(t, fdr_threshold, w_fp, w_fn):
    """(ranking_indices[:s], Nsums[s-1]) of multiple_testing.py:14-22 with a
    stable argsort."""
    t = np.asarray(t, dtype=np.float64)
    d = t - fdr_threshold
    ranking = w_fp * d / (w_fn * (1 - t) + w_fp * np.abs(d))
    idx = np.argsort(ranking, kind="stable")
    ns = np.cumsum((w_fp * d)[idx])
    s = int(np.count_nonzero(ns <= 0))
    return idx[:s], float(ns[s - 1])


def statistics_from_counts(c: np.ndarray, n_particles: int) -> np.ndarray:
    """1 - sum(indicator) / num_particles (get_dmps.py:68-69, 74)."""
    return 1.0 - np.asarray(c, dtype=np.int64) / n_particles


def site_counts(merged: np.ndarray, control_r: np.ndarray, case_r: np.ndarray, K: int):
    """Per-site counts over the particle axis of [T][P] arrays:
    (#merged==0, #(c != k), #(c == r)_r, #(k == r)_r) and pairs [T][K][K]."""
    T = merged.shape[0]
    out = np.zeros((T, 2 + 2 * K), dtype=np.int32)
    out[:, 0] = (merged == 0).sum(axis=1)
    out[:, 1] = (control_r != case_r).sum(axis=1)
    pairs = np.zeros((T, K, K), dtype=np.int32)
    for r in range(K):
        out[:, 2 + r] = (control_r == r).sum(axis=1)
        out[:, 2 + K + r] = (case_r == r).sum(axis=1)
        for j in range(K):
            pairs[:, r, j] = ((control_r == r) & (case_r == j)).sum(axis=1)
    return out, pairs


def false_negative_weights(positions: np.ndarray) -> np.ndarray:
    """1 / (1/3 (diff1 + diff2 + diff3)) of the positions, NaN -> 1e5
    (get_dmps.py:79-80, 101)."""
    p = np.asarray(positions, dtype=np.float64)
    n = p.shape[0]
    d = []
    for k in (1, 2, 3):
        x = np.full(n, np.nan)
        x[k:] = p[k:] - p[:-k]
        d.append(x)
    pd_ = 1 / 3 * (d[0] + d[1] + d[2])
    pd_ = np.where(np.isnan(pd_), 1e5, pd_)
    return 1.0 / pd_
