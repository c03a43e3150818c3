"""The single-group kernel's keep-top certificate (sg_kernels.hip, resampleCp).

With fewer than M weights whose F = 100 image is nonzero, the K / log c fixed
point of optimalFiniteState (reference resample.h:333-342, restated in
oracle/sg_oracle.c sg_chain_core) always ends with a non-finite log c, i.e. in
the keep-top fallback, so the kernel skips the loop on such steps. This runs
the oracle's loop, in the contract's arithmetic (det_log, exact F = 100 images,
the truncating u128 -> f64 conversion), on adversarial weight vectors and
checks the claim; the GPU chain tests check the kernel against the oracle.
"""
import math

import numpy as np
import pytest

from oracle.tg_oracle_np import det_log, fix100


def _u128_to_f64(v: int) -> float:
    # hyg_u128_to_f64(a, 100): the top 53 bits, truncated
    if v == 0:
        return 0.0
    p = v.bit_length() - 1
    if p <= 52:
        return math.ldexp(float(v), -100)
    sh = p - 52
    return math.ldexp(float(v >> sh), sh - 100)


def _k_loop(w_sorted, M):
    """oracle/sg_oracle.c K loop on weights sorted descending; returns (K, log c)."""
    Np = len(w_sorted)
    logq = [det_log(q) if q > 0 else -math.inf for q in w_sorted]
    cum = [0] * (Np + 1)
    for q in range(Np - 1, -1, -1):
        cum[q] = cum[q + 1] + fix100(w_sorted[q])
    k_old, k_new, log_c = 1, 0, 0.0
    while k_new != k_old:
        k_old = k_new
        mk = M - k_old
        lm = det_log(float(mk)) if mk > 0 else (-math.inf if mk == 0 else math.nan)
        Qk = _u128_to_f64(cum[k_old])
        lQ = det_log(Qk) if Qk > 0 else -math.inf
        log_c = lm - lQ  # IEEE: -inf - (-inf) is NaN
        thr = -log_c
        k_new = k_old + sum(1 for q in range(k_old, Np) if logq[q] > thr)
    return k_new, log_c


def _weights(rng, Np, nz, kind):
    """Np descending weights, exactly nz of them >= 2^-100."""
    tiny = 2.0 ** -100
    if kind == "geometric":
        big = np.exp(-rng.uniform(0.0, 60.0) * np.sort(rng.random(nz)))
    elif kind == "flat":
        big = 1.0 + 1e-12 * rng.random(nz)  # near-ties at the margin
    elif kind == "edge":
        big = tiny * (1.0 + rng.random(nz))  # every nonzero image small
        big[0] = 1.0
    else:  # one dominant weight, the rest just above the image threshold
        big = np.full(nz, tiny * 1.5)
        big[0] = 1.0
    big = big / big.sum()
    big = np.maximum(big, tiny)  # keep exactly nz nonzero images after normalising
    small = tiny * rng.random(Np - nz) * 0.999
    w = np.concatenate([np.sort(big)[::-1], np.sort(small)[::-1]])
    assert sum(1 for x in w if x >= tiny) == nz
    return [float(x) for x in w]


@pytest.mark.parametrize("kind", ["geometric", "flat", "edge", "dominant"])
def test_fewer_than_m_nonzero_images_end_in_keep_top(kind):
    rng = np.random.default_rng(7)
    Np, M = 250, 244  # the pipeline's N_max = 250, K = 6
    for trial in range(40):
        nz = int(rng.integers(1, M))  # nz <= M - 1
        w = _weights(rng, Np, nz, kind)
        k, log_c = _k_loop(w, M)
        assert not math.isfinite(log_c), (kind, trial, nz, k, log_c)


def test_small_m_boundary():
    # nz = M - 1 exactly, for small M where log(M-k)/(M-1-k) margins are largest and smallest
    rng = np.random.default_rng(11)
    for M in (2, 3, 5, 17, 64, 200):
        for _ in range(10):
            Np = M + 6
            w = _weights(rng, Np, M - 1, "geometric")
            _, log_c = _k_loop(w, M)
            assert not math.isfinite(log_c)


def test_certificate_is_not_vacuous():
    # with nz >= M the loop does reach a finite log c (the optimal branch) on spread weights
    rng = np.random.default_rng(3)
    finite = 0
    for _ in range(20):
        w = _weights(rng, 250, 250, "geometric")
        _, log_c = _k_loop(w, 244)
        finite += math.isfinite(log_c)
    assert finite > 0
