"""The systematic-target count of the top-set finish (hygeia_amd/csrc/tg_kernels.hip:
sys_count), restated in Python and checked against a brute-force count.

top_set_finish1 assigns the systematic residual targets (resampling_functions.py:
56-69) per sorted position: position p takes the targets j in
[count(C(p-1)), count(C(p))), count(v) = #{j < L : ceil(T_j R) <= v}, with
T_j = f32((f32(j) + U) / f32(L)) and R the exact residual mass image. The kernel
estimates the threshold j ~ (v / R) L - U in f64 (relative error below 2^-49),
counts every j below floor(estimate) and compares only the two candidates at and
above it: in f64 outside a 2^-46 guard band, exactly in integers inside it. This
test pins that argument: the restatement (with y perturbed by up to 2^-49, the
kernel's error bound) must equal the brute-force count everywhere, including v
exactly at, one below and one above every target, v = 0 and v = R.
"""
import random

import numpy as np

from oracle.tg_oracle_np import ceil_mul_f32, u01f

GUARD = 2.0 ** -46


def targets(L, U):
    return [np.float32((np.float32(j) + U) / np.float32(L)) for j in range(L)]


def count_brute(v, R, T):
    return sum(1 for t in T if ceil_mul_f32(t, R) <= v)


def count_kernel(v, R, L, U, T, rel_err=0.0):
    """sys_count's arithmetic: y = v / R as f64 (perturbed by rel_err), the
    estimate, two candidates, guard band, exact compare inside it."""
    y = (float(v) / float(R)) * (1.0 + rel_err)
    jf = y * float(L) - float(U)
    jf = -1.0 if jf < -1.0 else (float(L) if jf > float(L) else jf)
    j0 = int(np.floor(jf))
    ylo, yhi = y * (1.0 - GUARD), y * (1.0 + GUARD)
    c = j0 if j0 > 0 else 0
    for k in range(2):
        j = j0 + k
        if not (0 <= j < L):
            continue
        t = float(T[j])
        le = t < ylo
        if not le and not (t > yhi):
            le = v >= ceil_mul_f32(T[j], R)
        c += 1 if le else 0
    return c


def cases(rng, n):
    for _ in range(n):
        L = rng.randint(1, 64)
        U = u01f(rng.getrandbits(64))
        R = rng.randint(1, 2 ** rng.randint(20, 151))
        T = targets(L, U)
        vs = [0, R, rng.randint(0, R), rng.randint(0, R)]
        for j in rng.sample(range(L), min(L, 3)):
            tau = ceil_mul_f32(T[j], R)
            vs += [tau, max(tau - 1, 0), min(tau + 1, R)]
        yield L, U, R, T, vs


def test_sys_count_matches_brute_force():
    rng = random.Random(20261017)
    n = 0
    for L, U, R, T, vs in cases(rng, 1500):
        for v in vs:
            want = count_brute(v, R, T)
            for err in (0.0, 2.0 ** -49, -(2.0 ** -49)):
                assert count_kernel(v, R, L, U, T, err) == want, (L, float(U), R, v, err)
                n += 1
    assert n > 40000


def test_sys_count_u_zero_and_one_target():
    # U = 0: T_0 = 0, so target 0 sits at C(K - 1) exactly (v = 0 counts it)
    for L in (1, 2, 17, 64):
        T = targets(L, np.float32(0.0))
        for R in (1, 3, 2 ** 149 + 12345):
            assert count_kernel(0, R, L, np.float32(0.0), T) == count_brute(0, R, T) == 1
            assert count_kernel(R, R, L, np.float32(0.0), T) == count_brute(R, R, T) == L
