"""The deterministic arithmetic contract (include/hyg_arith.h), CPU only.

hyg_exp / hyg_log are what every weight in the filter goes through; the GPU
kernels compile the same header, so pinning them here pins both sides. The
exact fixed-point mass sums and the Philox stream are checked against
independent implementations (Python ints, numpy's Philox).
"""
import ctypes as C
import math

import numpy as np
import pytest

from oracle import tg_oracle_np as onp


def _ulps(a: float, b: float) -> int:
    ia = np.array(a, np.float64).view(np.int64)
    ib = np.array(b, np.float64).view(np.int64)
    return abs(int(ia) - int(ib))


def test_exp_accuracy_and_python_restatement(oracle):
    L = oracle.lib()
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.uniform(-745, 709, 4000), rng.uniform(-1, 1, 2000), rng.uniform(-60, 0, 2000),
                         [0.0, -0.0, 1.0, -1.0, 709.78, -708.4, -740.0, -745.2, 710.0]])
    worst = 0
    for x in xs:
        v = L.oracle_exp(float(x))
        assert v == onp.det_exp(float(x)) or (math.isnan(v) and math.isnan(onp.det_exp(float(x))))
        ref = math.exp(x) if x < 709.78 else math.inf
        if ref > 2.2250738585072014e-308 and math.isfinite(ref):
            worst = max(worst, _ulps(v, ref))
    assert worst <= 2, worst
    assert L.oracle_exp(float("-inf")) == 0.0
    assert L.oracle_exp(1000.0) == math.inf
    assert math.isnan(L.oracle_exp(float("nan")))


def test_expf_accuracy_and_python_restatement(oracle):
    """hyg_expf (float32 arithmetic): within 2 f32 ulp of the correctly rounded
    exp over the log-weight range, exact 0 below the subnormal range, and the
    same bits as the numpy-float32 restatement."""
    L = oracle.lib()
    rng = np.random.default_rng(5)
    xs = np.concatenate([rng.uniform(-104.5, 0, 6000), rng.uniform(-1, 1, 2000), rng.uniform(-88, 88.7, 1000),
                         [0.0, -0.0, 1.0, -1.0, -87.3, -87.34, -100.0, -103.27, -103.3, -103.97, -104.0, -104.1,
                          88.72, 88.73, 89.5]]).astype(np.float32)
    worst = 0
    for x in xs:
        v = np.float32(L.oracle_expf(C.c_float(x)))
        p = onp.det_expf(x)
        assert v.view(np.uint32) == np.float32(p).view(np.uint32), (x, v, p)
        ref = np.float32(math.exp(float(x))) if float(x) < 88.72283935546875 else np.float32(np.inf)
        if np.isfinite(ref):
            # ulps in the f32 grid (subnormals included: the bit patterns are consecutive)
            worst = max(worst, abs(int(v.view(np.int32)) - int(ref.view(np.int32))))
        else:
            assert v == np.inf
    assert worst <= 2, worst
    assert L.oracle_expf(C.c_float(-110.0)) == 0.0
    assert L.oracle_expf(C.c_float(float("-inf"))) == 0.0
    assert math.isnan(L.oracle_expf(C.c_float(float("nan"))))


def test_log_accuracy_and_python_restatement(oracle):
    L = oracle.lib()
    rng = np.random.default_rng(2)
    xs = np.concatenate([np.exp(rng.uniform(-700, 700, 4000)), rng.uniform(0.5, 2.0, 2000),
                         [1.0, 2.0, 0.5, 1e-300, 5e-324, 1.7e308]])
    worst = 0
    for x in xs:
        v = L.oracle_log(float(x))
        assert v == onp.det_log(float(x))
        worst = max(worst, _ulps(v, math.log(x)) if x != 1.0 else 0)
    assert worst <= 2, worst
    assert L.oracle_log(1.0) == 0.0
    assert L.oracle_log(0.0) == -math.inf
    assert math.isnan(L.oracle_log(-1.0))


def test_philox_matches_numpy(oracle):
    """hyg_philox4x64 is Philox4x64-10; numpy increments its counter before
    the first block, so numpy counter c is our counter c + 1."""
    L = oracle.lib()
    out = (C.c_uint64 * 4)()
    for key in ([0, 0], [5, 7], [2**64 - 1, 12345]):
        bg = np.random.Philox(key=np.array(key, dtype=np.uint64), counter=[0, 0, 0, 0])
        raw = bg.random_raw(12)
        for blk in range(3):
            L.oracle_philox(blk + 1, 0, 0, 0, key[0], key[1], out)
            assert list(out) == [int(v) for v in raw[4 * blk:4 * blk + 4]]
            assert onp.philox4x64((blk + 1, 0, 0, 0), tuple(key)) == list(out)


def test_fixed_point_roundtrips(oracle):
    L = oracle.lib()
    rng = np.random.default_rng(3)
    # f32 masses in [0, 1] (normal and subnormal) are exact multiples of 2^-149
    ms = np.concatenate([rng.uniform(0, 1, 2000).astype(np.float32),
                         np.array([0, 1, 1e-45, 1e-40, 1.1754943e-38, 0.5], np.float32)])
    for m in ms:
        assert L.oracle_u192_roundtrip(C.c_float(m)) == float(m)
        assert onp.int_to_f64(onp.fix149f(m), 149) == float(m)
    # f64 masses: floor(e * 2^100), back to f64 with the top 53 bits truncated
    es = np.concatenate([rng.uniform(0, 1, 2000), np.exp(rng.uniform(-69, 0, 1000)), [1.0, 2.0 ** -70]])
    for e in es:
        v = L.oracle_u128_roundtrip(float(e))
        assert v == onp.int_to_f64(onp.fix100(float(e)), 100)
        assert abs(v - e) <= max(e * 2.0 ** -52, 2.0 ** -100)  # truncation of floor(e 2^100)
    assert L.oracle_u128_roundtrip(2.0 ** -101) == 0.0
    # the limbs themselves, exactly (Python ints)
    out = (C.c_uint64 * 2)()
    edge = [0.0, -0.0, -1.0, 1.0, 2.0 ** -100, 2.0 ** -101, 2.0 ** -100 * 1.5, 5e-324, 2.0 ** -52, 0.5,
            1.0 - 2.0 ** -53, 3.75, 65535.99, 65536.0, float("inf"), float("nan")]
    for e in list(es) + list(rng.uniform(0, 2.0 ** -60, 500)) + edge:
        L.oracle_fix100(float(e), out)
        assert (out[1] << 64) | out[0] == onp.fix100(float(e)), e


@pytest.mark.parametrize("T", [0.0, 1.0, 0.5, 1e-45, 3.3e-39, 0.999999940395, 0.123456789])
def test_ceil_mul_is_exact(T):
    """The systematic-resampling threshold ceil(T * R) against rational arithmetic."""
    from fractions import Fraction

    rng = np.random.default_rng(4)
    Tf = np.float32(T)
    for R in [0, 1, 2**149, 2**151 - 1] + [int(x) << int(s) for x, s in
                                           zip(rng.integers(1, 2**62, 20), rng.integers(0, 88, 20))]:
        want = math.ceil(Fraction(float(Tf)) * R)
        assert onp.ceil_mul_f32(Tf, R) == want
