"""Independent pure-Python restatement of the two-group chain (TEST INFRASTRUCTURE).

A second, language-independent implementation of the same reference algorithm
as oracle/tg_oracle.c, used only by tests to cross-check the C oracle bit for
bit on small chains (T ~ 100, M ~ 10). It re-implements the arithmetic
contract of include/hyg_arith.h itself (Python floats are IEEE doubles; the
contract's explicit fused multiply-adds are computed exactly with Python
integers and rounded once (det_fma / det_fmaf); numpy float32 scalars give IEEE
single ops; Python ints make the exact mass sums trivially exact) and reads only the model TABLES from the C side
(constants and hazard), which tests/test_model_tables.py pins against scipy.

Reference (src/two_group/hygeia): filter_and_smoother_algorithm.py:141-288
(forward steps), 368-447 (backward simulation); resampling_functions.py:7-69;
case_control_regime_model.py:80-231; case_control_distributions.py:138-291;
case_control_proposal_mappings.py:11-216; run_inference_two_groups.py:233-296.
"""
from __future__ import annotations

import math

import numpy as np

NINF = float("-inf")
STEP_HOOK = None
M64 = (1 << 64) - 1

# ------------------------------------------------------------ arithmetic
_LN2_HI = 6.93147180369123816490e-01
_LN2_LO = 1.90821492927058770002e-10
_INV_LN2 = 1.44269504088896338700e+00
_EXP_C = [1.6059043836821614599e-10, 2.0876756987868098979e-09, 2.5052108385441718775e-08,
          2.7557319223985890653e-07, 2.7557319223985890653e-06, 2.4801587301587301566e-05,
          1.9841269841269841253e-04, 1.3888888888888888889e-03, 8.3333333333333332177e-03,
          4.1666666666666664354e-02, 1.6666666666666665741e-01, 0.5, 1.0, 1.0]
_LOG_C = [0.08695652173913043478, 0.09523809523809523810, 0.10526315789473684211,
          0.11764705882352941176, 0.13333333333333333333, 0.15384615384615384615,
          0.18181818181818181818, 0.22222222222222222222, 0.28571428571428571429,
          0.40000000000000000000, 0.66666666666666666667]


def _pow2(e: int) -> float:
    return math.ldexp(1.0, e)


def _exact(x: float):
    """finite double x = m 2^e with integer m"""
    m, e = math.frexp(x)
    return int(m * (1 << 53)), e - 53


def _exact_sum(a, b, c):
    """a * b + c exactly, as an integer mantissa and exponent (finite inputs)"""
    ma, ea = _exact(float(a))
    mb, eb = _exact(float(b))
    mc, ec = _exact(float(c))
    mp, ep = ma * mb, ea + eb
    e0 = min(ep, ec)
    return (mp << (ep - e0)) + (mc << (ec - e0)), e0


def det_fma(a: float, b: float, c: float) -> float:
    """IEEE fma (one rounding) of finite doubles: the exact a b + c as a Python
    integer, rounded once (int -> float conversion is correctly rounded; the
    exponent scaling is exact for the normal results the contract uses)."""
    m, e = _exact_sum(a, b, c)
    if m == 0:
        return a * b + c
    return math.ldexp(float(m), e)


def det_fmaf(a, b, c) -> np.float32:
    """IEEE fmaf (one rounding to binary32, ties to even) of float32 values."""
    m, e = _exact_sum(a, b, c)
    if m == 0:
        return np.float32(np.float32(a) * np.float32(b) + np.float32(c))
    neg = m < 0
    m = -m if neg else m
    shift = m.bit_length() - 24
    if e + shift < -149:  # subnormal result: the lsb is 2^-149
        shift = -149 - e
    if shift > 0:
        q, r = divmod(m, 1 << shift)
        half = 1 << (shift - 1)
        if r > half or (r == half and (q & 1)):
            q += 1
        m, e = q, e + shift
    v = np.float32(math.ldexp(float(m), e))  # exact: <= 24 significant bits
    return -v if neg else v


def det_exp(x: float) -> float:
    """hyg_exp: Taylor degree 13 by Estrin's scheme (same operations, same order)."""
    if x != x:
        return x
    if x > 709.782712893383973096:
        return math.inf
    if x < -745.13321910194110842:
        return 0.0
    kd = math.floor(x * _INV_LN2 + 0.5)
    k = int(kd)
    hi = x - kd * _LN2_HI  # exact
    r = det_fma(-kd, _LN2_LO, hi)
    r2 = r * r
    r4 = r2 * r2
    r8 = r4 * r4
    c = [1.0, 1.0, 0.5, 1.6666666666666665741e-01, 4.1666666666666664354e-02, 8.3333333333333332177e-03,
         1.3888888888888888889e-03, 1.9841269841269841253e-04, 2.4801587301587301566e-05,
         2.7557319223985890653e-06, 2.7557319223985890653e-07, 2.5052108385441718775e-08,
         2.0876756987868098979e-09, 1.6059043836821614599e-10]
    q = [det_fma(c[2 * i + 1], r, c[2 * i]) for i in range(7)]
    s0 = det_fma(q[1], r2, q[0])
    s1 = det_fma(q[3], r2, q[2])
    s2 = det_fma(q[5], r2, q[4])
    u0 = det_fma(s1, r4, s0)
    u1 = det_fma(q[6], r4, s2)
    p = det_fma(u1, r8, u0)
    if k > 1023:
        return (p * 2.0) * _pow2(k - 1)
    if k >= -1021:
        return p * _pow2(k)
    return (p * _pow2(k + 54)) * _pow2(-54)


def det_log(x: float) -> float:
    """hyg_log: atanh series by Estrin's scheme (same operations, same order)."""
    if x != x or x < 0.0:
        return math.nan
    if x == 0.0:
        return NINF
    if x == math.inf:
        return x
    m, e = math.frexp(x)  # x = m 2^e, m in [0.5, 1)
    m *= 2.0
    e -= 1
    if m > 1.41421356237309504880:
        m *= 0.5
        e += 1
    f = m - 1.0
    s = f / (2.0 + f)
    z = s * s
    z2 = z * z
    z4 = z2 * z2
    z8 = z4 * z4
    a = [0.66666666666666666667, 0.40000000000000000000, 0.28571428571428571429, 0.22222222222222222222,
         0.18181818181818181818, 0.15384615384615384615, 0.13333333333333333333, 0.11764705882352941176,
         0.10526315789473684211, 0.09523809523809523810]
    a01 = det_fma(a[1], z, a[0])
    a23 = det_fma(a[3], z, a[2])
    a45 = det_fma(a[5], z, a[4])
    a67 = det_fma(a[7], z, a[6])
    a89 = det_fma(a[9], z, a[8])
    a10 = 0.08695652173913043478
    b0 = det_fma(a23, z2, a01)
    b1 = det_fma(a67, z2, a45)
    b2 = det_fma(a10, z2, a89)
    c0 = det_fma(b1, z4, b0)
    R = z * det_fma(b2, z8, c0)
    hfsq = 0.5 * f * f
    l1p = f - det_fma(-s, hfsq + R, hfsq)
    ed = float(e)
    return det_fma(ed, _LN2_HI, det_fma(ed, _LN2_LO, l1p))


def f32(x) -> np.float32:
    return np.float32(x)


_F = lambda h: np.float32(float.fromhex(h))  # noqa: E731
_EXPF_C = {k: _F(v) for k, v in dict(log2e="0x1.715476p+0", hi="0x1.62e4p-1", lo="0x1.7f7d1cp-20",
                                      c3="0x1.555556p-3", c4="0x1.555556p-5", c5="0x1.111112p-7",
                                      c6="0x1.6c16c2p-10", c7="0x1.a01a02p-13").items()}


def det_expf(x: np.float32) -> np.float32:
    """hyg_expf: exp in float32 basic operations (Cody-Waite + degree-7 Taylor,
    Estrin), the same operations in the same order as include/hyg_arith.h."""
    x = np.float32(x)
    if x != x:
        return x
    if x < np.float32(-104.0):
        return np.float32(0.0)
    if x > np.float32(89.0):
        return np.float32(np.inf)
    c = _EXPF_C
    one, half = np.float32(1.0), np.float32(0.5)
    kf = np.float32(math.floor(float(x * c["log2e"] + half)))
    r = det_fmaf(-kf, c["lo"], x - kf * c["hi"])
    r2 = r * r
    r4 = r2 * r2
    q0 = one + r
    q1 = det_fmaf(c["c3"], r, half)
    q2 = det_fmaf(c["c5"], r, c["c4"])
    q3 = det_fmaf(c["c7"], r, c["c6"])
    p = det_fmaf(det_fmaf(q3, r2, q2), r4, det_fmaf(q1, r2, q0))
    k = int(kf)
    if k > 127:
        return p * np.float32(2.0) * np.float32(2.0 ** (k - 1))
    if k < -126:
        return (p * np.float32(2.0 ** (k + 64))) * np.float32(2.0 ** -64)
    return p * np.float32(2.0 ** k)


def det_logf(x: np.float32) -> np.float32:
    return np.float32(det_log(float(x)))


def fix100(e: float) -> int:
    """floor(e * 2^100) exactly (0 for e <= 0, NaN and e >= 2^16, as hyg_fix100)."""
    if not 0.0 < e < 65536.0:
        return 0
    m, ex = math.frexp(e)  # e = m 2^ex, m in [0.5,1): mant = m*2^53
    mant = int(m * (1 << 53))
    sh = ex - 53 + 100
    return mant << sh if sh >= 0 else mant >> (-sh)


def fix149f(m: np.float32) -> int:
    """exact m * 2^149 for an f32 m in [0, 1]."""
    v = float(m)
    if v <= 0.0:
        return 0
    fr, ex = math.frexp(v)
    mant = int(fr * (1 << 24))
    sh = ex - 24 + 149
    if sh >= 0:
        return mant << sh
    assert mant & ((1 << -sh) - 1) == 0  # f32 subnormals are multiples of 2^-149
    return mant >> (-sh)


def ceil_mul_f32(T: np.float32, R: int) -> int:
    """ceil(T * R) exactly, for an f32 T (the systematic comparison threshold)."""
    b = int(np.array(T, dtype=np.float32).view(np.uint32))
    if b == 0 or (b >> 31):
        return 0
    E = (b >> 23) & 0xFF
    m = (b & 0x7FFFFF) if E == 0 else ((b & 0x7FFFFF) | 0x800000)
    s = 149 if E == 0 else 150 - E
    return (m * R + (1 << s) - 1) >> s


def int_to_f64(V: int, scale: int) -> float:
    """top 53 bits (truncated) of V, times 2^-scale."""
    if V == 0:
        return 0.0
    p = V.bit_length() - 1
    if p <= 52:
        return float(V) * _pow2(-scale)
    sh = p - 52
    return float(V >> sh) * _pow2(sh - scale)


def philox4x64(c, k):
    c = list(c)
    k0, k1 = k
    for _ in range(10):
        p0 = 0xD2E7470EE14C6C93 * c[0]
        p1 = 0xCA5A826395121157 * c[2]
        hi0, lo0 = (p0 >> 64) & M64, p0 & M64
        hi1, lo1 = (p1 >> 64) & M64, p1 & M64
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
        k0 = (k0 + 0x9E3779B97F4A7C15) & M64
        k1 = (k1 + 0xBB67AE8584CAA73B) & M64
    return c


RNG_PHANTOM, RNG_SYSTEMATIC, RNG_MULTINOMIAL, RNG_BACKWARD = 1, 2, 3, 4


def rand64(seed, chain, stream, step, index):
    return philox4x64((stream, step, index >> 2, 0), (seed, chain))[index & 3]


def u01f(r: int) -> np.float32:
    return np.float32((r >> 40) * 5.9604644775390625e-08)


def categorical(logits, r: int) -> int:
    lmax = max(logits)
    if lmax == NINF:
        return -1
    masses = [fix100(det_exp(l - lmax)) for l in logits]
    total = sum(masses)
    target = (r * total) >> 64
    cdf = 0
    for n, q in enumerate(masses):
        cdf += q
        if target < cdf:
            return n
    return len(logits) - 1


# ---------------------------------------------------------------- model
class Model:
    def __init__(self, consts, hazard_rows, dcap):
        """consts: binding.TgConsts; hazard_rows[(g, r)] = array [dcap, 2]"""
        c = consts
        self.K, self.u, self.M, self.B, self.I = c.K, c.u, c.M, c.B, c.I
        self.lPc = [c.lPc[i] for i in range(c.K * c.K)]
        self.lPm = [c.lPm[i] for i in range(4)]
        self.lU1, self.lU2, self.log_M = c.lU1, c.lU2, c.log_M
        self.hz = hazard_rows
        self.dcap = dcap

    def haz(self, g, r, d):
        d = min(max(d, 0), self.dcap - 1)
        row = self.hz[(g, r)]
        return float(row[d, 0]), float(row[d, 1])

    def trans(self, prev, nxt):
        m, dc, rc, dk, rk = prev
        m2, dc2, rc2, dk2, rk2 = nxt
        K = self.K
        if min(dk, dc) >= self.u:
            lm = self.lPm[m * 2 + m2]
        else:
            lm = 0.0 if m2 == m else NINF
        lr, l1 = self.haz(0, rc, dc)
        if dc2 == 1:
            lc = lr + self.lPc[rc * K + rc2]
        else:
            lc = l1 if (dc2 == dc + 1 and rc2 == rc) else NINF
        if m2 == 1:
            lk = 0.0 if (rk2 == rc2 and dk2 == dc2) else NINF
        elif m == 1 and dc2 != 1:
            lk = self.lU1 if (dk2 == 1 and rk2 != rc2) else NINF
        elif rc2 == rk and m == 0:
            lk = self.lU1 if (dk2 == 1 and rk2 != rc2) else NINF
        else:
            kr, k1 = self.haz(1, rk, dk)
            if dk2 == 1:
                lk = kr + (self.lU1 if rc2 == rk else self.lU2) if (rk2 != rc2 and rk2 != rk) else NINF
            else:
                lk = k1 if (dk2 == dk + 1 and rk2 == rk) else NINF
        return (lm + lc) + lk

    def xi(self, a, s):
        m, dc, rc, dk, rk = a
        K = self.K
        if s == 0:
            return (m, dc + 1, rc, dk + 1, rk)
        if s < K:
            r = s - 1 if s - 1 < rk else s
            return (0, 1, r, dk + 1, rk)
        if s < 2 * K - 1:
            q = s - K
            r = q if q < rc else q + 1
            return (0, dc + 1, rc, 1, r)
        if s == 2 * K - 1:
            d = dc + 1 if m == 0 else 0
            return (1, d, rc, d, rc)
        j = s - 2 * K
        i, jj = divmod(j, K)
        return (int(i == jj), 1, i, 1, jj)


def _sort_key(x: np.float32, idx: int) -> int:
    u = int(np.array(x, dtype=np.float32).view(np.uint32))
    if u == 0x80000000:
        u = 0
    ord_ = (~u & 0xFFFFFFFF) if (u >> 31) else (u | 0x80000000)
    return ((~ord_ & 0xFFFFFFFF) << 32) | idx


def run_chain(model: Model, E: np.ndarray, seed: int, chain: int):
    K, M, B, I = model.K, model.M, model.B, model.I
    T = E.shape[0]
    recs = []

    def particles(t):
        rec = recs[t]
        Et = [float(v) for v in E[t]]
        st, W = [], []
        if rec["mode"] == "init":
            rph = rec["r_ph"]
            for i in range(K):
                for j in range(K):
                    st.append((int(i == j), 1, i, 1, j))
                    tr = model.lPc[rph * K + i] if i == j else NINF
                    W.append((Et[i] + Et[K + j]) + tr)
            return st, W
        ps, pw = rec["ps"], rec["pw"]
        np_ = len(ps)
        for s in range(I):
            for a in range(np_):
                x = model.xi(ps[a], s)
                st.append(x)
                tr = model.trans(ps[a], x)
                if not math.isfinite(tr):
                    W.append(NINF)
                    continue
                lg = tr + (Et[x[2]] + Et[K + x[4]])
                if rec["mode"] == "keep":
                    w = pw[a] + lg
                elif rec["mode"] == "unbiased":
                    w = (-model.log_M + rec["lse"]) + lg
                else:
                    v = float(rec["log_c"]) + (pw[a] - rec["lse"])
                    w = (pw[a] + lg) - (v if v < 0.0 else 0.0)
                W.append(w)
        return st, W

    def lse_exact(W):
        mx = max(W)
        if mx == NINF:
            return mx, NINF
        S = sum(fix100(det_exp(w - mx)) for w in W)
        return mx, det_log(int_to_f64(S, 100))

    rph = (rand64(seed, chain, RNG_PHANTOM, 0, 0) * K) >> 64
    recs.append({"mode": "init", "r_ph": rph})
    st, W = particles(0)
    for t in range(1, T):
        mx, logS = lse_exact(W)
        if mx == NINF:
            raise FloatingPointError("all weights -inf")
        lse = logS + mx
        N = len(W)
        nz = [n for n in range(N) if W[n] > NINF]
        rec = {"lse": lse, "log_c": np.float32(0.0)}
        if len(nz) <= M:
            parents = nz
            rec["mode"] = "keep"
        else:
            lw32 = [np.float32((w - mx) - logS) for w in W]
            if STEP_HOOK is not None:  # diagnostics (tools/), not part of the algorithm
                STEP_HOOK(t, lw32)
            keys = sorted(_sort_key(lw32[n], n) for n in range(N))
            order = [k & 0xFFFFFFFF for k in keys]
            mass = [det_expf(lw32[n]) for n in order]
            ints = [fix149f(m) for m in mass]
            revcum = [0] * (N + 1)
            for p in range(N - 1, -1, -1):
                revcum[p] = revcum[p + 1] + ints[p]
            a, b, lc = 0, -1, np.float32(-1.0)
            while a != b and a < N and a < M:
                l1 = det_logf(np.float32(M - a))
                rv = int_to_f64(revcum[a], 149)
                l2 = np.float32(NINF) if rv == 0.0 else np.float32(det_log(rv))
                with np.errstate(invalid="ignore"):
                    cnew = np.float32(l1 - l2)
                    cnt = sum(1 for p in range(a, N) if np.float32(cnew + lw32[order[p]]) > np.float32(0.0))
                b, a, lc = a, a + cnt, cnew
            Kk, log_c = b, lc
            if Kk >= N:
                Kk, log_c = N, np.float32(NINF)
            if not np.isfinite(log_c):
                l = [float(x) for x in lw32]
                parents = [categorical(l, rand64(seed, chain, RNG_MULTINOMIAL, t, j)) for j in range(M)]
                rec["mode"] = "unbiased"
            else:
                L = M - Kk
                parents = order[:Kk]
                R = revcum[Kk]
                U = u01f(rand64(seed, chain, RNG_SYSTEMATIC, t, 0))
                sys_ = [0] * L
                i, j, C = 0, 0, ints[Kk]
                ln = N - Kk
                while j < L and i < ln:
                    Tj = np.float32((np.float32(j) + U) / np.float32(L))
                    if C >= ceil_mul_f32(Tj, R):
                        sys_[j] = i
                        j += 1
                    else:
                        i += 1
                        if i < ln:
                            C += ints[Kk + i]
                parents = parents + [order[Kk + s] for s in sys_]
                rec["mode"] = "optimal"
                rec["log_c"] = log_c
        rec["ps"] = [st[q] for q in parents]
        rec["pw"] = [W[q] for q in parents]
        recs.append(rec)
        st, W = particles(t)
    mx, logS = lse_exact(W)
    log_z = logS + mx
    final_w = list(W)
    merged = np.zeros((T, B), np.int16)
    control = np.zeros((T, B, 2), np.int16)
    case = np.zeros((T, B, 2), np.int16)
    X = [None] * B
    for t in range(T - 1, -1, -1):
        st, W = particles(t)
        idx = []
        for b in range(B):
            r = rand64(seed, chain, RNG_BACKWARD, t, b)
            if t == T - 1:
                q = categorical(W, r)
            else:
                logits = []
                for n in range(len(W)):
                    f = model.trans(st[n], X[b]) if math.isfinite(W[n]) else NINF
                    logits.append(f + W[n] if (math.isfinite(f) and math.isfinite(W[n])) else NINF)
                q = categorical(logits, r)
            if q < 0:
                raise FloatingPointError("backward kernel all -inf")
            idx.append(q)
        for b in range(B):
            x = st[idx[b]]
            X[b] = x
            merged[t, b] = x[0]
            control[t, b] = (x[1], x[2])
            case[t, b] = (x[3], x[4])
    split = (merged == 0).sum(1).astype(np.float32) / np.float32(B)
    reg = np.concatenate([np.stack([(control[:, :, 1] == r).sum(1) for r in range(K)], 1),
                          np.stack([(case[:, :, 1] == r).sum(1) for r in range(K)], 1)], 1)
    regime = reg.astype(np.float32) / np.float32(B)
    return {"merged": merged, "control": control, "case": case, "split_probs": split,
            "regime_probs": regime, "log_z": log_z, "final_log_weights": final_w}
