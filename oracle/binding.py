"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product package (hygeia_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# HYG_ORACLE_DIR=build_san: the sanitizer build (make SAN=1, tools/sanitize.sh)
LIB_PATH = os.path.join(HERE, os.environ.get("HYG_ORACLE_DIR", "build"), "libtg_oracle.so")
KMAX = 16

# pipeline defaults (run_inference_two_groups.py:19-36, nextflow.config)
DEFAULT_MU = (0.95, 0.05, 0.80, 0.20, 0.50, 0.50)
DEFAULT_SIGMA = (0.05, 0.05, 0.1, 0.1, 0.1, 0.2886751)


class TgParams(C.Structure):
    """Mirror of hyg_tg_params (include/hygeia_amd.h)."""

    _fields_ = [
        ("n_regimes", C.c_int32),
        ("minimum_duration", C.c_int32),
        ("num_resampled_ancestors", C.c_int32),
        ("num_samples_backward", C.c_int32),
        ("optimal_resampling", C.c_int32),
        ("multinomial", C.c_int32),
        ("theta_len", C.c_int32),
        ("_pad", C.c_int32),
        ("mu", C.c_double * KMAX),
        ("sigma", C.c_double * KMAX),
        ("theta", C.c_double * (KMAX * KMAX)),
        ("omega_case", C.c_double),
        ("merge_log_prob", C.c_double),
        ("split_prob", C.c_double),
        ("kappa_control", C.c_double),
        ("kappa_case", C.c_double),
    ]


class TgConsts(C.Structure):
    """Mirror of hyg_tg_consts (include/hyg_model.h)."""

    _fields_ = [
        ("K", C.c_int32), ("u", C.c_int32), ("M", C.c_int32), ("B", C.c_int32),
        ("I", C.c_int32), ("Nmax", C.c_int32), ("optimal", C.c_int32), ("multinomial", C.c_int32),
        ("alpha", C.c_double * KMAX), ("beta", C.c_double * KMAX),
        ("p_ctrl", C.c_double * KMAX), ("p_case", C.c_double * KMAX),
        ("kappa_ctrl", C.c_double), ("kappa_case", C.c_double),
        ("lPc", C.c_double * (KMAX * KMAX)), ("lPm", C.c_double * 4),
        ("lU1", C.c_double), ("lU2", C.c_double), ("log_M", C.c_double),
        ("sig_thresh", C.c_float), ("_pad", C.c_int32),
    ]


def theta_from(p_matrix: np.ndarray, omega_ctrl: np.ndarray) -> np.ndarray:
    """theta_{chrom}.csv.gz layout (run_inference_two_groups.py:76-89): off-diagonal
    log-weights row by row, then logit(omega)."""
    K = p_matrix.shape[0]
    vals = [math.log(p_matrix[r, r1]) for r in range(K) for r1 in range(K) if r != r1]
    vals += [math.log(w / (1.0 - w)) for w in omega_ctrl]
    return np.asarray(vals, dtype=np.float64)


def make_params(K: int = 6, mu=None, sigma=None, theta=None, u: int = 3, M: int = 50, B: int = 25,
                omega_case: float = 0.8, omega_ctrl: float = 0.8, merge_log_prob: float = math.log(0.1),
                split_prob: float = 0.01, optimal: int = 1, multinomial: int = 0) -> TgParams:
    p = TgParams()
    if mu is None:
        mu = list(DEFAULT_MU) if K == 6 else [((i + 0.5) / K) for i in range(K)]
    if sigma is None:
        sigma = list(DEFAULT_SIGMA) if K == 6 else [0.05 + 0.2 * min(m, 1 - m) for m in mu]
    if theta is None:
        P = np.full((K, K), 1.0 / (K - 1))
        np.fill_diagonal(P, 0.0)
        theta = theta_from(P, np.full(K, omega_ctrl))
    p.n_regimes = K
    p.minimum_duration = u
    p.num_resampled_ancestors = M
    p.num_samples_backward = B
    p.optimal_resampling = optimal
    p.multinomial = multinomial
    p.theta_len = len(theta)
    for i in range(K):
        p.mu[i] = float(mu[i])
        p.sigma[i] = float(sigma[i])
    for i, v in enumerate(theta):
        p.theta[i] = float(v)
    p.omega_case = omega_case
    p.merge_log_prob = merge_log_prob
    p.split_prob = split_prob
    p.kappa_control = 2.0
    p.kappa_case = 2.0
    return p


_lib = None


def build() -> str:
    subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB_PATH


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        d, i32, u64, vp = C.c_double, C.c_int32, C.c_uint64, C.c_void_p
        L.oracle_exp.restype = d
        L.oracle_exp.argtypes = [d]
        L.oracle_log.restype = d
        L.oracle_log.argtypes = [d]
        L.oracle_expf.restype = C.c_float
        L.oracle_expf.argtypes = [C.c_float]
        L.oracle_fix100.restype = None
        L.oracle_fix100.argtypes = [d, C.POINTER(C.c_uint64)]
        L.oracle_philox.restype = None
        L.oracle_philox.argtypes = [u64] * 6 + [vp]
        L.oracle_u192_roundtrip.restype = d
        L.oracle_u192_roundtrip.argtypes = [C.c_float]
        L.oracle_u128_roundtrip.restype = d
        L.oracle_u128_roundtrip.argtypes = [d]
        L.oracle_tg_emission.restype = i32
        L.oracle_tg_emission.argtypes = [C.POINTER(TgParams), vp, vp, i32, vp, vp, i32, C.c_int64, vp]
        L.oracle_tg_chain.restype = i32
        L.oracle_tg_chain.argtypes = [C.POINTER(TgParams), vp, i32, u64, u64, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.oracle_tg_chain_refstruct.restype = i32
        L.oracle_tg_chain_refstruct.argtypes = [C.POINTER(TgParams), vp, vp, i32, vp, vp, i32, i32, u64, u64, vp, vp,
                                                vp, vp, vp, vp]
        L.oracle_tg_trans.restype = d
        L.oracle_tg_trans.argtypes = [C.POINTER(TgParams), i32, u64, u64]
        L.oracle_tg_xi.restype = u64
        L.oracle_tg_xi.argtypes = [i32, u64, i32]
        L.oracle_tg_hazard.restype = i32
        L.oracle_tg_hazard.argtypes = [C.POINTER(TgParams), i32, i32, i32, vp]
        L.oracle_tg_consts.restype = i32
        L.oracle_tg_consts.argtypes = [C.POINTER(TgParams), C.POINTER(TgConsts)]
        L.oracle_sizeof_params.restype = i32
        L.oracle_sizeof_consts.restype = i32
        assert L.oracle_sizeof_params() == C.sizeof(TgParams)
        assert L.oracle_sizeof_consts() == C.sizeof(TgConsts)
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def consts(p: TgParams) -> TgConsts:
    c = TgConsts()
    rc = lib().oracle_tg_consts(C.byref(p), C.byref(c))
    if rc != 0:
        raise ValueError(f"invalid parameters (code {rc})")
    return c


def emission(p: TgParams, meth_c, tot_c, meth_k, tot_k) -> np.ndarray:
    meth_c = np.ascontiguousarray(meth_c, dtype=np.uint16)
    tot_c = np.ascontiguousarray(tot_c, dtype=np.uint16)
    meth_k = np.ascontiguousarray(meth_k, dtype=np.uint16)
    tot_k = np.ascontiguousarray(tot_k, dtype=np.uint16)
    T = tot_c.shape[0]
    K = p.n_regimes
    E = np.empty((T, 2 * K), dtype=np.float64)
    rc = lib().oracle_tg_emission(C.byref(p), _ptr(meth_c), _ptr(tot_c), tot_c.shape[1], _ptr(meth_k),
                                  _ptr(tot_k), tot_k.shape[1], T, _ptr(E))
    if rc != 0:
        raise ValueError(f"oracle_tg_emission failed ({rc})")
    return E


def chain(p: TgParams, E: np.ndarray, seed: int, chain_id: int, want_modes: bool = False) -> dict:
    """One chain (filter + backward simulation) on the emission table E [T][2K]."""
    E = np.ascontiguousarray(E, dtype=np.float64)
    T = E.shape[0]
    K, B = p.n_regimes, p.num_samples_backward
    c = consts(p)
    out = {
        "merged": np.empty((T, B), np.int16),
        "control": np.empty((T, B, 2), np.int16),
        "case": np.empty((T, B, 2), np.int16),
        "split_probs": np.empty(T, np.float32),
        "regime_probs": np.empty((T, 2 * K), np.float32),
        "final_log_weights": np.empty(c.Nmax, np.float64),
        "final_states": np.empty(c.Nmax, np.uint64),
    }
    modes = np.zeros(T, np.int32)
    logz = C.c_double(0.0)
    rc = lib().oracle_tg_chain(C.byref(p), _ptr(E), T, seed, chain_id, _ptr(out["merged"]), _ptr(out["control"]),
                               _ptr(out["case"]), _ptr(out["split_probs"]), _ptr(out["regime_probs"]),
                               C.byref(logz), _ptr(out["final_log_weights"]), _ptr(out["final_states"]),
                               _ptr(modes) if want_modes else None)
    out["status"] = rc
    out["log_z"] = logz.value
    if want_modes:
        out["modes"] = modes
    return out


def chain_refstruct(p: TgParams, meth_c, tot_c, meth_k, tot_k, seed: int, chain_id: int) -> dict:
    """The reference-structure CPU variant (oracle_tg_chain_refstruct): per-particle
    Beta-Binomial from the counts, full sort, full-N history, [B, N] backward
    rows. Same outputs as chain() on the same counts."""
    mc, tc, mk, tk = (np.ascontiguousarray(a, dtype=np.uint16) for a in (meth_c, tot_c, meth_k, tot_k))
    T = tc.shape[0]
    K, B = p.n_regimes, p.num_samples_backward
    out = {
        "merged": np.empty((T, B), np.int16),
        "control": np.empty((T, B, 2), np.int16),
        "case": np.empty((T, B, 2), np.int16),
        "split_probs": np.empty(T, np.float32),
        "regime_probs": np.empty((T, 2 * K), np.float32),
    }
    logz = C.c_double(0.0)
    out["status"] = lib().oracle_tg_chain_refstruct(
        C.byref(p), _ptr(mc), _ptr(tc), tc.shape[1], _ptr(mk), _ptr(tk), tk.shape[1], T, seed, chain_id,
        _ptr(out["merged"]), _ptr(out["control"]), _ptr(out["case"]), _ptr(out["split_probs"]),
        _ptr(out["regime_probs"]), C.byref(logz))
    out["log_z"] = logz.value
    return out


def hazard(p: TgParams, g: int, r: int, n: int) -> np.ndarray:
    out = np.empty((n, 2), np.float64)
    rc = lib().oracle_tg_hazard(C.byref(p), g, r, n, _ptr(out))
    if rc != 0:
        raise ValueError(rc)
    return out


def trans(p: TgParams, prev: int, nxt: int, max_duration: int = 1000) -> float:
    return lib().oracle_tg_trans(C.byref(p), max_duration, prev, nxt)


def pack(m, dc, rc, dk, rk) -> int:
    return (dc & 0xFFFFFF) | ((dk & 0xFFFFFF) << 24) | (rc << 48) | (rk << 54) | (m << 60)


def unpack(s: int):
    return ((s >> 60) & 1, s & 0xFFFFFF, (s >> 48) & 63, (s >> 24) & 0xFFFFFF, (s >> 54) & 63)
