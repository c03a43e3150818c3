"""ctypes binding of the single-group CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# HYG_ORACLE_DIR=build_san: the sanitizer build (make SAN=1, tools/sanitize.sh)
LIB_PATH = os.path.join(HERE, os.environ.get("HYG_ORACLE_DIR", "build"), "libsg_oracle.so")
KMAX = 16

# pipeline defaults: regimes_config / nextflow.config, bin/simulate_data:147-157
DEFAULT_MU = (0.95, 0.05, 0.80, 0.20, 0.50, 0.50)
DEFAULT_SIGMA = (0.05, 0.05, 0.1, 0.1, 0.1, 0.2886751)
DEFAULT_OMEGA = (0.995, 0.975, 0.95, 0.925, 0.9, 0.9)


class SgParams(C.Structure):
    """Mirror of hyg_sg_params (include/hygeia_amd.h)."""

    _fields_ = [
        ("n_regimes", C.c_int32), ("minimum_duration", C.c_int32), ("num_particles_max", C.c_int32),
        ("resample_type", C.c_int32), ("is_kappa_fixed", C.c_int32), ("theta_len", C.c_int32),
        ("alpha", C.c_double * KMAX), ("beta", C.c_double * KMAX), ("kappa", C.c_double * KMAX),
        ("theta", C.c_double * (KMAX * (KMAX + 1))), ("epsilon", C.c_double),
    ]


class SgPeParams(C.Structure):
    """Mirror of hyg_sg_pe_params (include/hygeia_amd.h); defaults are the
    estimate_parameters_and_regimes flags (bin/estimate_parameters_and_regimes:130-200)."""

    _fields_ = [("use_adam", C.c_int32), ("normalise_gradients", C.c_int32),
                ("n_steps_without_update", C.c_int32), ("_pad", C.c_int32),
                ("learning_rate_exponent", C.c_double), ("learning_rate_factor", C.c_double)]


def make_pe(use_adam=True, normalise_gradients=False, every=200, lr_exponent=0.1, lr_factor=0.01):
    pe = SgPeParams()
    pe.use_adam, pe.normalise_gradients, pe.n_steps_without_update = int(use_adam), int(normalise_gradients), every
    pe.learning_rate_exponent, pe.learning_rate_factor = lr_exponent, lr_factor
    return pe


class SgPeRow(C.Structure):
    _fields_ = [("base", C.c_double), ("cont", C.c_double), ("gomg", C.c_double), ("gcont", C.c_double)]


class SgConsts(C.Structure):
    _fields_ = [
        ("K", C.c_int32), ("u", C.c_int32), ("Nmax", C.c_int32), ("is_kappa_fixed", C.c_int32),
        ("alpha", C.c_double * KMAX), ("beta", C.c_double * KMAX), ("kappa", C.c_double * KMAX),
        ("omega", C.c_double * KMAX), ("logP", C.c_double * (KMAX * KMAX)), ("log_K", C.c_double),
        ("epsilon", C.c_double),
    ]


def beta_params(mu, sigma):
    """get_known_parameters (model_functions.R:36-59): method of moments."""
    mu, sigma = np.asarray(mu, float), np.asarray(sigma, float)
    nu = mu * (1 - mu) / sigma ** 2 - 1
    return mu * nu, (1 - mu) * nu


def theta_from(P, omega):
    """convert_model_parameters_to_theta (model_functions.R:62-76) with the rows
    of P as the C++ reads them (singleGroup.h:204-212)."""
    K = len(omega)
    vals = [math.log(P[r][r1]) for r in range(K) for r1 in range(K) if r != r1]
    vals += [math.log(w / (1 - w)) for w in omega]
    return np.asarray(vals)


def make_params(K=6, mu=None, sigma=None, P=None, omega=None, u=3, Nmax=250, epsilon=0.01, kappa=2.0,
                kappa_fixed=True):
    """hyg_sg_params; kappa_fixed=False: kappa is estimated, theta gains the K
    entries log kappa (model_functions.R:65-78) and vartheta has no kappa."""
    if mu is None:
        mu = DEFAULT_MU if K == 6 else [(i + 0.5) / K for i in range(K)]
    if sigma is None:
        sigma = DEFAULT_SIGMA if K == 6 else [0.05 + 0.2 * min(m, 1 - m) for m in mu]
    if omega is None:
        omega = DEFAULT_OMEGA if K == 6 else [0.95] * K
    if P is None:
        P = np.full((K, K), 1.0 / (K - 1))
        np.fill_diagonal(P, 0.0)
    a, b = beta_params(mu, sigma)
    th = theta_from(P, omega)
    kap = np.broadcast_to(np.asarray(kappa, float), (K,))
    if not kappa_fixed:
        th = np.concatenate([th, np.log(kap)])
    p = SgParams()
    p.n_regimes, p.minimum_duration, p.num_particles_max = K, u, Nmax
    p.resample_type, p.is_kappa_fixed, p.theta_len = 2, int(bool(kappa_fixed)), len(th)
    for i in range(K):
        p.alpha[i], p.beta[i], p.kappa[i] = a[i], b[i], (kap[i] if kappa_fixed else 0.0)
    for i, v in enumerate(th):
        p.theta[i] = v
    p.epsilon = epsilon
    return p


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-C", HERE, "-s"], check=True)
        L = C.CDLL(LIB_PATH)
        vp, i32, u64 = C.c_void_p, C.c_int32, C.c_uint64
        L.oracle_sg_chain.restype = i32
        L.oracle_sg_chain.argtypes = [C.POINTER(SgParams), vp, i32, u64, u64, vp, vp]
        L.oracle_sg_chain_refstruct.restype = i32
        L.oracle_sg_chain_refstruct.argtypes = [C.POINTER(SgParams), vp, vp, i32, i32, u64, u64, vp, vp]
        L.oracle_sg_chain_pe.restype = i32
        L.oracle_sg_chain_pe.argtypes = [C.POINTER(SgParams), C.POINTER(SgPeParams), vp, i32, u64, u64, vp, vp]
        L.oracle_sg_pe_hazard.restype = i32
        L.oracle_sg_pe_hazard.argtypes = [C.POINTER(SgParams), vp, i32, vp, vp]
        L.oracle_sg_emission.restype = i32
        L.oracle_sg_emission.argtypes = [C.POINTER(SgParams), vp, vp, i32, C.c_int64, vp]
        L.oracle_sg_hazard.restype = i32
        L.oracle_sg_hazard.argtypes = [C.POINTER(SgParams), i32, i32, vp, vp, C.POINTER(i32)]
        L.oracle_sg_digamma.restype = C.c_double
        L.oracle_sg_digamma.argtypes = [C.c_double]
        L.oracle_sg_consts.restype = i32
        L.oracle_sg_consts.argtypes = [C.POINTER(SgParams), C.POINTER(SgConsts)]
        assert L.oracle_sizeof_sg_params() == C.sizeof(SgParams)
        assert L.oracle_sizeof_sg_consts() == C.sizeof(SgConsts)
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def consts(p):
    c = SgConsts()
    rc = lib().oracle_sg_consts(C.byref(p), C.byref(c))
    if rc != 0:
        raise ValueError(f"invalid parameters ({rc})")
    return c


def emission(p, meth, tot):
    meth = np.ascontiguousarray(meth, np.uint16)
    tot = np.ascontiguousarray(tot, np.uint16)
    if meth.ndim == 1:
        meth, tot = meth[:, None], tot[:, None]
    T, S = tot.shape
    E = np.empty((T, p.n_regimes), np.float64)
    rc = lib().oracle_sg_emission(C.byref(p), _ptr(meth), _ptr(tot), S, T, _ptr(E))
    if rc != 0:
        raise ValueError(rc)
    return E


def chain(p, E, seed=0, chain_id=0, want_nparts=False):
    E = np.ascontiguousarray(E, np.float64)
    T = E.shape[0]
    probs = np.empty((T, p.n_regimes), np.float64)
    nparts = np.zeros(T, np.int32)
    rc = lib().oracle_sg_chain(C.byref(p), _ptr(E), T, seed, chain_id, _ptr(probs),
                               _ptr(nparts) if want_nparts else None)
    out = {"status": rc, "regime_probs": probs}
    if want_nparts:
        out["nparts"] = nparts
    return out


def chain_refstruct(p, meth, tot, seed=0, chain_id=0):
    """chain() with the emission evaluated from the counts at every use (the
    reference's cost structure, sg_oracle.c:sg_em_ref): the same outputs."""
    meth = np.ascontiguousarray(meth, np.uint16)
    tot = np.ascontiguousarray(tot, np.uint16)
    if meth.ndim == 1:
        meth, tot = meth[:, None], tot[:, None]
    T, S = tot.shape
    probs = np.empty((T, p.n_regimes), np.float64)
    rc = lib().oracle_sg_chain_refstruct(C.byref(p), _ptr(meth), _ptr(tot), S, T, seed, chain_id, _ptr(probs), None)
    return {"status": rc, "regime_probs": probs}


def hazard(p, r, n):
    out = np.empty((n, 2), np.float64)
    ex = np.empty(n, np.uint8)
    dcap = C.c_int32(0)
    rc = lib().oracle_sg_hazard(C.byref(p), r, n, _ptr(out), _ptr(ex), C.byref(dcap))
    if rc != 0:
        raise ValueError(rc)
    return out, ex, dcap.value


def chain_pe(p, pe, E, seed=0, chain_id=0):
    """SMC + online smoothing with online parameter estimation: regime
    probabilities [T][K] and theta rows [1 + (T-1)//every][K^2, or K (K + 1)
    with kappa estimated]."""
    E = np.ascontiguousarray(E, np.float64)
    T, K = E.shape[0], p.n_regimes
    probs = np.empty((T, K), np.float64)
    dim = K * K if p.is_kappa_fixed else K * (K + 1)
    theta = np.full((1 + (T - 1) // pe.n_steps_without_update, dim), np.nan)
    rc = lib().oracle_sg_chain_pe(C.byref(p), C.byref(pe), _ptr(E), T, seed, chain_id, _ptr(probs), _ptr(theta))
    return {"status": rc, "regime_probs": probs, "theta": theta}


def pe_hazard(p, theta, L):
    """hazard rows of the estimation path: (base, cont, gomg, gcont) [K][L] and rows valid per regime"""
    K = p.n_regimes
    rows = np.zeros((K, L, 4), np.float64)
    Lr = np.zeros(K, np.int32)
    th = np.ascontiguousarray(theta, np.float64)
    rc = lib().oracle_sg_pe_hazard(C.byref(p), _ptr(th), L, _ptr(rows), _ptr(Lr))
    if rc != 0:
        raise ValueError(rc)
    return rows, Lr


def digamma(x: float) -> float:
    """hyg_digamma (include/hyg_sg_pe.h), the psi of the estimated-kappa tables"""
    return lib().oracle_sg_digamma(float(x))
