"""ctypes binding of the C ABI (include/hygeia_amd.h) -> hygeia_amd/lib/libhygeia_amd.so.

There is no CPU fallback: if the library cannot be loaded this module raises,
and every compute entry point of the library returns HYG_EDEVICE without a HIP
device.
"""
from __future__ import annotations

import ctypes as C
import math
import os

KMAX = 16
HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libhygeia_amd.so")

HYG_OK, HYG_EINVAL, HYG_ENUMERIC, HYG_EDEVICE, HYG_ENOMEM, HYG_EUNSUPPORTED = 0, -1, -2, -3, -4, -5
ERROR_NAMES = {0: "HYG_OK", -1: "HYG_EINVAL", -2: "HYG_ENUMERIC", -3: "HYG_EDEVICE", -4: "HYG_ENOMEM",
               -5: "HYG_EUNSUPPORTED"}


class HygError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code


class TgParams(C.Structure):
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


class TgChain(C.Structure):
    _fields_ = [
        ("site_begin", C.c_int64),
        ("n_sites", C.c_int32),
        ("_pad", C.c_int32),
        ("seed", C.c_uint64),
        ("chain_id", C.c_uint64),
        ("out_begin", C.c_int64),
    ]


class TgOutputs(C.Structure):
    _fields_ = [
        ("merged", C.c_void_p),
        ("control", C.c_void_p),
        ("kase", C.c_void_p),
        ("split_probs", C.c_void_p),
        ("regime_probs", C.c_void_p),
        ("log_z", C.c_void_p),
        ("final_log_weights", C.c_void_p),
        ("status", C.c_void_p),
    ]


class SgParams(C.Structure):
    """Mirror of hyg_sg_params (include/hygeia_amd.h)."""

    _fields_ = [
        ("n_regimes", C.c_int32),
        ("minimum_duration", C.c_int32),
        ("num_particles_max", C.c_int32),
        ("resample_type", C.c_int32),
        ("is_kappa_fixed", C.c_int32),
        ("theta_len", C.c_int32),
        ("alpha", C.c_double * KMAX),
        ("beta", C.c_double * KMAX),
        ("kappa", C.c_double * KMAX),
        ("theta", C.c_double * (KMAX * (KMAX + 1))),
        ("epsilon", C.c_double),
    ]


class SgPeParams(C.Structure):
    """Mirror of hyg_sg_pe_params (include/hygeia_amd.h)."""

    _fields_ = [
        ("use_adam", C.c_int32),
        ("normalise_gradients", C.c_int32),
        ("n_steps_without_update", C.c_int32),
        ("_pad", C.c_int32),
        ("learning_rate_exponent", C.c_double),
        ("learning_rate_factor", C.c_double),
    ]


class SgChain(C.Structure):
    _fields_ = [
        ("site_begin", C.c_int64),
        ("n_sites", C.c_int32),
        ("_pad", C.c_int32),
        ("seed", C.c_uint64),
        ("chain_id", C.c_uint64),
        ("out_begin", C.c_int64),
    ]


EXPORTS = ("hyg_tg_params_default", "hyg_tg_model_create", "hyg_tg_model_destroy", "hyg_tg_num_particles",
           "hyg_tg_threads_per_chain", "hyg_tg_force_threads", "hyg_tg_set_tail_overlap", "hyg_tg_device_cus",
           "hyg_tg_set_device_cus", "hyg_sg_force_key_drop", "hyg_tg_chains_per_cu", "hyg_tg_lds_bytes",
           "hyg_tg_emission", "hyg_tg_workspace_bytes", "hyg_tg_run_chains", "hyg_tg_run_chain_host",
           "hyg_tg_run_chains_host",
           "hyg_device_count", "hyg_device_slot_acquire", "hyg_device_slot_release", "hyg_set_device",
           "hyg_get_device", "hyg_last_error", "hyg_version", "hyg_set_kernel_timing", "hyg_tg_last_kernel_ms",
           "hyg_sg_params_default", "hyg_sg_model_create", "hyg_sg_model_destroy", "hyg_sg_emission",
           "hyg_sg_workspace_bytes", "hyg_sg_run_chains", "hyg_sg_run_chain_host",
           "hyg_sg_pe_params_default", "hyg_sg_pe_theta_rows", "hyg_sg_pe_workspace_bytes", "hyg_sg_run_chains_pe",
           "hyg_sg_run_chain_host_pe", "hyg_bed_labels", "hyg_bed_format", "hyg_pre_collapse",
           "hyg_dmp_site_counts", "hyg_dmp_fdr", "hyg_dmp_weighted_fdr", "hyg_tg_posterior_counts")


class DmpGroup(C.Structure):
    """Mirror of hyg_dmp_group (include/hygeia_amd.h)."""

    _fields_ = [("site_begin", C.c_int64), ("n_rows", C.c_int64)]

_lib = None

# The library's version string (hyg_version(), capi.cpp); `hygeia --version`
# prints it without loading the library (tests/test_capi_cpu.py pins the two
# equal).
VERSION = "hygeia_amd 0.1.0 (gfx950)"

_with_torch = False  # whether torch was imported before the library loaded


def loaded_with_torch() -> bool:
    """True when the library was loaded after torch (its HIP runtime first)."""
    return _lib is not None and _with_torch


def load(import_torch: bool = True) -> C.CDLL:
    """Loads (building first if needed) the HIP library; raises if impossible.

    import_torch=False: for a process that never touches torch (the single-task
    `hygeia infer`, which runs its chain through the host-pointer entry
    hyg_tg_run_chain_host): torch's import (about 2 s of a fresh process) is
    skipped. Such a process must not use torch's HIP afterwards (DeviceChains
    refuses to)."""
    global _lib, _with_torch
    if _lib is not None:
        return _lib
    # PyTorch-ROCm ships its own HIP runtime (torch/lib/libamdhip64.so) next to
    # the system one this library links. Both work in one process only when
    # torch's is initialised first, so torch is imported before our runtime
    # can initialise (it is the device-memory / stream plumbing anyway).
    if import_torch:
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    import sys

    _with_torch = "torch" in sys.modules  # (its runtime loaded first, whoever imported it)
    path = os.environ.get("HYG_LIB_PATH", LIB_PATH)  # A/B builds of the same sources (tools/)
    if path == LIB_PATH and not os.path.exists(LIB_PATH):
        from . import build as _build
        _build.build()
    L = C.CDLL(path)
    vp, i32, i64, u64, sz = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.c_size_t
    L.hyg_tg_params_default.restype = None
    L.hyg_tg_params_default.argtypes = [C.POINTER(TgParams)]
    L.hyg_tg_model_create.restype = C.c_int
    L.hyg_tg_model_create.argtypes = [C.POINTER(TgParams), i32, i32, C.POINTER(vp)]
    L.hyg_tg_model_destroy.restype = None
    L.hyg_tg_model_destroy.argtypes = [vp]
    L.hyg_tg_num_particles.restype = i32
    L.hyg_tg_num_particles.argtypes = [vp]
    L.hyg_tg_threads_per_chain.restype = i32
    L.hyg_tg_threads_per_chain.argtypes = [vp, i32]
    L.hyg_tg_force_threads.restype = C.c_int
    L.hyg_tg_force_threads.argtypes = [i32, i32]
    L.hyg_tg_set_tail_overlap.restype = C.c_int
    L.hyg_tg_set_tail_overlap.argtypes = [i32]
    L.hyg_tg_device_cus.restype = i32
    L.hyg_tg_device_cus.argtypes = [i32]
    L.hyg_tg_set_device_cus.restype = C.c_int
    L.hyg_tg_set_device_cus.argtypes = [i32, i32]
    L.hyg_sg_force_key_drop.restype = C.c_int
    L.hyg_sg_force_key_drop.argtypes = [i32]
    L.hyg_tg_chains_per_cu.restype = i32
    L.hyg_tg_chains_per_cu.argtypes = [vp, i32]
    L.hyg_tg_lds_bytes.restype = sz
    L.hyg_tg_lds_bytes.argtypes = [vp, i32, i32]
    L.hyg_tg_emission.restype = C.c_int
    L.hyg_tg_emission.argtypes = [vp, vp, vp, i32, vp, vp, i32, i64, vp, vp]
    L.hyg_tg_workspace_bytes.restype = sz
    L.hyg_tg_workspace_bytes.argtypes = [vp, i32, i64]
    L.hyg_tg_run_chains.restype = C.c_int
    L.hyg_tg_run_chains.argtypes = [vp, C.POINTER(TgChain), i32, vp, vp, sz, C.POINTER(TgOutputs), vp]
    L.hyg_tg_run_chain_host.restype = C.c_int
    L.hyg_tg_run_chain_host.argtypes = [vp, vp, vp, i32, vp, vp, i32, i32, u64, u64, vp, vp, vp, vp, vp, vp, vp]
    L.hyg_tg_run_chains_host.restype = C.c_int
    L.hyg_tg_run_chains_host.argtypes = [vp, vp, vp, i32, vp, vp, i32, i64, C.POINTER(TgChain), i32, i64,
                                         vp, vp, vp, vp, vp, vp, vp, vp]
    L.hyg_device_count.restype = C.c_int
    L.hyg_device_count.argtypes = []
    L.hyg_device_slot_acquire.restype = C.c_int
    L.hyg_device_slot_acquire.argtypes = [C.c_char_p, i32, i32, C.POINTER(i32), C.POINTER(i32)]
    L.hyg_device_slot_release.restype = C.c_int
    L.hyg_device_slot_release.argtypes = []
    L.hyg_set_device.restype = C.c_int
    L.hyg_set_device.argtypes = [i32]
    L.hyg_get_device.restype = C.c_int
    L.hyg_get_device.argtypes = []
    L.hyg_last_error.restype = C.c_char_p
    L.hyg_last_error.argtypes = []
    L.hyg_set_kernel_timing.restype = None
    L.hyg_set_kernel_timing.argtypes = [C.c_int]
    L.hyg_tg_last_kernel_ms.restype = C.c_int
    L.hyg_tg_last_kernel_ms.argtypes = [C.POINTER(C.c_float)]
    L.hyg_sg_params_default.restype = None
    L.hyg_sg_params_default.argtypes = [C.POINTER(SgParams)]
    L.hyg_sg_model_create.restype = C.c_int
    L.hyg_sg_model_create.argtypes = [C.POINTER(SgParams), i32, i32, C.POINTER(vp)]
    L.hyg_sg_model_destroy.restype = None
    L.hyg_sg_model_destroy.argtypes = [vp]
    L.hyg_sg_emission.restype = C.c_int
    L.hyg_sg_emission.argtypes = [vp, vp, vp, i32, i64, vp, vp]
    L.hyg_sg_workspace_bytes.restype = sz
    L.hyg_sg_workspace_bytes.argtypes = [vp, i32, i32]
    L.hyg_sg_run_chains.restype = C.c_int
    L.hyg_sg_run_chains.argtypes = [vp, C.POINTER(SgChain), i32, vp, vp, sz, i32, vp, vp, vp]
    L.hyg_sg_run_chain_host.restype = C.c_int
    L.hyg_sg_run_chain_host.argtypes = [vp, vp, vp, i32, i32, u64, u64, vp]
    L.hyg_sg_pe_params_default.restype = None
    L.hyg_sg_pe_params_default.argtypes = [C.POINTER(SgPeParams)]
    L.hyg_sg_pe_theta_rows.restype = i64
    L.hyg_sg_pe_theta_rows.argtypes = [C.POINTER(SgChain), i32, i32]
    L.hyg_sg_pe_workspace_bytes.restype = sz
    L.hyg_sg_pe_workspace_bytes.argtypes = [vp, C.POINTER(SgChain), i32, i32]
    L.hyg_sg_run_chains_pe.restype = C.c_int
    L.hyg_sg_run_chains_pe.argtypes = [vp, C.POINTER(SgPeParams), C.POINTER(SgChain), i32, vp, vp, sz, i32, vp, vp,
                                       vp, vp]
    L.hyg_pre_collapse.restype = C.c_int
    L.hyg_pre_collapse.argtypes = [vp, i64, vp, vp, vp, vp, i64, vp, vp, vp, i64, i32, vp, vp, i32, i32, vp, vp]
    L.hyg_bed_labels.restype = C.c_int
    L.hyg_bed_labels.argtypes = [vp, i32, i64, vp, vp, vp]
    L.hyg_bed_format.restype = i64
    L.hyg_bed_format.argtypes = [C.c_char_p, vp, vp, vp, i64, i32, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                 vp, i64]
    L.hyg_sg_run_chain_host_pe.restype = C.c_int
    L.hyg_sg_run_chain_host_pe.argtypes = [vp, C.POINTER(SgPeParams), vp, vp, i32, i32, u64, u64, vp, vp]
    L.hyg_tg_posterior_counts.restype = C.c_int
    L.hyg_tg_posterior_counts.argtypes = [vp, vp, i32, i32, vp, i32, i64, i32, vp, vp]
    L.hyg_dmp_site_counts.restype = C.c_int
    L.hyg_dmp_site_counts.argtypes = [vp, vp, vp, i32, i32, C.POINTER(DmpGroup), C.POINTER(i64), i32, i32, i64, vp,
                                      vp, vp]
    L.hyg_dmp_fdr.restype = C.c_int
    L.hyg_dmp_fdr.argtypes = [vp, i32, i32, i64, i32, C.c_double, C.POINTER(i64), C.POINTER(C.c_double),
                              C.POINTER(C.c_double), vp]
    L.hyg_dmp_weighted_fdr.restype = C.c_int
    L.hyg_dmp_weighted_fdr.argtypes = [vp, i32, i32, i64, i32, C.c_double, vp, vp, vp, C.POINTER(i64),
                                       C.POINTER(C.c_double), vp]
    L.hyg_version.restype = C.c_char_p
    L.hyg_version.argtypes = []
    _lib = L
    return L


def check(code: int) -> None:
    if code != HYG_OK:
        msg = load().hyg_last_error().decode(errors="replace")
        raise HygError(code, msg)


def make_params(mu, sigma, theta, minimum_duration: int = 3, num_resampled_ancestors: int = 50,
                num_samples_backward: int = 25, omega_case: float = 0.8, merge_log_prob: float = math.log(0.1),
                split_prob: float = 0.01, kappa_control: float = 2.0, kappa_case: float = 2.0,
                optimal_resampling: bool = True, multinomial: bool = False) -> TgParams:
    K = len(mu)
    if len(sigma) != K:
        raise ValueError("mu and sigma must have the same length")
    if not 2 <= K <= KMAX:
        raise ValueError(f"number of regimes must be in [2, {KMAX}]")
    if len(theta) > KMAX * KMAX:
        raise ValueError("theta too long")
    p = TgParams()
    p.n_regimes = K
    p.minimum_duration = int(minimum_duration)
    p.num_resampled_ancestors = int(num_resampled_ancestors)
    p.num_samples_backward = int(num_samples_backward)
    p.optimal_resampling = 1 if optimal_resampling else 0
    p.multinomial = 1 if multinomial else 0
    p.theta_len = len(theta)
    for i in range(K):
        p.mu[i] = float(mu[i])
        p.sigma[i] = float(sigma[i])
    for i, v in enumerate(theta):
        p.theta[i] = float(v)
    p.omega_case = float(omega_case)
    p.merge_log_prob = float(merge_log_prob)
    p.split_prob = float(split_prob)
    p.kappa_control = float(kappa_control)
    p.kappa_case = float(kappa_case)
    return p
