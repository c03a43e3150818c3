"""The C-ABI library (include/hygeia_amd.h -> hygeia_amd/lib/libhygeia_amd.so) on a
host without a GPU: it loads, exports every declared symbol, validates
parameters, builds the model tables, and refuses to compute (HYG_EDEVICE):
there is no CPU fallback in the product path.
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

from hygeia_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(ROOT, "include", "hygeia_amd.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(hyg_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    return _lib.load()


def test_exports_every_declared_symbol(lib):
    names = _declared()
    assert len(names) >= 13
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_lib.EXPORTS)
    assert lib.hyg_version().decode().startswith("hygeia_amd")
    assert lib.hyg_version().decode() == _lib.VERSION  # what `hygeia --version` prints without loading it


def test_device_cus_cached_per_device(lib):
    """The launcher's CU count is kept per device (hyg_set_device may switch
    between GPUs of different sizes): two faked devices keep their own counts,
    and dropping an override leaves the other in place."""
    try:
        assert lib.hyg_tg_set_device_cus(0, 256) == 0 and lib.hyg_tg_set_device_cus(1, 64) == 0
        assert lib.hyg_tg_device_cus(0) == 256 and lib.hyg_tg_device_cus(1) == 64
        assert lib.hyg_tg_set_device_cus(1, 80) == 0
        assert lib.hyg_tg_device_cus(0) == 256 and lib.hyg_tg_device_cus(1) == 80
        assert lib.hyg_tg_set_device_cus(0, 0) == 0
        assert lib.hyg_tg_device_cus(1) == 80
        if lib.hyg_device_count() == 0:
            assert lib.hyg_tg_device_cus(0) == 0  # no HIP device: unknown
        assert lib.hyg_tg_set_device_cus(-1, 4) == -1 and lib.hyg_tg_set_device_cus(64, 4) == -1
        assert lib.hyg_tg_set_device_cus(0, -4) == -1
    finally:
        lib.hyg_tg_set_device_cus(0, 0)
        lib.hyg_tg_set_device_cus(1, 0)


def test_params_default_matches_reference_flags(lib):
    p = _lib.TgParams()
    lib.hyg_tg_params_default(C.byref(p))
    assert (p.n_regimes, p.minimum_duration, p.num_resampled_ancestors, p.num_samples_backward) == (6, 3, 50, 25)
    assert p.optimal_resampling == 1 and p.multinomial == 0
    assert p.omega_case == pytest.approx(0.8)
    assert p.split_prob == pytest.approx(0.01)
    assert p.merge_log_prob == pytest.approx(np.log(0.1))
    assert p.kappa_control == 2.0 and p.kappa_case == 2.0


def _params():
    from hygeia_amd import two_group
    mu = [0.95, 0.05, 0.8, 0.2, 0.5, 0.5]
    sg = [0.05, 0.05, 0.1, 0.1, 0.1, 0.2886751]
    return _lib.make_params(mu, sg, two_group.uniform_theta(6, 0.8))


def test_model_create_and_sizes_without_device(lib):
    m = C.c_void_p()
    rc = lib.hyg_tg_model_create(C.byref(_params()), 200, 1000, C.byref(m))
    assert rc == _lib.HYG_OK, lib.hyg_last_error()
    try:
        assert lib.hyg_tg_num_particles(m) == 2400
        ws = lib.hyg_tg_workspace_bytes(m, 3, 1000)
        assert ws >= 1000 * (32 + 16 * 50)
    finally:
        lib.hyg_tg_model_destroy(m)


@pytest.mark.parametrize("field,value", [("n_regimes", 1), ("n_regimes", 17), ("num_resampled_ancestors", 0),
                                         ("num_samples_backward", 0), ("minimum_duration", -1)])
def test_model_create_rejects_invalid(lib, field, value):
    p = _params()
    setattr(p, field, value)
    m = C.c_void_p()
    rc = lib.hyg_tg_model_create(C.byref(p), 200, 1000, C.byref(m))
    assert rc == _lib.HYG_EINVAL
    assert lib.hyg_last_error()


def test_sigma_outside_beta_range_is_rejected(lib):
    p = _params()
    p.sigma[0] = 0.6  # nu = mu(1-mu)/sigma^2 - 1 < 0
    m = C.c_void_p()
    assert lib.hyg_tg_model_create(C.byref(p), 200, 1000, C.byref(m)) == _lib.HYG_EINVAL


def test_compute_refuses_without_device(lib):
    if lib.hyg_device_count() > 0:
        pytest.skip("host without a GPU only")
    m = C.c_void_p()
    assert lib.hyg_tg_model_create(C.byref(_params()), 200, 1000, C.byref(m)) == _lib.HYG_OK
    try:
        T = 10
        z = np.zeros((T, 2), np.uint16)
        out = {k: np.zeros(s, dt) for k, s, dt in (("mg", (T, 25), np.int16), ("ct", (T, 25, 2), np.int16),
                                                   ("ks", (T, 25, 2), np.int16), ("sp", T, np.float32),
                                                   ("rp", (T, 12), np.float32), ("lz", 1, np.float64))}
        ptr = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
        rc = lib.hyg_tg_run_chain_host(m, ptr(z), ptr(z), 2, ptr(z), ptr(z), 2, T, 0, 0, ptr(out["mg"]),
                                       ptr(out["ct"]), ptr(out["ks"]), ptr(out["sp"]), ptr(out["rp"]),
                                       ptr(out["lz"]), None)
        assert rc == _lib.HYG_EDEVICE
        assert b"no CPU fallback" in lib.hyg_last_error()
        E = np.zeros((T, 12))
        rc = lib.hyg_tg_emission(m, ptr(z), ptr(z), 2, ptr(z), ptr(z), 2, T, ptr(E), None)
        assert rc == _lib.HYG_EDEVICE
        ch = (_lib.TgChain * 1)()
        ch[0].n_sites = T
        st = np.zeros(1, np.int32)
        rc = lib.hyg_tg_run_chains_host(m, ptr(z), ptr(z), 2, ptr(z), ptr(z), 2, T, ch, 1, T, ptr(out["mg"]),
                                        ptr(out["ct"]), ptr(out["ks"]), ptr(out["sp"]), ptr(out["rp"]),
                                        ptr(out["lz"]), None, ptr(st))
        assert rc == _lib.HYG_EDEVICE
    finally:
        lib.hyg_tg_model_destroy(m)


def test_pipeline_shape_lds_stays_under_the_three_per_cu_boundary(lib):
    """C3 on one GPU holds three 256-thread forward chains per CU. The forward's
    LDS at the pipeline shape (K = 6, M = 50, B = 25) is 53 648 B (53 520 B and a
    32-entry uniform ring, round 5), which fits three times (C3 forward 1973 ->
    1907 ms, profiles/r05p_uring256_ab.txt); 53 776 B measured two per CU on the
    MI355X while the HIP occupancy query still said three (C3 forward 1957 ->
    2887 ms, profiles/r04s). Growing the 256-thread layout needs a GPU check of C3
    first."""
    m = C.c_void_p()
    assert lib.hyg_tg_model_create(C.byref(_params()), 200, 1000, C.byref(m)) == _lib.HYG_OK
    try:
        fwd256 = lib.hyg_tg_lds_bytes(m, 256, 0)
        assert 0 < fwd256 <= 53648
        assert 3 * lib.hyg_tg_lds_bytes(m, 256, 1) <= 160 * 1024  # the backward at three per CU
        for nt in (512, 768):  # one chain per CU
            assert 0 < lib.hyg_tg_lds_bytes(m, nt, 0) <= 160 * 1024
        assert lib.hyg_tg_lds_bytes(m, 300, 0) == 0 and lib.hyg_tg_lds_bytes(None, 256, 0) == 0
    finally:
        lib.hyg_tg_model_destroy(m)


def test_product_package_does_not_import_oracle():
    """The product path must never route through the CPU oracle."""
    pkg = os.path.join(ROOT, "hygeia_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.sub(r"(#|//).*", "", txt).replace("oracle/", ""), f


# ------------------------------------------------------------ single group
def _sg_params(**kw):
    from oracle import sg_binding

    return _lib.SgParams.from_buffer_copy(bytes(sg_binding.make_params(**kw)))


def test_sg_struct_layout_matches_c():
    from oracle import sg_binding

    assert C.sizeof(_lib.SgParams) == sg_binding.lib().oracle_sizeof_sg_params()
    assert C.sizeof(_lib.SgChain) == 40


def test_sg_params_default_is_pipeline_config(lib):
    p = _lib.SgParams()
    lib.hyg_sg_params_default(C.byref(p))
    assert (p.n_regimes, p.minimum_duration, p.num_particles_max, p.resample_type) == (6, 3, 250, 2)
    assert p.epsilon == 0.01 and p.is_kappa_fixed == 1 and p.theta_len == 36
    np.testing.assert_allclose(list(p.alpha[:6]), [17.1, 0.9, 12, 3, 12, 1], rtol=1e-6)
    m = C.c_void_p()
    assert lib.hyg_sg_model_create(C.byref(p), 100, 1000, C.byref(m)) == _lib.HYG_OK
    lib.hyg_sg_model_destroy(m)


def test_sg_model_create_and_workspace(lib):
    m = C.c_void_p()
    assert lib.hyg_sg_model_create(C.byref(_sg_params(K=6)), 100, 5000, C.byref(m)) == _lib.HYG_OK
    try:
        one = lib.hyg_sg_workspace_bytes(m, 1, 64)
        assert one >= 64 * 6 * 256 * 8
        # a per-launch header (descriptors, status, ring control words) plus a region per chain
        two, three = lib.hyg_sg_workspace_bytes(m, 2, 64), lib.hyg_sg_workspace_bytes(m, 3, 64)
        assert three - two >= 64 * 6 * 256 * 8 and two - one >= 64 * 6 * 256 * 8
        assert lib.hyg_sg_workspace_bytes(m, 1, 0) > lib.hyg_sg_workspace_bytes(m, 1, 64)
    finally:
        lib.hyg_sg_model_destroy(m)


@pytest.mark.parametrize("field,value,code", [("n_regimes", 1, _lib.HYG_EINVAL), ("num_particles_max", 6, _lib.HYG_EINVAL),
                                              ("num_particles_max", 300, _lib.HYG_EUNSUPPORTED),
                                              ("resample_type", 1, _lib.HYG_EUNSUPPORTED),
                                              ("minimum_duration", 0, _lib.HYG_EINVAL),
                                              ("theta_len", 35, _lib.HYG_EINVAL), ("epsilon", 0.0, _lib.HYG_EINVAL)])
def test_sg_model_create_rejects_invalid(lib, field, value, code):
    p = _sg_params(K=6)
    setattr(p, field, value)
    m = C.c_void_p()
    assert lib.hyg_sg_model_create(C.byref(p), 100, 1000, C.byref(m)) == code
    assert lib.hyg_last_error()


def test_sg_compute_refuses_without_device(lib):
    if lib.hyg_device_count() > 0:
        pytest.skip("host without a GPU only")
    m = C.c_void_p()
    assert lib.hyg_sg_model_create(C.byref(_sg_params(K=6)), 100, 1000, C.byref(m)) == _lib.HYG_OK
    try:
        T = 10
        z = np.zeros((T, 2), np.uint16)
        out = np.zeros((T, 6))
        ptr = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
        assert lib.hyg_sg_run_chain_host(m, ptr(z), ptr(z), 2, T, 0, 0, ptr(out)) == _lib.HYG_EDEVICE
        assert b"no CPU fallback" in lib.hyg_last_error()
        assert lib.hyg_sg_emission(m, ptr(z), ptr(z), 2, T, ptr(out), None) == _lib.HYG_EDEVICE
    finally:
        lib.hyg_sg_model_destroy(m)


def test_run_chains_host_rejects_empty_and_overlapping_chains(lib):
    """run_chains_host refuses an empty chain list and chains whose output rows
    [out_begin, out_begin + n_sites) overlap or leave [0, n_out_rows): the
    kernels would write the same rows from two workgroups."""
    from hygeia_amd import two_group

    mu = [0.95, 0.05, 0.8, 0.2, 0.5, 0.5]
    sg = [0.05, 0.05, 0.1, 0.1, 0.1, 0.2886751]
    model = two_group.CaseControlModel(mu, sg, two_group.uniform_theta(6, 0.8), max_total_reads=50, max_duration=100)
    z = np.zeros((60, 2), np.uint16)
    obs, tot = {"control": z, "case": z}, {"control": z, "case": z}
    with pytest.raises(ValueError, match="no chains"):
        two_group.run_chains_host(obs, tot, model, [], 10)
    for chains, rows in (([(0, 30, 0, 1, 0), (10, 30, 1, 1, 29)], 60), ([(0, 30, 0, 1, 31)], 60),
                         ([(0, 30, 0, 1, -1)], 60)):
        with pytest.raises(ValueError, match="disjoint"):
            two_group.run_chains_host(obs, tot, model, chains, rows)


def test_threads_per_chain_m_above_64_takes_256(lib):
    """A model with M > 64 runs the 256-thread kernels whatever its LDS (the wider
    kernels hold one ancestor per lane); this branch needs no device."""
    from hygeia_amd import two_group

    mu = [(i + 0.5) / 12 for i in range(12)]
    sg = [0.08 + 0.04 * (i % 2) for i in range(12)]
    model = two_group.CaseControlModel(mu, sg, two_group.uniform_theta(12, 0.8), num_resampled_ancestors=65,
                                       max_total_reads=50, max_duration=100)
    assert lib.hyg_tg_threads_per_chain(model.handle, 1) == 256
    assert lib.hyg_tg_threads_per_chain(model.handle, 10000) == 256


def test_c5_backward_keeps_full_weights_in_global_memory(lib):
    """The C5 shape's 256-thread backward (GW) holds its lists alone in LDS: three
    chains per CU fit (the LDS W of 8 400 f64 held one); its full-N weights take
    one Nmax f64 scratch per chain in the workspace. No device needed."""
    from hygeia_amd import synthetic as syn
    from hygeia_amd import two_group

    mu, sg = syn.regime_params(12)
    m = two_group.CaseControlModel(mu, sg, two_group.uniform_theta(12, 0.8), max_total_reads=300, max_duration=1000)
    assert 3 * lib.hyg_tg_lds_bytes(m.handle, 256, 1) <= 160 * 1024
    assert lib.hyg_tg_lds_bytes(m.handle, 768, 1) > 8400 * 8  # the one-per-CU width keeps W in LDS
    one, two = (lib.hyg_tg_workspace_bytes(m.handle, n, 1000) for n in (1, 2))
    assert two - one >= 8400 * 8
    mu6, sg6 = syn.regime_params(6)
    m6 = two_group.CaseControlModel(mu6, sg6, two_group.uniform_theta(6, 0.8), max_total_reads=300, max_duration=1000)
    one6, two6 = (lib.hyg_tg_workspace_bytes(m6.handle, n, 1000) for n in (1, 2))
    assert two6 - one6 < 2400 * 8  # no scratch for the pipeline shape
