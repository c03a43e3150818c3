"""GPU parity of single-group online parameter estimation (SURVEY.md 8f-1;
hyg_sg_run_chain_host_pe / hyg_sg_run_chains_pe of the C ABI) against the CPU
oracle (oracle/sg_oracle.c:oracle_sg_chain_pe): the smoothed regime
probabilities and every theta row (initial + one per update) bit-identical
(f64), for ADAM, plain and L1-normalised gradient steps, K = 3 .. 12, one
chain and batches of chains of different lengths; the committed golden chain.
"""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def lib():
    from hygeia_amd import _lib

    L = _lib.load()
    if L.hyg_device_count() <= 0:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X (gpurun)")
    return L


@pytest.fixture(scope="module")
def sg():
    from oracle import sg_binding

    sg_binding.lib()
    return sg_binding


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def _pe(use_adam, normalise, every, lr_exp=0.1, lr_fac=0.01):
    from hygeia_amd import _lib

    pe = _lib.SgPeParams()
    pe.use_adam, pe.normalise_gradients, pe.n_steps_without_update = use_adam, normalise, every
    pe.learning_rate_exponent, pe.learning_rate_factor = lr_exp, lr_fac
    return pe


def _model(lib, p, max_reads, max_dur):
    from hygeia_amd import _lib

    pp = _lib.SgParams.from_buffer_copy(bytes(p))
    h = C.c_void_p()
    _lib.check(lib.hyg_sg_model_create(C.byref(pp), int(max_reads), int(max_dur), C.byref(h)))
    return h


def _data(K, T, S, cov, seed, u=3):
    from hygeia_amd import synthetic as syn

    mu, sgm = syn.regime_params(K)
    d = syn.simulate(T, S, 1, K=K, seed=seed, coverage=cov, omega=0.9, u=u)
    return d["meth_control"], d["tot_control"], mu, sgm


def _uniform_P(K):
    P = np.full((K, K), 1.0 / (K - 1))
    np.fill_diagonal(P, 0.0)
    return P


def _oracle(sg, p, pe, E, seed, chain_id):
    ope = sg.make_pe(use_adam=bool(pe.use_adam), normalise_gradients=bool(pe.normalise_gradients),
                     every=pe.n_steps_without_update, lr_exponent=pe.learning_rate_exponent,
                     lr_factor=pe.learning_rate_factor)
    return sg.chain_pe(p, ope, E, seed, chain_id)


def _assert_same(out, th, ref):
    bad = np.argwhere(out != ref["regime_probs"])
    assert bad.size == 0, (bad[:5], out[tuple(bad[0])], ref["regime_probs"][tuple(bad[0])])
    badt = np.argwhere(th != ref["theta"])
    assert badt.size == 0, (badt[:5], th[tuple(badt[0])], ref["theta"][tuple(badt[0])])


CASES = [
    # K, T, S, coverage, data seed, N_max, every, use_adam, normalise, u, seed
    (6, 3000, 2, 12.0, 1, 250, 200, 1, 0, 3, 0),  # the pipeline's settings
    (6, 2500, 1, 15.0, 2, 250, 50, 1, 0, 3, 1),   # one sample (the pipeline's per-sample chains), frequent updates
    (4, 1500, 3, 8.0, 3, 30, 25, 0, 1, 2, 2),     # L1-normalised plain steps, small N_max
    (3, 200, 2, 8.0, 4, 250, 199, 0, 0, 3, 3),    # plain step, no resampling (exact score)
    (8, 800, 2, 20.0, 5, 250, 40, 1, 0, 3, 4),    # K = 8
    (12, 400, 2, 20.0, 6, 250, 30, 1, 0, 3, 5),   # K = 12 (256-thread workgroups)
    (6, 1, 2, 10.0, 7, 250, 200, 1, 0, 3, 6),     # one site: theta stays theta_0
    (6, 450, 2, 10.0, 8, 7, 1, 1, 0, 3, 7),       # an update every step, N_max = K + 1
]


@pytest.mark.parametrize("K,T,S,cov,dseed,Nmax,every,adam,norm,u,seed", CASES)
def test_pe_chain_bit_exact(lib, sg, K, T, S, cov, dseed, Nmax, every, adam, norm, u, seed):
    meth, tot, mu, sgm = _data(K, T, S, cov, dseed, u=u)
    omega = sg.DEFAULT_OMEGA if K == 6 else [0.93] * K
    p = sg.make_params(K=K, mu=mu, sigma=sgm, P=_uniform_P(K), omega=omega, u=u, Nmax=Nmax)
    pe = _pe(adam, norm, every, lr_fac=0.01 if adam else 1e-4)
    E = sg.emission(p, meth, tot)
    chain_id = (5 << 32) | seed
    ref = _oracle(sg, p, pe, E, seed, chain_id)
    assert ref["status"] == 0
    h = _model(lib, p, max(int(tot.max()), 1), T + 10)
    try:
        out = np.full((T, K), np.nan)
        th = np.full(ref["theta"].shape, np.nan)
        rc = lib.hyg_sg_run_chain_host_pe(h, C.byref(pe), _ptr(np.ascontiguousarray(meth)),
                                          _ptr(np.ascontiguousarray(tot)), S, T, seed, chain_id, _ptr(out), _ptr(th))
        assert rc == 0, lib.hyg_last_error()
    finally:
        lib.hyg_sg_model_destroy(h)
    _assert_same(out, th, ref)
    if T > every:
        assert not np.array_equal(th[0], th[-1])


def test_pe_golden_fixture(lib, sg):
    g = np.load(os.path.join(GOLDEN, "sg_pe_chain.npz"))
    p = sg.make_params(K=6)
    meth, tot = np.ascontiguousarray(g["meth"]), np.ascontiguousarray(g["tot"])
    T, S = tot.shape
    pe = _pe(1, 0, int(g["every"]))
    h = _model(lib, p, int(tot.max()), T)
    try:
        out = np.full((T, 6), np.nan)
        th = np.full(g["theta"].shape, np.nan)
        rc = lib.hyg_sg_run_chain_host_pe(h, C.byref(pe), _ptr(meth), _ptr(tot), S, T, int(g["seed"]),
                                          int(g["chain_id"]), _ptr(out), _ptr(th))
        assert rc == 0, lib.hyg_last_error()
    finally:
        lib.hyg_sg_model_destroy(h)
    np.testing.assert_array_equal(out, g["regime_probs"])
    np.testing.assert_array_equal(th, g["theta"])


def test_pe_batched_chains_bit_exact(lib, sg):
    """Chains of different lengths in one launch (one workgroup each, theta rows
    of chain i after chain i-1's), each equal to its own oracle chain."""
    from hygeia_amd import _lib

    K, S, every = 6, 2, 60
    lens = [1, 61, 900, 2500, 1200, 3, 640, 120]
    total = sum(lens)
    meth, tot, mu, sgm = _data(K, total, S, 15.0, 31)
    p = sg.make_params(K=K)
    pe = _pe(1, 0, every)
    h = _model(lib, p, int(tot.max()), max(lens))
    try:
        arr = (_lib.SgChain * len(lens))()
        begins = np.concatenate([[0], np.cumsum(lens)[:-1]])
        for i, (b, n) in enumerate(zip(begins, lens)):
            arr[i].site_begin, arr[i].n_sites = int(b), int(n)
            arr[i].seed, arr[i].chain_id, arr[i].out_begin = 13, (i << 32) | 9, int(b)
        rows = lib.hyg_sg_pe_theta_rows(arr, len(lens), every)
        assert rows == sum(1 + (n - 1) // every for n in lens)
        dm = torch.from_numpy(meth.view(np.int16)).cuda()
        dt = torch.from_numpy(tot.view(np.int16)).cuda()
        E = torch.empty((total, K), dtype=torch.float64, device="cuda")
        stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        _lib.check(lib.hyg_sg_emission(h, dm.data_ptr(), dt.data_ptr(), S, total, E.data_ptr(), stream))
        wsb = lib.hyg_sg_pe_workspace_bytes(h, arr, len(lens), 1024)
        ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
        probs = torch.full((total, K), float("nan"), dtype=torch.float64, device="cuda")
        theta = torch.full((rows, K * K), float("nan"), dtype=torch.float64, device="cuda")
        st = torch.full((len(lens),), 99, dtype=torch.int32, device="cuda")
        _lib.check(lib.hyg_sg_run_chains_pe(h, C.byref(pe), arr, len(lens), E.data_ptr(), ws.data_ptr(), wsb, 1024,
                                            probs.data_ptr(), theta.data_ptr(), st.data_ptr(), stream))
        torch.cuda.synchronize()
        out, th, status = probs.cpu().numpy(), theta.cpu().numpy(), st.cpu().numpy()
        # too small a workspace is refused
        assert lib.hyg_sg_run_chains_pe(h, C.byref(pe), arr, len(lens), E.data_ptr(), ws.data_ptr(), wsb - 1, 1024,
                                        probs.data_ptr(), theta.data_ptr(), st.data_ptr(), stream) == -1
    finally:
        lib.hyg_sg_model_destroy(h)
    assert np.all(status == 0)
    Eh = sg.emission(p, meth, tot)
    r0 = 0
    for i, (b, n) in enumerate(zip(begins, lens)):
        ref = _oracle(sg, p, pe, Eh[b:b + n], 13, (i << 32) | 9)
        nr = ref["theta"].shape[0]
        _assert_same(out[b:b + n], th[r0:r0 + nr], ref)
        r0 += nr


KAPPA_CASES = [
    # K, T, S, coverage, data seed, N_max, every, use_adam, normalise, kappa, seed
    (6, 3000, 2, 12.0, 11, 250, 200, 1, 0, (2.0, 1.5, 3.0, 0.7, 2.5, 5.0), 0),  # pipeline settings, kappa estimated
    (4, 1500, 3, 8.0, 12, 30, 25, 0, 1, (1.2, 2.0, 0.4, 8.0), 1),               # L1-normalised plain steps
    (3, 600, 2, 10.0, 13, 250, 20, 1, 0, (2.0, 2.0, 2.0), 2),
    (12, 400, 2, 20.0, 14, 250, 30, 1, 0, (0.8, 1.0, 1.5, 2.0, 2.5, 3.0, 4.0, 0.5, 1.2, 2.2, 6.0, 1.7), 3),  # 256 threads
]


@pytest.mark.parametrize("K,T,S,cov,dseed,Nmax,every,adam,norm,kappa,seed", KAPPA_CASES)
def test_pe_kappa_estimated_bit_exact(lib, sg, K, T, S, cov, dseed, Nmax, every, adam, norm, kappa, seed):
    """--is_kappa_fixed FALSE: theta of K (K + 1) entries; the kernel's score
    drops the kappa coordinates (identically 0, include/hyg_sg_pe.h) where the
    oracle carries all K (K + 1) as singleGroup.h:641-706 writes them: every
    regime probability and theta row bit-identical, log kappa unmoved."""
    meth, tot, mu, sgm = _data(K, T, S, cov, dseed)
    omega = sg.DEFAULT_OMEGA if K == 6 else [0.93] * K
    p = sg.make_params(K=K, mu=mu, sigma=sgm, P=_uniform_P(K), omega=omega, Nmax=Nmax, kappa=kappa,
                       kappa_fixed=False)
    pe = _pe(adam, norm, every, lr_fac=0.01 if adam else 1e-4)
    E = sg.emission(p, meth, tot)
    chain_id = (7 << 32) | seed
    ref = _oracle(sg, p, pe, E, seed, chain_id)
    assert ref["status"] == 0 and ref["theta"].shape[1] == K * (K + 1)
    h = _model(lib, p, max(int(tot.max()), 1), T + 10)
    try:
        out = np.full((T, K), np.nan)
        th = np.full(ref["theta"].shape, np.nan)
        rc = lib.hyg_sg_run_chain_host_pe(h, C.byref(pe), _ptr(np.ascontiguousarray(meth)),
                                          _ptr(np.ascontiguousarray(tot)), S, T, seed, chain_id, _ptr(out), _ptr(th))
        assert rc == 0, lib.hyg_last_error()
    finally:
        lib.hyg_sg_model_destroy(h)
    _assert_same(out, th, ref)
    np.testing.assert_array_equal(th[:, K * K:], np.tile(np.log(np.asarray(kappa, float)), (th.shape[0], 1)))
    assert not np.array_equal(th[0, :K * K], th[-1, :K * K])
