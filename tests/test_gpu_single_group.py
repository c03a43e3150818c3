"""GPU parity of the single-group path (hyg_sg_* of the C ABI) against the CPU
oracle (oracle/sg_oracle.c): bit-exact emission tables and bit-exact smoothed
regime probabilities (f64), chain by chain, for one chain through
hyg_sg_run_chain_host and for batches of chains through hyg_sg_run_chains on
device buffers. Also the error paths (pending-time capacity, invalid counts).
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


class Model:
    def __init__(self, lib, p, max_reads, max_dur):
        from hygeia_amd import _lib

        self.lib, self._lib = lib, _lib
        self.p = _lib.SgParams.from_buffer_copy(bytes(p))
        self.K = p.n_regimes
        self.h = C.c_void_p()
        _lib.check(lib.hyg_sg_model_create(C.byref(self.p), int(max_reads), int(max_dur), C.byref(self.h)))

    def chain_host(self, meth, tot, seed, chain_id):
        meth = np.ascontiguousarray(meth, np.uint16)
        tot = np.ascontiguousarray(tot, np.uint16)
        T, S = tot.shape
        out = np.full((T, self.K), np.nan)
        rc = self.lib.hyg_sg_run_chain_host(self.h, _ptr(meth), _ptr(tot), S, T, seed, chain_id, _ptr(out))
        return rc, out

    def close(self):
        self.lib.hyg_sg_model_destroy(self.h)


def _data(K, T, S, cov, seed, omega=0.9, u=3):
    from hygeia_amd import synthetic as syn

    mu, sgm = syn.regime_params(K)
    d = syn.simulate(T, S, 1, K=K, seed=seed, coverage=cov, omega=omega, u=u)
    return d["meth_control"], d["tot_control"], mu, sgm


def _uniform_P(K):
    P = np.full((K, K), 1.0 / (K - 1))
    np.fill_diagonal(P, 0.0)
    return P


CASES = [
    # K, T, S, coverage, data seed, N_max, epsilon, u, seed
    (6, 3000, 2, 12.0, 1, 250, 0.01, 3, 0),    # pipeline configuration
    (6, 2000, 4, 40.0, 2, 250, 0.01, 3, 1),    # C2 sample count
    (3, 1500, 3, 8.0, 3, 20, 1e-4, 2, 2),      # small N_max: resampling dominated
    (2, 1200, 2, 15.0, 4, 250, 0.01, 1, 3),    # K = 2, u = 1
    (4, 800, 1, 5.0, 5, 64, 1e-3, 5, 4),       # low coverage, u = 5
    (16, 400, 2, 30.0, 6, 250, 0.01, 3, 5),    # K = 16 (largest)
    (6, 500, 2, 10.0, 7, 250, 1e-12, 3, 6),    # epsilon ~ 0: hundreds of pending times
    (6, 1, 2, 10.0, 8, 250, 0.01, 3, 7),       # one site
    (6, 45, 2, 10.0, 9, 250, 0.01, 3, 8),      # shorter than the first cap at N_max
    (5, 700, 2, 20.0, 10, 7, 0.01, 3, 9),      # N_max = K + 2: M = 2
]


@pytest.mark.parametrize("K,T,S,cov,dseed,Nmax,eps,u,seed", CASES)
def test_chain_bit_exact(lib, sg, K, T, S, cov, dseed, Nmax, eps, u, seed):
    meth, tot, mu, sgm = _data(K, T, S, cov, dseed, u=u)
    omega = sg.DEFAULT_OMEGA if K == 6 else [0.93] * K
    p = sg.make_params(K=K, mu=mu, sigma=sgm, P=_uniform_P(K), omega=omega, u=u, Nmax=Nmax, epsilon=eps)
    E = sg.emission(p, meth, tot)
    ref = sg.chain(p, E, seed=seed, chain_id=(3 << 32) | seed)
    assert ref["status"] == 0
    m = Model(lib, p, max(int(tot.max()), 1), T + 10)
    try:
        rc, out = m.chain_host(meth, tot, seed, (3 << 32) | seed)
        assert rc == 0, lib.hyg_last_error()
    finally:
        m.close()
    bad = np.argwhere(out != ref["regime_probs"])
    assert bad.size == 0, (bad[:5], out[tuple(bad[0])], ref["regime_probs"][tuple(bad[0])])


@pytest.mark.parametrize("drop", [40, 52])
def test_packed_sort_collisions_resort_exactly(lib, sg, drop):
    """The chain's log-weight sort orders one word per particle: the order key's
    top bits and the index. Keys that agree on those bits but not below them
    are caught (the keep-top path checks every adjacent pair with the full keys
    and re-sorts exactly; the optimal branch re-checks the order against w).
    With `drop` low bits dropped instead of 8 (hyg_sg_force_key_drop; 52 keeps
    only the sign and exponent) keys collide on most steps, so both checks
    carry the order, and every chain stays bit-exact."""
    for K, T, S, cov, dseed, Nmax, eps, u, seed in (CASES[0], CASES[1], CASES[2], CASES[9]):
        meth, tot, mu, sgm = _data(K, T, S, cov, dseed, u=u)
        omega = sg.DEFAULT_OMEGA if K == 6 else [0.93] * K
        p = sg.make_params(K=K, mu=mu, sigma=sgm, P=_uniform_P(K), omega=omega, u=u, Nmax=Nmax, epsilon=eps)
        ref = sg.chain(p, sg.emission(p, meth, tot), seed=seed, chain_id=(3 << 32) | seed)
        assert ref["status"] == 0
        m = Model(lib, p, max(int(tot.max()), 1), T + 10)
        assert lib.hyg_sg_force_key_drop(drop) == 0
        try:
            rc, out = m.chain_host(meth, tot, seed, (3 << 32) | seed)
            assert rc == 0, lib.hyg_last_error()
        finally:
            lib.hyg_sg_force_key_drop(0)
            m.close()
        bad = np.argwhere(out != ref["regime_probs"])
        assert bad.size == 0, (K, T, bad[:5])
    assert lib.hyg_sg_force_key_drop(7) != 0 and lib.hyg_sg_force_key_drop(61) != 0


def test_golden_fixtures(lib, sg):
    for name in ("sg_chain_k6", "sg_chain_k3"):
        g = np.load(os.path.join(GOLDEN, name + ".npz"))
        K = int(g["K"])
        p = sg.make_params(K=K, mu=g["mu"], sigma=g["sigma"], P=g["P"], omega=g["omega"], u=int(g["u"]),
                           Nmax=int(g["Nmax"]), epsilon=float(g["epsilon"]))
        m = Model(lib, p, 1023, g["tot"].shape[0])
        try:
            rc, out = m.chain_host(g["meth"], g["tot"], int(g["seed"]), int(g["chain_id"]))
            assert rc == 0, lib.hyg_last_error()
        finally:
            m.close()
        assert np.array_equal(out, g["regime_probs"]), name


def test_emission_bit_exact_on_device(lib, sg):
    from hygeia_amd import _lib

    rng = np.random.default_rng(4)
    T, S = 100_000, 3
    tot = rng.integers(0, 400, size=(T, S)).astype(np.uint16)
    meth = (rng.integers(0, 401, size=(T, S)) % (tot.astype(np.int64) + 1)).astype(np.uint16)
    meth[17, 1] = tot[17, 1] + 1  # y > n: the row is -inf
    p = sg.make_params(K=6)
    ref = sg.emission(p, meth, tot)
    m = Model(lib, p, 400, 10)
    try:
        dm = torch.from_numpy(meth.view(np.int16)).cuda()
        dt = torch.from_numpy(tot.view(np.int16)).cuda()
        E = torch.empty((T, 6), dtype=torch.float64, device="cuda")
        _lib.check(lib.hyg_sg_emission(m.h, dm.data_ptr(), dt.data_ptr(), S, T, E.data_ptr(),
                                       C.c_void_p(torch.cuda.current_stream().cuda_stream)))
        out = E.cpu().numpy()
    finally:
        m.close()
    assert np.all(out[17] == -np.inf)
    assert np.array_equal(out, ref)


def test_batched_chains_bit_exact(lib, sg):
    """Many chains of different lengths in one launch (one workgroup each), as
    the per-chromosome driver runs them; each equals its own oracle chain."""
    from hygeia_amd import _lib

    K, S = 6, 2
    lens = [1, 37, 900, 2500, 1200, 3, 640, 2000, 1500, 77]
    total = sum(lens)
    meth, tot, mu, sgm = _data(K, total, S, 15.0, 30)
    p = sg.make_params(K=K)
    m = Model(lib, p, int(tot.max()), max(lens))
    try:
        arr = (_lib.SgChain * len(lens))()
        begins = np.concatenate([[0], np.cumsum(lens)[:-1]])
        for i, (b, n) in enumerate(zip(begins, lens)):
            arr[i].site_begin, arr[i].n_sites = int(b), int(n)
            arr[i].seed, arr[i].chain_id, arr[i].out_begin = 11, (i << 32) | 7, int(b)
        dm = torch.from_numpy(meth.view(np.int16)).cuda()
        dt = torch.from_numpy(tot.view(np.int16)).cuda()
        E = torch.empty((total, K), dtype=torch.float64, device="cuda")
        stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        _lib.check(lib.hyg_sg_emission(m.h, dm.data_ptr(), dt.data_ptr(), S, total, E.data_ptr(), stream))
        wsb = lib.hyg_sg_workspace_bytes(m.h, len(lens), 1024)
        ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
        probs = torch.full((total, K), float("nan"), dtype=torch.float64, device="cuda")
        st = torch.full((len(lens),), 99, dtype=torch.int32, device="cuda")
        _lib.check(lib.hyg_sg_run_chains(m.h, arr, len(lens), E.data_ptr(), ws.data_ptr(), wsb, 1024,
                                         probs.data_ptr(), st.data_ptr(), stream))
        torch.cuda.synchronize()
        out, status = probs.cpu().numpy(), st.cpu().numpy()
    finally:
        m.close()
    assert np.all(status == 0)
    Eh = sg.emission(p, meth, tot)
    for i, (b, n) in enumerate(zip(begins, lens)):
        ref = sg.chain(p, Eh[b:b + n], seed=11, chain_id=(i << 32) | 7)
        assert np.array_equal(out[b:b + n], ref["regime_probs"]), i


def test_pending_capacity_exceeded_reports_enomem(lib, sg):
    from hygeia_amd import _lib

    K, T = 3, 300
    meth, tot, mu, sgm = _data(K, T, 1, 2.0, 40)
    p = sg.make_params(K=K, mu=mu, sigma=sgm, P=_uniform_P(K), omega=[0.95] * 3, epsilon=1e-300)
    m = Model(lib, p, int(tot.max()), T)
    try:
        arr = (_lib.SgChain * 1)()
        arr[0].site_begin, arr[0].n_sites, arr[0].seed, arr[0].chain_id, arr[0].out_begin = 0, T, 1, 1, 0
        E = torch.from_numpy(sg.emission(p, meth, tot)).cuda()
        wsb = lib.hyg_sg_workspace_bytes(m.h, 1, 16)
        ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
        probs = torch.empty((T, K), dtype=torch.float64, device="cuda")
        st = torch.zeros(1, dtype=torch.int32, device="cuda")
        _lib.check(lib.hyg_sg_run_chains(m.h, arr, 1, E.data_ptr(), ws.data_ptr(), wsb, 16, probs.data_ptr(),
                                         st.data_ptr(), C.c_void_p(torch.cuda.current_stream().cuda_stream)))
        torch.cuda.synchronize()
        assert int(st.item()) == _lib.HYG_ENOMEM
        # too small a workspace is refused before launch
        assert lib.hyg_sg_run_chains(m.h, arr, 1, E.data_ptr(), ws.data_ptr(), wsb - 1, 16, probs.data_ptr(),
                                     st.data_ptr(), None) == _lib.HYG_EINVAL
    finally:
        m.close()


def test_invalid_inputs(lib, sg):
    from hygeia_amd import _lib

    p = sg.make_params(K=6)
    m = Model(lib, p, 50, 100)
    try:
        meth = np.array([[1], [2]], np.uint16)
        tot = np.array([[3], [60]], np.uint16)  # beyond max_total_reads
        rc, _ = m.chain_host(meth, tot, 0, 0)
        assert rc == _lib.HYG_EINVAL
        tot = np.array([[3], [1]], np.uint16)  # y > n at site 1: all weights -inf
        rc, _ = m.chain_host(meth, tot, 0, 0)
        assert rc == _lib.HYG_ENUMERIC
        # y > n at site 0: no finite initial weight. The SMC workgroup must
        # publish the abort at t = 0 (it used to return silently and
        # leave the smoothing workgroup polling for ~25 s, then HYG_EDEVICE)
        import time
        t0 = time.perf_counter()
        rc, _ = m.chain_host(np.array([[4], [1]], np.uint16), np.array([[3], [2]], np.uint16), 0, 0)
        assert rc == _lib.HYG_ENUMERIC
        assert time.perf_counter() - t0 < 5.0
        long = np.zeros((101, 1), np.uint16)  # longer than max_duration
        rc, _ = m.chain_host(long, long, 0, 0)
        assert rc == _lib.HYG_EINVAL
    finally:
        m.close()
