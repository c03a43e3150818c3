"""The node chain server (hygeia_amd/serve.py) without a GPU: wire framing,
batching of concurrent requests into one engine call per parameter set, the
task-side discovery rules, and `hygeia infer` writing its result files from a
server's replies (a fake engine stands in for the HIP launch; the GPU test
tests/test_gpu_serve.py runs the real one)."""
import os
import socket
import threading
import time

import numpy as np
import pytest

from hygeia_amd import _lib, serve, two_group


def test_framing_round_trip():
    a, b = socket.socketpair()
    with a, b:
        bufs = [np.arange(7, dtype=np.int16), np.zeros(0, np.uint8), np.linspace(0, 1, 5).astype(np.float32)]
        t = threading.Thread(target=serve.send_msg, args=(a, {"op": "x", "n": 3}, bufs))
        t.start()
        h, got = serve.recv_msg(b)
        t.join()
    assert h["op"] == "x" and h["n"] == 3 and h["sizes"] == [14, 0, 20]
    for x, y in zip(bufs, got):
        assert bytes(y) == x.tobytes()


class FakeEngine:
    """Stands in for the HIP launch: outputs are functions of each request's
    counts, seed and chain id, so a reply that went to the wrong task shows."""

    delay = 0.2
    calls = []

    def __init__(self, device):
        self.device = device

    def start(self):
        pass

    def run(self, reqs):
        time.sleep(self.delay)
        FakeEngine.calls.append(len(reqs))
        for r in reqs:
            h = r.header
            p = _lib.TgParams.from_buffer_copy(bytes.fromhex(h["params"]))
            K, B, T = p.n_regimes, p.num_samples_backward, h["T"]
            tc = np.frombuffer(r.bufs[1], np.uint16).reshape(T, h["s_c"]).astype(np.int64)
            v = (tc.sum(1) + h["seed"] + (h["chain_id"] & 0xFFFF)) % 1000
            merged = np.repeat(v[:, None], B, 1).astype(np.int16)
            ctrl = np.repeat(merged[:, :, None], 2, 2)
            split = (v / 1000.0).astype(np.float32)
            regime = np.repeat(split[:, None], 2 * K, 1)
            r.reply = ({"rc": 0, "log_z": float(v.sum()), "batch": len(reqs), "wait_s": 0.0, "run_s": self.delay},
                       [merged, ctrl, ctrl + 1, split, regime])


@pytest.fixture
def fake_server(tmp_path):
    path = str(tmp_path / "s.sock")
    FakeEngine.calls = []
    srv = serve.Server(path, 1, engine_factory=FakeEngine, idle=30)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    t0 = time.monotonic()
    while not serve.connectable(path):
        assert time.monotonic() - t0 < 10
        time.sleep(0.02)
    yield path, srv
    serve.Client(path).stop()
    th.join(timeout=30)
    assert not th.is_alive() and not os.path.exists(path)


def _req(T, S, seed, K=6, B=5, data_seed=0):
    rng = np.random.default_rng(data_seed)
    tot = rng.integers(0, 60, (T, 2 * S)).astype(np.uint16)
    meth = (tot // 2).astype(np.uint16)
    p = _lib.make_params([0.5] * K, [0.1] * K, two_group.uniform_theta(K), num_samples_backward=B)
    return p, meth[:, :S], tot[:, :S], meth[:, S:], tot[:, S:], seed


def test_concurrent_requests_batch_and_route(fake_server):
    path, srv = fake_server
    c = serve.Client(path)
    n = 8
    reqs = [_req(100 + 13 * i, 3, i, data_seed=i) for i in range(n)]
    out = [None] * n

    def one(i):
        p, mc, tc, mk, tk, sd = reqs[i]
        out[i] = serve.Client(path).run_chain(p, 60, mc, tc, mk, tk, sd, (7 << 32) | i)

    ths = [threading.Thread(target=one, args=(i,)) for i in range(n)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for i, (res, fw, ex) in enumerate(out):
        p, mc, tc, mk, tk, sd = reqs[i]
        v = (tc.astype(np.int64).sum(1) + sd + i) % 1000
        assert fw is None
        np.testing.assert_array_equal(res.particle["merged_state"][:, 0], v)
        np.testing.assert_array_equal(res.particle["case_state"][:, 0, 1], v + 1)
        np.testing.assert_array_equal(ex["split_probs"], (v / 1000.0).astype(np.float32))
        assert ex["regime_probs"].shape == (len(v), 12) and ex["log_z"] == float(v.sum())
    st = c.status()
    assert st["requests"] == n and st["chains"] == n and st["pending"] == 0
    # the first request runs alone; the others arrive while it runs and share launches
    assert sum(FakeEngine.calls) == n and max(FakeEngine.calls) > 1 and len(FakeEngine.calls) < n


def test_parameter_sets_are_not_mixed(fake_server):
    path, _ = fake_server
    a = _req(50, 2, 1, K=6)
    b = _req(50, 2, 2, K=4, B=3)
    outs = {}

    def one(name, r):
        outs[name] = serve.Client(path).run_chain(r[0], 60, *r[1:5], r[5], 1)

    ths = [threading.Thread(target=one, args=x) for x in (("a", a), ("b", b))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert outs["a"][2]["regime_probs"].shape == (50, 12) and outs["b"][2]["regime_probs"].shape == (50, 8)
    assert outs["b"][0].particle["control_state"].shape == (50, 3, 2)


def test_task_client_discovery(fake_server, tmp_path):
    path, _ = fake_server
    env = {"HYGEIA_DEVICE_LOCK_DIR": str(tmp_path)}
    os.symlink(path, str(tmp_path / serve.SOCK_NAME))  # the server answers in the lock directory
    c = serve.task_client(env)
    assert c is not None and c.path == str(tmp_path / serve.SOCK_NAME)
    assert serve.task_client(dict(env, HYGEIA_SERVER="0")) is None
    assert serve.task_client({"HYGEIA_DEVICE_LOCK_DIR": str(tmp_path / "elsewhere")}) is None
    long_dir = "/x" * 60
    assert len(serve.socket_path(long_dir)) < 100 and serve.socket_path(long_dir).startswith("/tmp/")


def test_server_exits_when_idle_or_socket_removed(tmp_path):
    for how in ("idle", "unlink"):
        path = str(tmp_path / f"{how}.sock")
        srv = serve.Server(path, 1, engine_factory=FakeEngine, idle=0.5 if how == "idle" else 0)
        th = threading.Thread(target=srv.serve_forever, daemon=True)
        th.start()
        t0 = time.monotonic()
        while not os.path.exists(path):
            assert time.monotonic() - t0 < 10
            time.sleep(0.02)
        if how == "unlink":
            os.unlink(path)
        th.join(timeout=20)
        assert not th.is_alive()


def test_infer_writes_the_server_replies(fake_server, tmp_path, monkeypatch):
    """`hygeia infer` with a server answering: the task parses its inputs,
    hands the chain over and writes the reply as its result files (no HIP
    library needed in the task)."""
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_cli import _write_inputs

    from hygeia_amd import cli

    path, _ = fake_server
    lockd = tmp_path / "locks"
    lockd.mkdir()
    os.symlink(path, str(lockd / serve.SOCK_NAME))
    monkeypatch.setenv("HYGEIA_DEVICE_LOCK_DIR", str(lockd))
    _write_inputs(str(tmp_path), "3", 900)
    rc = cli.main(["infer", "--chrom", "3", "--batch", "0", "--seed", "2", "--segment_size", "1000",
                   "--num_samples_backward", "5", "--data_dir", str(tmp_path / "data"),
                   "--single_group_dir", str(tmp_path / "sg"), "--results_dir", str(tmp_path / "out")])
    assert rc == 0
    assert cli.LAST_TIMINGS["server_batch"] == 1
    d = tmp_path / "out" / "chrom_3_0"
    merged = np.load(d / "optimal_backward_particles_merged_state_2400_2.npz")["arr_0"]
    assert merged.shape == (900, 5) and merged.dtype == np.int16
    tc = np.loadtxt(tmp_path / "data" / "n_total_reads_control_3.txt.gz", delimiter=",", ndmin=2)
    v = (tc.sum(1).astype(np.int64) + 2 + (cli.chain_id("3", 0) & 0xFFFF)) % 1000
    np.testing.assert_array_equal(merged[:, 0], v)
    assert (d / "log_normalizing_constants_optimal_2.txt").read_text().strip() == str({2400: float(v.sum())})


class FailingEngine(FakeEngine):
    """Chains whose seed is 13 fail as the library would (all weights -inf);
    seed 99 makes the engine itself raise (a server fault)."""

    def run(self, reqs):
        if any(r.header["seed"] == 99 for r in reqs):
            raise RuntimeError("device lost")
        super().run(reqs)
        for r in reqs:
            if r.header["seed"] == 13:
                r.reply = ({"rc": _lib.HYG_ENUMERIC, "error": "all particle weights became -inf"}, [])


def test_chain_errors_and_server_faults(tmp_path):
    """A chain's own failure reaches the task as the library's error (as if it
    had run in-process); a failure of the server reaches it as
    ServerUnavailable, on which `hygeia infer` runs the chain itself; so does a
    connection the server drops."""
    path = str(tmp_path / "f.sock")
    srv = serve.Server(path, 1, engine_factory=FailingEngine, idle=30)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    t0 = time.monotonic()
    while not serve.connectable(path):
        assert time.monotonic() - t0 < 10
        time.sleep(0.02)
    try:
        p, mc, tc, mk, tk, _ = _req(40, 2, 0)
        c = serve.Client(path)
        with pytest.raises(_lib.HygError) as ei:
            c.run_chain(p, 60, mc, tc, mk, tk, 13, 1)
        assert ei.value.code == _lib.HYG_ENUMERIC
        with pytest.raises(serve.ServerUnavailable, match="device lost"):
            c.run_chain(p, 60, mc, tc, mk, tk, 99, 1)
        c.run_chain(p, 60, mc, tc, mk, tk, 1, 1)  # the server still serves
    finally:
        serve.Client(path).stop()
        th.join(timeout=30)
    # a listener that drops every connection
    dead = str(tmp_path / "d.sock")
    ls = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    ls.bind(dead)
    ls.listen(4)

    def drop():
        for _ in range(2):
            conn, _ = ls.accept()
            conn.close()

    dt = threading.Thread(target=drop, daemon=True)
    dt.start()
    try:
        assert not serve.connectable(dead)
        with pytest.raises(serve.ServerUnavailable):
            serve.Client(dead).run_chain(p, 60, mc, tc, mk, tk, 1, 1)
    finally:
        dt.join(timeout=10)
        ls.close()
