"""GPU: the C4 job's sharded HIP path (BASELINE.json configs[3]; main.nf:46-75,
modules/two_group/4_infer.nf:28) over two torch.distributed ranks on one GPU.

The ranks are fresh processes (tests/c4_rank.py, "gloo": both share the one
GPU of the test box) that each run their LPT shard of a fixed 3-seed job on a
small genome through the code bench.py's SCALE runs execute: the chain kernels,
the per-seed posterior-count kernel (hyg_tg_posterior_counts, atomic-free) and
the all-reduce of the device counts (parallel.gather_counts). Required: the
2-rank counts equal the 1-rank run's (in this process) and the counts of the CPU
oracle's chains summed by torch (parallel.posterior_counts), bit for bit. A
second test runs the same collective through the "nccl" backend (RCCL) on the
box's one GPU."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import c4_rank  # noqa: E402


def _run_ranks(tmp_path, world, backend="gloo"):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tmp_path / f"counts_{backend}_{world}.npz"
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "c4_rank.py"), "--rank", str(r), "--world",
                               str(world), "--port", str(port), "--out", str(out), "--backend", backend], env=env)
             for r in range(world)]
    try:
        rcs = [p.wait(timeout=400) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * world
    return np.load(out)


@pytest.mark.timeout(600)
def test_c4_two_ranks_equal_one_rank_and_oracle(tmp_path):
    got = _run_ranks(tmp_path, 2)
    one, units1, n_chains1, _, excl = c4_rank.rank_counts(0, 1)
    ref, units_ref = c4_rank.oracle_counts()
    assert all(excl) and len(excl) == c4_rank.SEEDS  # one atomic-free gather per seed, as in bench.py
    assert bool(np.all(got["exclusive"]))
    assert int(got["units"]) == units1 == units_ref == c4_rank.SEEDS * c4_rank.N_SITES
    assert int(got["chains"]) == n_chains1
    np.testing.assert_array_equal(got["counts"], one.numpy())
    np.testing.assert_array_equal(got["counts"], ref.numpy())
    # every site once per trajectory of every seed
    assert np.all(got["counts"][:, 1:1 + c4_rank.K].sum(1) == c4_rank.SEEDS * c4_rank.B)


@pytest.mark.last
@pytest.mark.timeout(600)
def test_c4_rccl_collective_one_rank(tmp_path):
    """The product collective (parallel.allreduce_counts on device tensors)
    through the "nccl" backend, i.e. RCCL, on the box's GPU: a one-rank group
    (the test box has one GPU; RCCL puts one rank per GPU), so the sum is the
    rank's own counts, which must equal the in-process run's bit for bit."""
    got = _run_ranks(tmp_path, 1, backend="nccl")
    one, units1, n_chains1, _, _ = c4_rank.rank_counts(0, 1)
    assert str(got["backend"]) == "nccl"
    assert int(got["units"]) == units1 and int(got["chains"]) == n_chains1
    np.testing.assert_array_equal(got["counts"], one.numpy())
