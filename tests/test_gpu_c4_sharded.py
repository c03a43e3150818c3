"""GPU: the C4 job's sharded HIP path (BASELINE.json configs[3]; main.nf:46-75,
modules/two_group/4_infer.nf:28) over two torch.distributed ranks on one GPU.

The ranks are fresh processes (tests/c4_rank.py, "gloo": both share the one
GPU of the test box) that each run their LPT shard of a fixed 3-seed job on a
small genome through the chain kernels and all-reduce the per-site posterior
counts. Required: the 2-rank counts equal the 1-rank run's (in this process)
and the counts of the CPU oracle's chains, bit for bit."""
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


@pytest.mark.timeout(600)
def test_c4_two_ranks_equal_one_rank_and_oracle(tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tmp_path / "counts.npz"
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "c4_rank.py"), "--rank", str(r), "--world", "2",
                               "--port", str(port), "--out", str(out)], env=env) for r in range(2)]
    try:
        rcs = [p.wait(timeout=400) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0]
    got = np.load(out)
    one, units1, n_chains1, _ = c4_rank.rank_counts(0, 1)
    ref, units_ref = c4_rank.oracle_counts()
    assert int(got["units"]) == units1 == units_ref == c4_rank.SEEDS * c4_rank.N_SITES
    assert int(got["chains"]) == n_chains1
    np.testing.assert_array_equal(got["counts"], one.numpy())
    np.testing.assert_array_equal(got["counts"], ref.numpy())
    # every site once per trajectory of every seed
    assert np.all(got["counts"][:, 1:1 + c4_rank.K].sum(1) == c4_rank.SEEDS * c4_rank.B)
