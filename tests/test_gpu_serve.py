"""GPU: the node chain server (`hygeia serve`, hygeia_amd/serve.py) behind
unchanged `hygeia infer` task processes (modules/two_group/4_infer.nf:42-48).

The server runs as a child process of the test; six task processes start at
once and hand their chains over; the server's gather window puts them into
one launch. Required: every result file equals the file of the same task run
stand-alone in this process (HYGEIA_SERVER=0), and the server ran the six
chains in fewer launches than chains."""
import gzip
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _compare_dirs(one, other):
    assert sorted(p.name for p in one.iterdir()) == sorted(p.name for p in other.iterdir())
    for d in one.iterdir():
        names = sorted(p.name for p in d.iterdir())
        assert names == sorted(p.name for p in (other / d.name).iterdir())
        for nm in names:
            a, b = d / nm, other / d.name / nm
            if nm.startswith("optimal_time_"):
                continue  # wall times
            if nm.endswith(".npz"):
                np.testing.assert_array_equal(np.load(a)["arr_0"], np.load(b)["arr_0"], err_msg=nm)
            elif nm.endswith(".gz"):
                assert gzip.open(a).read() == gzip.open(b).read(), nm
            else:  # the flags files name their own --results_dir
                assert a.read_text().replace(str(one), "R") == b.read_text().replace(str(other), "R"), nm


@pytest.mark.timeout(600)
def test_tasks_through_the_server_equal_stand_alone_tasks(tmp_path, monkeypatch):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_cli import _write_inputs

    from hygeia_amd import _lib, cli, serve

    if _lib.load().hyg_device_count() < 1:
        pytest.fail("no HIP device visible")
    _write_inputs(str(tmp_path), "7", 7000, S=3)
    common = ["--chrom", "7", "--segment_size", "2000", "--buffer_size", "100", "--data_dir", str(tmp_path / "data"),
              "--single_group_dir", str(tmp_path / "sg")]
    tasks = [(b, sd) for b in range(3) for sd in (0, 5)]  # 1 + 7000 // 2000 = 4 segments; 3 of them x 2 seeds
    lockd = tmp_path / "locks"
    lockd.mkdir()
    path = serve.socket_path(str(lockd))
    env = dict(os.environ, PYTHONPATH=ROOT, HYGEIA_DEVICE_LOCK_DIR=str(lockd))
    env.pop("HYGEIA_SERVER", None)
    log = open(tmp_path / "serve.log", "w")
    srv = subprocess.Popen([sys.executable, "-m", "hygeia_amd.serve", "--socket", path, "--idle", "300",
                            "--gather", "8"], env=env, stdout=log, stderr=log, cwd=ROOT)
    try:
        t0 = time.monotonic()
        while not serve.connectable(path):
            assert srv.poll() is None, (tmp_path / "serve.log").read_text()
            assert time.monotonic() - t0 < 120, "the server did not start"
            time.sleep(0.1)
        procs = [subprocess.Popen([sys.executable, "-m", "hygeia_amd.cli", "infer", "--batch", str(b), "--seed",
                                   str(sd), "--results_dir", str(tmp_path / "srv")] + common, env=env, cwd=ROOT,
                                  stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
                 for b, sd in tasks]
        errs = [p.communicate(timeout=300)[1] for p in procs]
        assert [p.returncode for p in procs] == [0] * len(tasks), [e[-800:] for e in errs]
        assert not any(b"unavailable" in e for e in errs), [e[-800:] for e in errs]  # no task ran its own chain
        st = serve.Client(path).status()
        assert st["chains"] == len(tasks) and st["batches"] < len(tasks), st
        serve.Client(path).stop()
        assert srv.wait(timeout=120) == 0
    finally:
        if srv.poll() is None:
            srv.kill()
            srv.wait()
        log.close()
    print(json.dumps(st))
    monkeypatch.setenv("HYGEIA_SERVER", "0")
    for b, sd in tasks:
        assert cli.main(["infer", "--batch", str(b), "--seed", str(sd), "--results_dir", str(tmp_path / "one")]
                        + common) == 0
    _compare_dirs(tmp_path / "one", tmp_path / "srv")
