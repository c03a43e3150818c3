"""The device policy of concurrent `hygeia infer` task processes (CPU: the
device count is faked; no HIP call is made).

The reference's Nextflow module starts one task process per (chrom, batch,
seed) (modules/two_group/4_infer.nf:28,42-48), all at once under the local
executor (nextflow.config:17-21), and no task names a device.
parallel.task_device spreads such tasks over a node's GPUs through per-node
slots (hyg_device_slot_acquire), or obeys an executor's device variables.
"""
import multiprocessing as mp
import os
from collections import Counter

import pytest

from hygeia_amd import _lib, parallel


def _task(lock_dir, n_devices, barrier, q):
    from hygeia_amd import _lib, parallel

    L = _lib.load(import_torch=False)
    q.put(parallel.task_device(L, n_devices=n_devices, lock_dir=lock_dir, environ={}))
    barrier.wait(timeout=60)  # every task holds its slot until all have taken one


def _run_tasks(lock_dir, n_tasks, n_devices):
    ctx = mp.get_context("spawn")
    barrier, q = ctx.Barrier(n_tasks), ctx.Queue()
    procs = [ctx.Process(target=_task, args=(lock_dir, n_devices, barrier, q)) for _ in range(n_tasks)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return got


def test_sixteen_concurrent_tasks_land_two_per_device(tmp_path):
    got = _run_tasks(str(tmp_path), 16, 8)
    per_device = Counter(d for d, _ in got)
    assert per_device == Counter({d: 2 for d in range(8)}), per_device
    assert sorted(got) == sorted((d, s) for d in range(8) for s in range(2))


def test_slots_freed_by_exited_tasks(tmp_path):
    """A task's slot is freed when its process ends (the flock dies with it):
    tasks that start after others have finished reuse device 0's first slot."""
    first = sorted(_run_tasks(str(tmp_path), 3, 8))
    second = sorted(_run_tasks(str(tmp_path), 3, 8))
    assert first == second == [(0, 0), (1, 0), (2, 0)]


def test_one_slot_per_process_and_release(tmp_path):
    L = _lib.load(import_torch=False)
    try:
        a = parallel.task_device(L, n_devices=4, lock_dir=str(tmp_path), environ={})
        b = parallel.task_device(L, n_devices=4, lock_dir=str(tmp_path), environ={})
        assert a == b == (0, 0)
        assert os.path.exists(os.path.join(str(tmp_path), "hygeia_amd.gpu0.slot0.lock"))
    finally:
        assert L.hyg_device_slot_release() == 0


@pytest.mark.parametrize("var", parallel.EXECUTOR_DEVICE_VARS)
def test_executor_device_variables_are_obeyed(tmp_path, var):
    L = _lib.load(import_torch=False)
    assert parallel.task_device(L, n_devices=8, lock_dir=str(tmp_path), environ={var: "5"}) == (0, -1)
    assert os.listdir(str(tmp_path)) == []  # no slot taken


def test_single_device_and_unusable_lock_dir(tmp_path):
    L = _lib.load(import_torch=False)
    assert parallel.task_device(L, n_devices=1, lock_dir=str(tmp_path), environ={}) == (0, -1)
    dev, slot = parallel.task_device(L, n_devices=8, lock_dir=str(tmp_path / "missing"), environ={})
    assert slot == -1 and 0 <= dev < 8  # a random device
    import ctypes as C

    d, s = C.c_int32(), C.c_int32()
    assert L.hyg_device_slot_acquire(str(tmp_path).encode(), 0, 4, C.byref(d), C.byref(s)) == _lib.HYG_EINVAL


def test_set_device_without_gpu_fails_loudly():
    L = _lib.load(import_torch=False)
    if L.hyg_device_count() > 0:
        pytest.skip("a GPU is visible")
    assert L.hyg_set_device(0) == _lib.HYG_EDEVICE


def test_nextflow_task_defaults_to_the_shared_work_dir(tmp_path, capsys):
    """Inside a Nextflow task (.command.sh in the working directory
    <workDir>/<xx>/<hash>), the slots go to <workDir>/.hygeia_device_locks,
    which every task of the run shares (and no warning is printed)."""
    L = _lib.load(import_torch=False)
    tasks = [tmp_path / "work" / "ab" / h for h in ("cdef01", "cdef02")]
    for t in tasks:
        t.mkdir(parents=True)
        (t / ".command.sh").write_text("hygeia infer\n")
    try:
        assert parallel.task_device(L, n_devices=4, environ={}, container=True, cwd=str(tasks[0])) == (0, 0)
        assert os.listdir(tmp_path / "work" / ".hygeia_device_locks") == ["hygeia_amd.gpu0.slot0.lock"]
    finally:
        assert L.hyg_device_slot_release() == 0
    assert "warning" not in capsys.readouterr().err
    d, why = parallel.default_lock_dir({"NXF_TASK_WORKDIR": str(tasks[1])}, cwd=str(tmp_path))
    assert why == "nextflow" and d == str(tmp_path / "work" / ".hygeia_device_locks")
    assert parallel.default_lock_dir({}, cwd=str(tmp_path))[1] == "tmp"


def test_container_without_shared_lock_dir_warns(tmp_path, capsys):
    L = _lib.load(import_torch=False)
    try:
        parallel.task_device(L, n_devices=4, environ={}, container=True, cwd=str(tmp_path))
        assert "no shared lock directory" in capsys.readouterr().err
        parallel.task_device(L, n_devices=4, environ={}, container=False, cwd=str(tmp_path))
        assert capsys.readouterr().err == ""
    finally:
        assert L.hyg_device_slot_release() == 0
