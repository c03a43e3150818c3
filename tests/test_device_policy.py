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
    assert slot == -1 and 0 <= dev < 8  # spread by process id
    import ctypes as C

    d, s = C.c_int32(), C.c_int32()
    assert L.hyg_device_slot_acquire(str(tmp_path).encode(), 0, 4, C.byref(d), C.byref(s)) == _lib.HYG_EINVAL


def test_set_device_without_gpu_fails_loudly():
    L = _lib.load(import_torch=False)
    if L.hyg_device_count() > 0:
        pytest.skip("a GPU is visible")
    assert L.hyg_set_device(0) == _lib.HYG_EDEVICE
