"""Multi-GPU driver pieces: chain sharding and the final posterior reduction.

The reference fans out one process per (chromosome, segment, seed)
(main.nf:46-75, modules/two_group/4_infer.nf:28) and aggregates the per-site
posteriors afterwards (aggregate_results.py:71-206: means over trajectories and
seeds). Here one process per GPU runs a shard of those chains in one launch
(longest-processing-time-first over ranks, no data-path communication), then
one collective sums the per-site posterior counts over ranks:

    counts[site] = [#trajectories split, #(r_ctrl = r) for r < K, #(r_case = r) for r < K]

summed over all seeds' B trajectories: int32 [n_sites][1 + 2K]. With
torch.distributed over RCCL ("nccl") on MI355X this is an all-reduce over xGMI;
the CPU tests drive the same code with "gloo".
"""
from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import numpy as np

Chain = Tuple[int, int, int, int, int]  # (site_begin, n_sites, seed, chain_id, out_begin)


def shard_chains(lengths: Sequence[int], world: int) -> List[List[int]]:
    """LPT assignment of chain indices to `world` ranks: longest chain first to
    the least-loaded rank (ties to the lowest rank). Deterministic."""
    order = sorted(range(len(lengths)), key=lambda i: (-int(lengths[i]), i))
    load = [0] * world
    out: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        out[r].append(i)
        load[r] += int(lengths[i])
    return out


def trimmed_rows(segments) -> Tuple[np.ndarray, np.ndarray]:
    """For synthetic.segment_chains rows (chrom, batch, site_begin, n, r0, rlen):
    (row offset inside each chain's output, global site index) of every returned
    site, in chain order; used to scatter a chain's outputs into the genome."""
    src, dst = [], []
    for (_, _, s0, _, r0, rl) in segments:
        src.append(np.arange(r0, r0 + rl, dtype=np.int64))
        dst.append(np.arange(s0 + r0, s0 + r0 + rl, dtype=np.int64))
    return np.concatenate(src), np.concatenate(dst)


def posterior_counts(split_probs, regime_probs, B: int, rows_out, rows_site, n_sites: int, counts=None):
    """Adds one run's posterior counts into counts [n_sites][1+2K] int32 (torch
    tensors, any device): split/regime probabilities are means over the B
    trajectories, so probs * B are exact integers."""
    import torch

    K2 = regime_probs.shape[1]
    if counts is None:
        counts = torch.zeros((n_sites, 1 + K2), dtype=torch.int32, device=regime_probs.device)
    sp = torch.round(split_probs[rows_out].to(torch.float64) * B).to(torch.int32)
    rp = torch.round(regime_probs[rows_out].to(torch.float64) * B).to(torch.int32)
    counts.index_add_(0, rows_site, torch.cat([sp[:, None], rp], dim=1))
    return counts


def posterior_counts_device(L, split_probs, regime_probs, B: int, segments, max_rows: int, counts, stream=0,
                            exclusive: bool = False):
    """The same sum as posterior_counts on the device, in one HIP kernel
    (hyg_tg_posterior_counts): segments is an int64 device tensor [n][3] of
    (output row, site, rows) per chain, as segment_table builds it; exclusive:
    the caller guarantees the segments cover disjoint sites (one seed's chains),
    so no atomics. Asynchronous on `stream` (a HIP stream handle; 0 = the null
    stream)."""
    from . import _lib

    K = regime_probs.shape[1] // 2
    _lib.check(L.hyg_tg_posterior_counts(split_probs.data_ptr(), regime_probs.data_ptr(), K, B,
                                         segments.data_ptr(), int(segments.shape[0]), int(max_rows),
                                         1 if exclusive else 0, counts.data_ptr(), stream))
    return counts


def seed_tables(chains, seg_of) -> List[np.ndarray]:
    """segment_table of each seed's chains (each covers disjoint sites), in seed
    order."""
    seeds = sorted({c[2] for c in chains})
    return [segment_table([c for c in chains if c[2] == sd], seg_of) for sd in seeds]


def disjoint_sites(table: np.ndarray) -> bool:
    """True when the (output row, site, rows) entries of a segment table cover
    pairwise disjoint site ranges, which the kernel's exclusive (atomic-free)
    mode needs."""
    if len(table) < 2:
        return True
    t = table[np.argsort(table[:, 1], kind="stable")]
    return bool(np.all(t[:-1, 1] + t[:-1, 2] <= t[1:, 1]))


def gather_tables(chains, seg_of, device) -> List[Tuple[object, int, bool]]:
    """The job's gather plan for one launch's chains: per seed, the segment
    table on `device` (int64 tensor), its longest row count and whether the
    atomic-free mode applies (the seed's trimmed rows are disjoint; a table
    whose rows overlap is summed with atomics instead of losing counts)."""
    import torch

    out = []
    for t in seed_tables(chains, seg_of):
        out.append((torch.from_numpy(t).to(device), int(t[:, 2].max()), disjoint_sites(t)))
    return out


def gather_counts(L, parts, B: int, counts, stream=0, always: bool = False):
    """The job's final gather (aggregate_results.py:71-206) as bench.py runs it:
    zero counts, add every launch's posterior counts with hyg_tg_posterior_counts
    (one kernel per seed table), then sum over the ranks (allreduce_counts).
    parts = [(split_probs, regime_probs, gather_tables(...)), ...] per launch;
    the torch work runs on torch's current stream, which the caller sets to
    `stream`. always: run the collective at world size 1 too (allreduce_counts)."""
    counts.zero_()
    for split, regime, tabs in parts:
        for tab, max_rows, exclusive in tabs:
            posterior_counts_device(L, split, regime, B, tab, max_rows, counts, stream, exclusive=exclusive)
    return allreduce_counts(counts, always=always)


def segment_table(chains, seg_of) -> np.ndarray:
    """int64 [n][3] (output row, site, rows) of the trimmed rows of each chain
    (site_begin, n_sites, seed, chain_id, out_begin); seg_of maps a chain id to
    its segment's (site_begin, trim offset, trimmed rows)."""
    t = np.empty((len(chains), 3), np.int64)
    for i, c in enumerate(chains):
        s0, r0, rl = seg_of[c[3]]
        t[i] = (c[4] + r0, s0 + r0, rl)
    return t


def allreduce_counts(counts, always: bool = False):
    """Sum of the per-site counts over all ranks (in place); a no-op without an
    initialised process group, and at world size 1 unless `always` (which runs
    the collective anyway, e.g. to exercise RCCL on a one-GPU box)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and (always or dist.get_world_size() > 1):
        dist.all_reduce(counts, op=dist.ReduceOp.SUM)
    return counts


# Environment variables through which an executor assigns GPUs to a task; when
# any is set the HIP runtime shows the task only its devices and the task uses
# the first of them.
EXECUTOR_DEVICE_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")
LOCK_DIR_VAR = "HYGEIA_DEVICE_LOCK_DIR"
MAX_SLOTS_PER_DEVICE = 1024


def in_container(root: str = "/") -> bool:
    """True inside a docker / podman container (the reference pipeline runs
    every task in one, nextflow.config:31-34)."""
    return any(os.path.exists(os.path.join(root, f)) for f in (".dockerenv", "run/.containerenv"))


def default_lock_dir(environ=None, cwd: str = None) -> Tuple[str, str]:
    """(directory, why) for the device slot locks when $HYGEIA_DEVICE_LOCK_DIR
    is unset. A Nextflow task runs in <workDir>/<xx>/<hash> (its .command.sh
    there); the pipeline's workDir is the one directory every task of the run
    shares (Nextflow mounts it into each task container), so the slots go to
    <workDir>/.hygeia_device_locks. Elsewhere: the temp directory, which is
    private to a container."""
    import tempfile

    env = os.environ if environ is None else environ
    cwd = cwd or os.getcwd()
    task_dir = env.get("NXF_TASK_WORKDIR") or (cwd if os.path.exists(os.path.join(cwd, ".command.sh")) else None)
    if task_dir:
        work = os.path.dirname(os.path.dirname(os.path.abspath(task_dir)))
        d = os.path.join(work, ".hygeia_device_locks")
        try:
            os.makedirs(d, exist_ok=True)
            if os.access(d, os.W_OK):
                return d, "nextflow"
        except OSError:
            pass
    return tempfile.gettempdir(), "tmp"


def task_device(L, n_devices: int = None, lock_dir: str = None, environ=None, container: bool = None,
                cwd: str = None) -> Tuple[int, int]:
    """The device of one `hygeia infer` task process: (device, slot).

    The reference's Nextflow module starts one task process per (chrom, batch,
    seed) (modules/two_group/4_infer.nf:28,42-48), concurrently under the local
    executor (nextflow.config:17-21), and a task names no device. Policy:

    - an executor that assigns devices (HIP_VISIBLE_DEVICES,
      ROCR_VISIBLE_DEVICES or CUDA_VISIBLE_DEVICES set) is obeyed: the task
      sees only those devices and takes the first (slot -1: no lock);
    - otherwise, with more than one device, the task takes a per-node slot
      (hyg_device_slot_acquire: an exclusive flock in a directory every
      concurrent task shares: $HYGEIA_DEVICE_LOCK_DIR, else the Nextflow run's
      workDir inside a Nextflow task, else the temp directory), the first free
      one in the order slot 0 of every device, slot 1 of every device, ...: N
      concurrent tasks spread N / n_devices per device, and a task that ends
      (or dies) frees its slot for the next;
    - the temp directory of a container is private to it, so a task in a
      container that falls back to it warns on stderr; and when no lock can be
      taken at all the device is drawn at random (os.urandom), not from the
      process id, which is the same small number in every container's PID
      namespace;
    - with one device (or none), device 0.

    n_devices / lock_dir / environ / container / cwd default to the live
    values; tests pass fake ones. Selecting the device (hyg_set_device) is the
    caller's."""
    import ctypes as C
    import sys

    env = os.environ if environ is None else environ
    if any(env.get(v, "").strip() for v in EXECUTOR_DEVICE_VARS):
        return 0, -1
    n = int(L.hyg_device_count()) if n_devices is None else int(n_devices)
    if n <= 1:
        return 0, -1
    d = lock_dir or env.get(LOCK_DIR_VAR)
    if not d:
        d, why = default_lock_dir(env, cwd)
        if why == "tmp" and (in_container() if container is None else container):
            print(f"hygeia: warning: {n} GPUs but no shared lock directory: the device slots in {d} are private to "
                  f"this container, so concurrent tasks may share one GPU; set {LOCK_DIR_VAR} to a host directory "
                  "mounted into every task container", file=sys.stderr)
    dev, slot = C.c_int32(-1), C.c_int32(-1)
    rc = L.hyg_device_slot_acquire(d.encode(), n, MAX_SLOTS_PER_DEVICE, C.byref(dev), C.byref(slot))
    if rc != 0:  # no usable lock directory: a random device, not the (namespaced) process id
        return int.from_bytes(os.urandom(4), "little") % n, -1
    return int(dev.value), int(slot.value)
