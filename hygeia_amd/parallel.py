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


def allreduce_counts(counts, always: bool = False):
    """Sum of the per-site counts over all ranks (in place); a no-op without an
    initialised process group, and at world size 1 unless `always` (which runs
    the collective anyway, e.g. to exercise RCCL on a one-GPU box)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and (always or dist.get_world_size() > 1):
        dist.all_reduce(counts, op=dist.ReduceOp.SUM)
    return counts
