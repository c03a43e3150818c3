"""Multi-rank driver logic on CPU: LPT sharding and the final posterior-count
reduction over torch.distributed ("gloo", world size 2). The per-chain outputs
come from the CPU oracle here (test infrastructure); on MI355X the same code
runs over RCCL with the HIP outputs.
"""
import os
import socket

import numpy as np
import pytest

from hygeia_amd import parallel, synthetic


def test_shard_chains_lpt_balanced_and_complete():
    rng = np.random.default_rng(0)
    lengths = list(rng.integers(1000, 110000, size=291)) * 2
    for world in (1, 2, 4, 8):
        sh = parallel.shard_chains(lengths, world)
        flat = sorted(i for s in sh for i in s)
        assert flat == list(range(len(lengths)))
        loads = [sum(lengths[i] for i in s) for s in sh]
        assert max(loads) - min(loads) <= max(lengths)
    assert parallel.shard_chains([5, 3, 3, 1], 2) == [[0, 3], [1, 2]]


def test_trimmed_rows_cover_genome_once():
    sizes = synthetic.chromosome_sizes(123457, n_chrom=3)
    segs = synthetic.segment_chains(sizes, 10000, 500)
    src, dst = parallel.trimmed_rows(segs)
    assert np.array_equal(np.sort(dst), np.arange(123457))
    assert np.all(src >= 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_rank(rank, world, port, outq):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = _shard_counts(rank, world)
        parallel.allreduce_counts(res)
        if rank == 0:
            outq.put(res.numpy())
    finally:
        dist.destroy_process_group()


def _problem():
    from oracle import binding as ob

    K, M, B = 4, 8, 5
    sizes = synthetic.chromosome_sizes(2400, n_chrom=2)
    segs = synthetic.segment_chains(sizes, 500, 40)
    d = synthetic.simulate(2400, 2, 2, K=K, seed=3, coverage=30.0)
    mu, sg = synthetic.regime_params(K)
    p = ob.make_params(K=K, M=M, B=B, mu=mu, sigma=sg)
    chains = [(si, seed) for seed in (0, 1) for si in range(len(segs))]
    return ob, p, d, segs, chains, K, B


def _chain_counts(ob, p, d, seg, seed, K, B, counts):
    import torch

    (ci, b, s0, n, r0, rl) = seg
    sl = slice(s0, s0 + n)
    E = ob.emission(p, d["meth_control"][sl], d["tot_control"][sl], d["meth_case"][sl], d["tot_case"][sl])
    out = ob.chain(p, E, seed, (ci << 32) | b)
    src, dst = parallel.trimmed_rows([seg])
    return parallel.posterior_counts(torch.from_numpy(out["split_probs"]), torch.from_numpy(out["regime_probs"]),
                                     B, torch.from_numpy(src), torch.from_numpy(dst), 2400, counts)


def _shard_counts(rank, world):
    import torch

    ob, p, d, segs, chains, K, B = _problem()
    mine = parallel.shard_chains([segs[si][3] for si, _ in chains], world)[rank]
    counts = torch.zeros((2400, 1 + 2 * K), dtype=torch.int32)
    for i in mine:
        si, seed = chains[i]
        counts = _chain_counts(ob, p, d, segs[si], seed, K, B, counts)
    return counts


def test_two_rank_reduce_equals_single_process(oracle):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run_rank, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    got = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    want = _shard_counts(0, 1).numpy()
    np.testing.assert_array_equal(got, want)
    K, B = 4, 5
    # two seeds x B trajectories per site, every site counted once per trajectory
    assert np.all(got[:, 1:1 + K].sum(1) == 2 * B)
    assert np.all(got[:, 1 + K:].sum(1) == 2 * B)


def test_segment_table_matches_row_lists():
    """parallel.segment_table (the device gather's chain table) expands to the
    (output row, site) pairs the torch reference's index lists hold."""
    from hygeia_amd import synthetic

    segs = synthetic.segment_chains(synthetic.chromosome_sizes(900_000))
    seg_of = {(ci << 32) | b: (s0, r0, rl) for (ci, b, s0, n, r0, rl) in segs}
    chains, out = [], 0
    for sd in (0, 1):
        for (ci, b, s0, n, r0, rl) in segs:
            chains.append((s0, n, sd, (ci << 32) | b, out))
            out += n
    tab = parallel.segment_table(chains, seg_of)
    src = np.concatenate([np.arange(c[4] + seg_of[c[3]][1], c[4] + seg_of[c[3]][1] + seg_of[c[3]][2]) for c in chains])
    dst = np.concatenate([np.arange(seg_of[c[3]][0] + seg_of[c[3]][1], seg_of[c[3]][0] + seg_of[c[3]][1]
                                    + seg_of[c[3]][2]) for c in chains])
    np.testing.assert_array_equal(np.concatenate([np.arange(a, a + n) for a, _, n in tab]), src)
    np.testing.assert_array_equal(np.concatenate([np.arange(s, s + n) for _, s, n in tab]), dst)
    # every site once per seed
    assert np.bincount(dst, minlength=900_000).tolist() == [2] * 900_000


def test_gather_plan_is_exclusive_only_for_disjoint_seeds():
    """parallel.disjoint_sites decides the gather kernel's atomic-free mode: a
    seed's segments tile the genome without overlap (bench.py's plan), while a
    table whose trimmed rows overlap is summed with atomics."""
    from hygeia_amd import synthetic

    segs = synthetic.segment_chains(synthetic.chromosome_sizes(900_000))
    seg_of = {(ci << 32) | b: (s0, r0, rl) for (ci, b, s0, n, r0, rl) in segs}
    chains = [(s0, n, sd, (ci << 32) | b, 0) for sd in (0, 1) for (ci, b, s0, n, r0, rl) in segs]
    tabs = parallel.seed_tables(chains, seg_of)
    assert len(tabs) == 2 and all(parallel.disjoint_sites(t) for t in tabs)
    assert not parallel.disjoint_sites(parallel.segment_table(chains, seg_of))  # both seeds: every site twice
    t = np.array([[0, 100, 50], [50, 10, 40], [90, 149, 3]], np.int64)  # unsorted, [149, 152) meets [100, 150)
    assert not parallel.disjoint_sites(t)
    t[2, 1] = 150
    assert parallel.disjoint_sites(t) and parallel.disjoint_sites(t[:1]) and parallel.disjoint_sites(t[:0])
