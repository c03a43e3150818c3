"""bench.py's host-side logic on CPU: the chain lists of the c3 and c4 jobs
(fixed jobs, LPT-sharded over the ranks), the host-core accounting of the CPU baseline, and
the c4 job end to end over torch.distributed ("gloo", world size 2) with the
oracle standing in for the GPU chains (test infrastructure)."""
import argparse
import os
import socket

import numpy as np

import bench
from hygeia_amd import parallel, synthetic


def _args(job, **kw):
    a = argparse.Namespace(job=job, seeds=2, total_seeds=8)
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def test_c3_strong_chains_cover_the_fixed_job_once():
    """at N > 1 GPUs the c3 job is the metric's fixed 2-seed job
    (582 chains at 28M sites), split over the ranks, not 2 seeds per rank."""
    segs = synthetic.segment_chains(synthetic.chromosome_sizes(1_000_000))
    job = {((ci << 32) | b, sd) for sd in range(2) for (ci, b, *_r) in segs}
    for world in (1, 2, 4, 8):
        got, units_total = [], 0
        for rank in range(world):
            chains, n_out, units, picked = bench.build_chains(_args("c3"), segs, rank, world)
            got += [(c[3], c[2]) for c in chains]
            units_total += units
            assert n_out == sum(c[1] for c in chains)
        assert sorted(got) == sorted(job) and len(got) == len(job)
        assert units_total == 2 * sum(s[5] for s in segs)


def test_c4_strong_chains_cover_the_job_once():
    segs = synthetic.segment_chains(synthetic.chromosome_sizes(3_000_000))
    job = {(cid, sd) for sd in range(8) for (ci, b, *_r) in segs for cid in [(ci << 32) | b]}
    for world in (1, 2, 4, 8):
        got, units_total, loads = [], 0, []
        for rank in range(world):
            chains, n_out, units, _ = bench.build_chains(_args("c4"), segs, rank, world)
            got += [(c[3], c[2]) for c in chains]
            units_total += units
            loads.append(sum(c[1] for c in chains))
            outs = sorted(c[4] for c in chains)  # disjoint output rows
            assert outs[0] == 0 and len(set(outs)) == len(outs)
        assert sorted(got) == sorted(job) and len(got) == len(job)
        assert units_total == 8 * sum(s[5] for s in segs)
        assert max(loads) - min(loads) <= max(s[3] for s in segs)  # LPT balance


def test_host_cpus_accounting():
    h = bench.host_cpus()
    assert 1 <= h["usable"] <= h["affinity"] <= h["nproc"]
    old = os.environ.get("OMP_NUM_THREADS")
    os.environ["OMP_NUM_THREADS"] = "1"
    try:
        assert bench.host_cpus()["usable"] == 1
    finally:
        if old is None:
            del os.environ["OMP_NUM_THREADS"]
        else:
            os.environ["OMP_NUM_THREADS"] = old


# ---------------------------------------------- c4 end to end over gloo
N_SITES, K, M, B = 3000, 4, 8, 5


def _problem():
    from oracle import binding as ob

    segs = synthetic.segment_chains(synthetic.chromosome_sizes(N_SITES, n_chrom=3), 600, 40)
    d = synthetic.simulate(N_SITES, 2, 2, K=K, seed=4, coverage=30.0)
    mu, sg = synthetic.regime_params(K)
    p = ob.make_params(K=K, M=M, B=B, mu=mu, sigma=sg)
    E = ob.emission(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
    return ob, p, E, segs


def _rank_counts(rank, world):
    """bench.py's c4 path on one rank: its LPT shard of the fixed 8-seed job,
    each chain's posterior counts scattered into the genome."""
    import torch

    ob, p, E, segs = _problem()
    chains, n_out, units, _ = bench.build_chains(_args("c4", total_seeds=3), segs, rank, world)
    seg_of = {(ci << 32) | b: (s0, r0, rl) for (ci, b, s0, n, r0, rl) in segs}
    split = torch.zeros(n_out, dtype=torch.float32)
    regime = torch.zeros((n_out, 2 * K), dtype=torch.float32)
    for (s0, n, sd, cid, o) in chains:
        out = ob.chain(p, E[s0:s0 + n], sd, cid)
        split[o:o + n] = torch.from_numpy(out["split_probs"])
        regime[o:o + n] = torch.from_numpy(out["regime_probs"])
    src = np.concatenate([np.arange(c[4] + seg_of[c[3]][1], c[4] + seg_of[c[3]][1] + seg_of[c[3]][2]) for c in chains])
    dst = np.concatenate([np.arange(seg_of[c[3]][0] + seg_of[c[3]][1], seg_of[c[3]][0] + seg_of[c[3]][1]
                                    + seg_of[c[3]][2]) for c in chains])
    counts = parallel.posterior_counts(split, regime, B, torch.from_numpy(src), torch.from_numpy(dst), N_SITES)
    return counts, units


def _run_rank(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        counts, units = _rank_counts(rank, world)
        parallel.allreduce_counts(counts)
        uu = torch.tensor([units], dtype=torch.int64)
        dist.all_reduce(uu)
        if rank == 0:
            q.put((counts.numpy(), int(uu.item())))
    finally:
        dist.destroy_process_group()


def test_c4_job_two_ranks_equals_one(oracle):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_run_rank, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    got, units = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    want, units1 = _rank_counts(0, 1)
    np.testing.assert_array_equal(got, want.numpy())
    assert units == units1 == 3 * N_SITES
    assert np.all(got[:, 1:1 + K].sum(1) == 3 * B)  # every site once per trajectory of every seed
