"""One rank of bench.py's C4 job on the GPU (TEST INFRASTRUCTURE): its LPT
shard of a fixed multi-seed job over a small genome, through the same code as
bench.py's SCALE runs: the chains on the HIP path (DeviceChains), the per-seed
posterior-count kernel (hyg_tg_posterior_counts) and the all-reduce of the
device counts over the ranks (parallel.gather_counts; "gloo": several ranks may
share one GPU; "nccl" = RCCL, one rank per GPU).

    python tests/c4_rank.py --rank R --world W --port P --out counts.npz [--backend nccl]

Used by tests/test_gpu_c4_sharded.py, which starts the ranks as fresh
processes before they touch the GPU."""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N_SITES, K, M, B, S, SEEDS = 30_000, 6, 50, 25, 4, 3
SEG, BUF = 4_000, 200


def problem():
    from hygeia_amd import synthetic

    segs = synthetic.segment_chains(synthetic.chromosome_sizes(N_SITES, n_chrom=3), SEG, BUF)
    d = synthetic.simulate(N_SITES, S, S, K=K, seed=44, coverage=100.0)
    return segs, d


def job_args():
    return argparse.Namespace(job="c4", seeds=2, total_seeds=SEEDS)


def rank_counts(rank: int, world: int, on_device: bool = False, always: bool = False):
    """This rank's chains on the GPU through the code a SCALE run executes
    (bench.py:main): bench.build_chains -> DeviceChains -> the gather plan
    parallel.gather_tables (per seed, hyg_tg_posterior_counts without atomics)
    -> parallel.gather_counts, whose allreduce_counts sums over the ranks when a
    process group is up. -> (counts [N_SITES][1+2K] int32, on the CPU unless
    on_device, units, chains, threads per chain, exclusive flags of the gather)."""
    import torch

    import bench
    from hygeia_amd import _lib, parallel, synthetic, two_group

    segs, d = problem()
    chains, n_out, units, _ = bench.build_chains(job_args(), segs, rank, world)
    dev = torch.device("cuda", torch.cuda.current_device())
    t = {k: torch.from_numpy(np.ascontiguousarray(d[k]).view(np.int16)).to(dev) for k in
         ("meth_control", "tot_control", "meth_case", "tot_case")}
    mu, sg = synthetic.regime_params(K)
    model = two_group.CaseControlModel(mu, sg, two_group.uniform_theta(K, 0.8), num_resampled_ancestors=M,
                                       num_samples_backward=B,
                                       max_total_reads=int(max(d["tot_control"].max(), d["tot_case"].max())),
                                       max_duration=SEG + 2 * BUF)
    L = _lib.load()
    dc = two_group.DeviceChains(model, chains, n_out, device=dev)
    seg_of = {(ci << 32) | b: (s0, r0, rl) for (ci, b, s0, n, r0, rl) in segs}
    tabs = parallel.gather_tables(chains, seg_of, dev)
    stream = torch.cuda.Stream(device=dev)
    sp = stream.cuda_stream
    E = dc.emission(t["meth_control"], t["tot_control"], t["meth_case"], t["tot_case"])
    torch.cuda.synchronize()
    counts = torch.empty((N_SITES, 1 + 2 * K), dtype=torch.int32, device=dev)
    dc.run(E, stream=sp)
    with torch.cuda.stream(stream):
        parallel.gather_counts(L, [(dc.split_probs, dc.regime_probs, tabs)], B, counts, sp, always=always)
    torch.cuda.synchronize()
    if not bool((dc.status == 0).all().item()):
        raise RuntimeError(f"chains failed: {dc.status.cpu().numpy()}")
    threads = int(L.hyg_tg_threads_per_chain(model.handle, len(chains)))
    return (counts if on_device else counts.cpu()), units, len(chains), threads, [x[2] for x in tabs]


def oracle_counts():
    """The same job's counts from the CPU oracle's chains (test infrastructure)."""
    import concurrent.futures as cf

    import torch

    import bench
    from hygeia_amd import parallel, synthetic
    from oracle import binding as ob

    segs, d = problem()
    chains, n_out, units, _ = bench.build_chains(job_args(), segs, 0, 1)
    mu, sg = synthetic.regime_params(K)
    p = ob.make_params(K=K, M=M, B=B, mu=mu, sigma=sg)
    E = ob.emission(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
    split = torch.zeros(n_out, dtype=torch.float32)
    regime = torch.zeros((n_out, 2 * K), dtype=torch.float32)

    def one(c):
        s0, n, sd, cid, o = c
        return c, ob.chain(p, E[s0:s0 + n], sd, cid)

    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        for (s0, n, sd, cid, o), out in ex.map(one, chains):
            assert out["status"] == 0
            split[o:o + n] = torch.from_numpy(out["split_probs"])
            regime[o:o + n] = torch.from_numpy(out["regime_probs"])
    seg_of = {(ci << 32) | b: (s0, r0, rl) for (ci, b, s0, n, r0, rl) in segs}
    src = np.concatenate([np.arange(c[4] + seg_of[c[3]][1], c[4] + seg_of[c[3]][1] + seg_of[c[3]][2]) for c in chains])
    dst = np.concatenate([np.arange(seg_of[c[3]][0] + seg_of[c[3]][1], seg_of[c[3]][0] + seg_of[c[3]][1]
                                    + seg_of[c[3]][2]) for c in chains])
    return parallel.posterior_counts(split, regime, B, torch.from_numpy(src), torch.from_numpy(dst), N_SITES), units


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--backend", default="gloo", choices=("gloo", "nccl"))
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(a.port)
    nccl = a.backend == "nccl"
    if nccl:  # RCCL: one rank per GPU, device tensors
        torch.cuda.set_device(a.rank % torch.cuda.device_count())
    dist.init_process_group(a.backend, rank=a.rank, world_size=a.world)
    try:
        # (world 1 under nccl: the same collective as bench.py's, through RCCL over this GPU)
        counts, units, n_chains, threads, excl = rank_counts(a.rank, a.world, on_device=True, always=nccl)
        uu = torch.tensor([units, n_chains], dtype=torch.int64, device=counts.device)
        dist.all_reduce(uu)
        if a.rank == 0:
            np.savez(a.out, counts=counts.cpu().numpy(), units=int(uu[0].item()), chains=int(uu[1].item()),
                     threads=threads, backend=a.backend,
                     exclusive=np.array(excl))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
