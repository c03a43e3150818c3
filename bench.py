"""bench.py -- CpG sites/s through forward-backward (BASELINE.json metric).

Workload (BASELINE.json configs[2], "C3"): two-group, 28M CpG over 22
chromosomes cut into the reference's 100k-site segments with 5k buffers
(run_inference_two_groups.py:194-218), 4 + 4 samples, K = 6, M = 50, B = 25,
2 inference seeds per GPU. One "step" = the whole hot path over that workload
with the counts resident in HBM: Beta-Binomial emission table, particle filter
with optimal finite-state resampling, backward simulation of 25 trajectories,
for every (chromosome segment, seed) chain. Units = trimmed CpG sites x seeds.

Multi-GPU (torchrun, one rank per GPU): the chains are independent; every rank
runs the full genome with its own seeds (weak scaling, no collective in the
filter); each step ends with the job's gather: per-site posterior counts over all
trajectories, summed over ranks by one RCCL all-reduce (hygeia_amd/parallel.py).
value = sum over ranks / max-over-ranks time.

Also reported: the roofline of the dominant kernel (HIP events on the launch
stream), and the CPU oracle timed on the host cores on a bounded sample.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "CpG sites/sec through forward-backward; 28M CpG, K=6, 2 seeds, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def bytes_per_unit(s_ctrl: int, s_case: int, K: int, M: int, B: int) -> int:
    """counts (uint16 meth+total) + ancestor history written and
    read (8 B weight + 8 B state per ancestor, twice) + trajectories (int16 x5
    per trajectory) + split/regime probs (f32)."""
    return 4 * (s_ctrl + s_case) + 2 * M * 16 + B * 10 + 4 * (1 + 2 * K)


def _config_name(args) -> str:
    """BASELINE.json config the arguments describe (SURVEY.md 8 shorthand)."""
    if args.K == 12 and args.samples == 50:
        return "C5"
    if args.K == 6 and args.samples == 4 and args.seeds == 2:
        return "C3"
    return "custom"


def cpu_baseline(args, d_host, chains, seconds: float, threads: int):
    """The CPU oracle (oracle/tg_oracle.c, 'port') on `threads` host threads,
    each running emission + filter + backward simulation on a prefix of one
    chain of the same workload, sized to ~`seconds` of CPU work."""
    from oracle import binding as ob
    from hygeia_amd import synthetic as syn

    mu, sg = syn.regime_params(args.K)
    p = ob.make_params(K=args.K, M=args.M, B=args.B, mu=mu, sigma=sg)
    # calibrate: time a short prefix on one thread
    c0 = chains[0]
    n_cal = 1500
    sl = slice(c0[2], c0[2] + n_cal)
    t0 = time.perf_counter()
    E = ob.emission(p, d_host["meth_control"][sl], d_host["tot_control"][sl], d_host["meth_case"][sl],
                    d_host["tot_case"][sl])
    ob.chain(p, E, 0, 1)
    per_site = (time.perf_counter() - t0) / n_cal
    n_sites = int(max(2000, min(100000, seconds / per_site)))
    results = [None] * threads
    starts = [chains[i % len(chains)][2] for i in range(threads)]

    def work(i):
        s0 = starts[i]
        n = n_sites
        sl = slice(s0, s0 + n)
        E = ob.emission(p, d_host["meth_control"][sl], d_host["tot_control"][sl], d_host["meth_case"][sl],
                        d_host["tot_case"][sl])
        out = ob.chain(p, E, i, 7 + i)
        results[i] = (n, out["status"])

    th = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    total = sum(r[0] for r in results)
    return {"value": total / dt, "unit": "CpG-sites*seeds/s", "cores": threads, "kind": "port",
            "sample": f"{threads} threads x {n_sites}-site prefixes of the workload's chains, each one "
                      f"oracle/tg_oracle.c emission + filter + backward simulation (M={args.M}, B={args.B}); "
                      f"{total} site-seeds in {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--sites", type=int, default=28_000_000)
    ap.add_argument("--seeds", type=int, default=2, help="inference seeds per GPU")
    ap.add_argument("--samples", type=int, default=4, help="samples per group")
    ap.add_argument("--K", type=int, default=6)
    ap.add_argument("--M", type=int, default=50)
    ap.add_argument("--B", type=int, default=25)
    ap.add_argument("--coverage", type=float, default=100.0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check", action="store_true", help="compare one short chain with the oracle first")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    from hygeia_amd import _lib, parallel, synthetic, two_group

    L = _lib.load()
    K, M, B = args.K, args.M, args.B
    # ---- synthetic workload, resident in HBM
    data = synthetic.simulate_device(args.sites, args.samples, args.samples, K=K, coverage=args.coverage,
                                     device=dev)
    sizes = synthetic.chromosome_sizes(args.sites)
    segs = synthetic.segment_chains(sizes)
    seeds = [rank * args.seeds + s for s in range(args.seeds)]
    chains, out = [], 0
    for sd in seeds:
        for (ci, b, s0, n, r0, rl) in segs:
            chains.append((s0, n, sd, (ci << 32) | b, out))
            out += n
    chains.sort(key=lambda c: -c[1])  # longest first: the tail chains start early
    units = sum(rl for (_, _, _, _, _, rl) in segs) * len(seeds)
    max_reads = int(max(data["tot_control"].to(torch.int32).max().item() & 0xFFFF,
                        data["tot_case"].to(torch.int32).max().item() & 0xFFFF))
    mu, sg = synthetic.regime_params(K)
    theta = two_group.uniform_theta(K, 0.8)
    model = two_group.CaseControlModel(mu, sg, theta, num_resampled_ancestors=M, num_samples_backward=B,
                                       max_total_reads=max_reads, max_duration=max(c[1] for c in chains))
    dc = two_group.DeviceChains(model, chains, out, device=dev)
    stream = torch.cuda.Stream(device=dev)
    sp = stream.cuda_stream
    E = torch.empty((args.sites, 2 * K), dtype=torch.float64, device=dev)
    # final gather of the job (aggregate_results.py:71-206): per-site posterior
    # counts over all seeds' trajectories, summed over ranks by one all-reduce
    seg_of = {(ci << 32) | b: (s0, r0, rl) for (ci, b, s0, n, r0, rl) in segs}
    src = np.concatenate([np.arange(c[4] + seg_of[c[3]][1], c[4] + seg_of[c[3]][1] + seg_of[c[3]][2]) for c in chains])
    dst = np.concatenate([np.arange(seg_of[c[3]][0] + seg_of[c[3]][1], seg_of[c[3]][0] + seg_of[c[3]][1]
                                    + seg_of[c[3]][2]) for c in chains])
    rows_out = torch.from_numpy(src).to(dev)
    rows_site = torch.from_numpy(dst).to(dev)
    counts = torch.zeros((args.sites, 1 + 2 * K), dtype=torch.int32, device=dev)

    def step():
        dc.emission(data["meth_control"], data["tot_control"], data["meth_case"], data["tot_case"], E=E,
                    stream=sp)
        dc.run(E, stream=sp)
        with torch.cuda.stream(stream):
            counts.zero_()
            parallel.posterior_counts(dc.split_probs, dc.regime_probs, B, rows_out, rows_site, args.sites, counts)
            parallel.allreduce_counts(counts)

    L.hyg_set_kernel_timing(1)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    kms = np.zeros(3)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        ms3 = (ctypes.c_float * 3)()
        _lib.check(L.hyg_tg_last_kernel_ms(ms3))
        kms += np.array(list(ms3))
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    L.hyg_set_kernel_timing(0)
    status = dc.status.cpu().numpy()
    if (status != 0).any():
        raise RuntimeError(f"{int((status != 0).sum())} chains failed: {np.unique(status)}")
    # every site is counted once per trajectory of every seed on every rank
    per_site = counts[:, 1:1 + K].sum(dim=1)
    if not bool((per_site == B * len(seeds) * world).all().item()):
        raise RuntimeError("posterior counts do not cover every site once per trajectory")
    if dist:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = tt.item()
    ms_per_step = dt * 1000.0 / args.steps
    value = units * world / (ms_per_step / 1000.0)
    kavg = kms / args.steps  # emission, forward, backward (ms per launch)
    names = ["tg_emission_kernel", "tg_forward_kernel", "tg_backward_kernel"]
    dom = int(np.argmax(kavg))
    bpu = bytes_per_unit(args.samples, args.samples, K, M, B)
    achieved = bpu * units / (kavg[dom] / 1000.0) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):  # HBM bytes per launch from the PMC pass of the same workload
        try:
            pj = json.load(open(pmc))
            if pj.get("workload_sites") == args.sites and pj.get("seeds_per_gpu") == args.seeds:
                traffic = pj.get(names[dom])
        except Exception:
            traffic = None
    line = {
        "metric": METRIC, "value": value, "unit": "CpG-sites*seeds/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"{_config_name(args)} two_group {args.sites} CpG (22 chromosomes, 100k segments + 5k buffers), "
                               f"{args.samples}+{args.samples} samples, K={K}, M={M}, B={B}, "
                               f"{args.seeds} seeds per GPU", "chains_per_gpu": len(chains),
                   "global_sites_x_seeds": units * world, "parallelism": f"chains over {world} GPU(s)"},
        "roofline": {"bound": "hbm", "kernel": names[dom], "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "bytes_per_unit": bpu, "kernel_ms": {n: float(v) for n, v in zip(names, kavg)}},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        host = {k: data[k].cpu().numpy().view(np.uint16) for k in
                ("meth_control", "tot_control", "meth_case", "tot_case")}
        line["cpu_baseline"] = cpu_baseline(args, host, [(ci, b, s0, n) for (ci, b, s0, n, r0, rl) in segs],
                                            args.cpu_seconds, args.cpu_threads)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
