"""bench.py -- CpG sites/s through forward-backward (BASELINE.json metric).

Default workload (BASELINE.json configs[2], "C3"): two-group, 28M CpG over 22
chromosomes cut into the reference's 100k-site segments with 5k buffers
(run_inference_two_groups.py:194-218), 4 + 4 samples, K = 6, M = 50, B = 25,
2 inference seeds. One "step" = the whole hot path over that workload
with the counts resident in HBM: Beta-Binomial emission table, particle filter
with optimal finite-state resampling, backward simulation of 25 trajectories,
for every (chromosome segment, seed) chain, then the job's gather: per-site
posterior counts over all trajectories, summed over ranks by one RCCL
all-reduce (hygeia_amd/parallel.py; aggregate_results.py:129,181).
Units = trimmed CpG sites x seeds.

Jobs (--job); every job is ONE fixed job whose chain list chrom x segment x
seed (main.nf:46-75, modules/two_group/4_infer.nf:28) is split over the ranks
longest-first by parallel.shard_chains (strong scaling, no data-path
collective; the final all-reduce of the posterior counts is the gather):
  c3  (default) the metric's job: 2 seeds (BASELINE.json configs[2]; at 1/2/4/8
      GPUs the same 582 chains);
  c4  --total-seeds (8) seeds (configs[3]);
  c5  the stress config: 50 + 50 samples, K = 12, 4 seeds (configs[4]).
A rehearsal of several ranks on fewer GPUs (--dist-backend gloo) reports the
GPUs it used in n_gpus and the ranks in "ranks".

Also reported: the roofline of the dominant kernel (HIP events on the launch
stream), the HBM traffic and VALU-issue fraction from the PMC passes of the same
kernel build (profiles/pmc_*.json, matched by build.source_hash(); null when the
build changed since), and two CPU baselines timed on the host cores available to
the job on a bounded sample: the reference-structure restatement and the
optimised port (oracle/, test infrastructure).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "CpG sites/sec through forward-backward; 28M CpG, K=6, 2 seeds, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
N_SIMD = 256 * 4       # 256 CUs x 4 SIMDs
VALU_ISSUE_CYCLES = 2  # a wave64 VALU instruction occupies a SIMD-32 for 2 cycles (MI355X_MICROARCH.md)


def bytes_per_unit(s_ctrl: int, s_case: int, K: int, M: int, B: int) -> int:
    """counts (uint16 meth+total) + ancestor history written and
    read (8 B weight + 8 B state per ancestor, twice) + trajectories (int16 x5
    per trajectory) + split/regime probs (f32)."""
    return 4 * (s_ctrl + s_case) + 2 * M * 16 + B * 10 + 4 * (1 + 2 * K)


def host_cpus() -> dict:
    """The host cores this job may use: the affinity mask, the cgroup CPU quota
    and OMP_NUM_THREADS (set by the GPU box to its per-GPU CPU share), whichever
    is smallest; plus nproc and the CPU model for the record."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    info["cgroup_cpu_quota"] = quota
    omp = os.environ.get("OMP_NUM_THREADS")
    info["omp_num_threads"] = int(omp) if omp and omp.isdigit() else None
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    info["cpu_model"] = model
    lim = [info["affinity"]]
    if quota:
        lim.append(max(1, int(math.floor(quota))))
    if info["omp_num_threads"]:
        lim.append(info["omp_num_threads"])
    info["usable"] = min(lim)
    return info


class _Heartbeat:
    """Prints a progress line to stderr every `every` seconds while a long
    host-side phase runs (a silent GPU job is taken to be hung)."""

    def __init__(self, what: str, every: float = 30.0):
        self.what, self.every = what, every
        self._stop = threading.Event()

    def __enter__(self):
        def beat():
            t0 = time.perf_counter()
            while not self._stop.wait(self.every):
                print(f"[bench] {self.what}: {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

        self._t = threading.Thread(target=beat, daemon=True)
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._t.join()


def _threads_run(fn, n):
    res = [None] * n
    th = [threading.Thread(target=lambda i=i: res.__setitem__(i, fn(i))) for i in range(n)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    return res, time.perf_counter() - t0


def cpu_baseline(args, d_host, chains, seconds: float) -> dict:
    """Both CPU restatements (oracle/, ctypes: the GIL is released) on every
    usable host core, one chain prefix per thread (one thread per chain, as
    SURVEY.md 8d plans), each sized to ~`seconds` of work:
      - reference structure: Beta-Binomial per particle from the counts, full
        sort, full-N history, [B, N] backward rows (oracle_tg_chain_refstruct);
      - optimised port: per-site emission table, one backward row per distinct
        state, M-ancestor history (oracle_tg_chain)."""
    from oracle import binding as ob
    from hygeia_amd import synthetic as syn

    host = host_cpus()
    threads = host["usable"]
    mu, sg = syn.regime_params(args.K)
    p = ob.make_params(K=args.K, M=args.M, B=args.B, mu=mu, sigma=sg)
    keys = ("meth_control", "tot_control", "meth_case", "tot_case")

    def rows(i, n):
        s0 = chains[i % len(chains)][2]
        return [d_host[k][s0:s0 + n] for k in keys]

    def refstruct(i, n):
        return ob.chain_refstruct(p, *rows(i, n), 7 + i, i)["status"]

    def port(i, n):
        E = ob.emission(p, *rows(i, n))
        return ob.chain(p, E, 7 + i, i)["status"]

    out = {}
    for name, fn, n_cal in (("reference_structure", refstruct, 40), ("optimised_port", port, 1500)):
        with _Heartbeat(f"cpu baseline {name}"):
            t0 = time.perf_counter()
            fn(0, n_cal)
            per_site = (time.perf_counter() - t0) / n_cal
            n_sites = int(max(100, min(100000, seconds / per_site)))
            st, dt = _threads_run(lambda i: fn(i, n_sites), threads)
        if any(s != 0 for s in st):
            raise RuntimeError(f"CPU baseline {name} failed: {st}")
        total = n_sites * threads
        out[name] = {"value": total / dt, "unit": "CpG-sites*seeds/s", "cores": threads, "kind": "port",
                     "sample": f"{threads} threads (one chain each) x {n_sites}-site prefixes of the workload's "
                               f"chains, M={args.M}, B={args.B}: {total} site-seeds in {dt:.1f} s"}
    line = dict(out["reference_structure"])
    line["variant"] = ("reference structure (oracle_tg_chain_refstruct: per-particle Beta-Binomial, full sort, "
                       "full-N history, [B,N] backward rows)")
    line["optimised_port"] = out["optimised_port"]
    line["host"] = host
    return line


def pmc_record(name: str, workload: str):
    """A profiles/pmc_<name>.json record if it was measured on this kernel
    build and workload, else None."""
    from hygeia_amd import build

    path = os.path.join(ROOT, "profiles", f"pmc_{name}.json")
    try:
        rec = json.load(open(path))
    except (OSError, ValueError):
        return None
    if rec.get("source_hash") != build.source_hash() or rec.get("workload") != workload:
        return None
    return rec


def job_seeds(args) -> int:
    """Inference seeds of the whole (fixed) job."""
    return args.total_seeds if args.job == "c4" else args.seeds


def build_chains(args, segs, rank, world):
    """This rank's chains (site_begin, n_sites, seed, chain_id, out_begin), the
    units (trimmed site-seeds) it processes, and the seeds it uses."""
    from hygeia_amd import parallel

    allc = [(seg, sd) for sd in range(job_seeds(args)) for seg in segs]
    mine = parallel.shard_chains([c[0][3] for c in allc], world)[rank]
    picked = [allc[i] for i in mine]
    chains, out, units = [], 0, 0
    for (ci, b, s0, n, r0, rl), sd in picked:
        chains.append((s0, n, sd, (ci << 32) | b, out))
        out += n
        units += rl
    chains.sort(key=lambda c: -c[1])  # longest first: the tail chains start early
    return chains, out, units, picked


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--job", choices=("c3", "c4", "c5"), default="c3")
    ap.add_argument("--sites", type=int, default=28_000_000)
    ap.add_argument("--seeds", type=int, default=None, help="inference seeds of the c3 / c5 job")
    ap.add_argument("--total-seeds", type=int, default=8, help="seeds of the fixed c4 job")
    ap.add_argument("--samples", type=int, default=None, help="samples per group")
    ap.add_argument("--K", type=int, default=None)
    ap.add_argument("--M", type=int, default=50)
    ap.add_argument("--B", type=int, default=25)
    ap.add_argument("--coverage", type=float, default=100.0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--history-gib", type=float, default=100.0, help="forward->backward history budget in HBM")
    ap.add_argument("--launch-chains", type=int, default=768, help="chains per launch when over the budget")
    ap.add_argument("--no-batch-merge", action="store_true",
                    help="A/B: keep a partial last launch of --launch-chains chains on its own")
    ap.add_argument("--no-tail-overlap", action="store_true",
                    help="A/B: no tail overlap in the launch (hyg_tg_set_tail_overlap(0))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--shard", default=None, metavar="R/W",
                    help="run only rank R's chains of a W-rank job on this one GPU (a projection of one rank of "
                         "a W-GPU run; the line is labelled as such)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL on ROCm); gloo rehearses the multi-rank path, e.g. 2 ranks on one GPU")
    args = ap.parse_args()
    preset = {"c3": (2, 4, 6), "c4": (None, 4, 6), "c5": (4, 50, 12)}[args.job]
    args.seeds = args.seeds if args.seeds is not None else preset[0]
    args.samples = args.samples if args.samples is not None else preset[1]
    args.K = args.K if args.K is not None else preset[2]

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        # (local % device count: a gloo rehearsal may put several ranks on one GPU)
        torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group(args.dist_backend)
    dev = torch.device("cuda", local % torch.cuda.device_count() if world > 1 else 0)
    torch.cuda.set_device(dev)

    from hygeia_amd import _lib, parallel, synthetic, two_group

    L = _lib.load()
    if args.no_tail_overlap:
        _lib.check(L.hyg_tg_set_tail_overlap(0))
    K, M, B = args.K, args.M, args.B
    # ---- synthetic workload, resident in HBM (every rank holds the genome's counts)
    data = synthetic.simulate_device(args.sites, args.samples, args.samples, K=K, coverage=args.coverage,
                                     device=dev)
    sizes = synthetic.chromosome_sizes(args.sites)
    segs = synthetic.segment_chains(sizes)
    if args.shard:
        if world > 1:
            raise SystemExit("--shard is a single-process projection")
        srank, sworld = (int(x) for x in args.shard.split("/"))
        chains, n_out, units, picked = build_chains(args, segs, srank, sworld)
    else:
        chains, n_out, units, picked = build_chains(args, segs, rank, world)
    max_reads = int(max(data["tot_control"].to(torch.int32).max().item() & 0xFFFF,
                        data["tot_case"].to(torch.int32).max().item() & 0xFFFF))
    mu, sg = synthetic.regime_params(K)
    theta = two_group.uniform_theta(K, 0.8)
    model = two_group.CaseControlModel(mu, sg, theta, num_resampled_ancestors=M, num_samples_backward=B,
                                       max_total_reads=max_reads, max_duration=max(c[1] for c in chains))
    # launches: all chains at once while the forward->backward history fits the
    # budget, else batches of --launch-chains (one full round of resident
    # workgroups each) sharing one history buffer, run back to back
    budget = args.history_gib * 2 ** 30
    batches = [chains]
    if two_group.DeviceChains.workspace_bytes(model, chains) > budget:
        batches = [chains[i:i + args.launch_chains] for i in range(0, len(chains), args.launch_chains)]
        # a partial last batch (the 1-GPU C4 job: 3 x 768 + 24 of its shortest
        # chains) joins the one before when the history still fits: its chains
        # start in the slots that batch's shorter chains free, instead of a
        # launch of its own at low occupancy
        if (not args.no_batch_merge and len(batches) > 1 and len(batches[-1]) < args.launch_chains
                and two_group.DeviceChains.workspace_bytes(model, batches[-2] + batches[-1]) <= budget):
            batches[-2:] = [batches[-2] + batches[-1]]
    ws = torch.empty(max(two_group.DeviceChains.workspace_bytes(model, b) for b in batches), dtype=torch.uint8,
                     device=dev)
    seg_of = {(ci << 32) | b: (s0, r0, rl) for (ci, b, s0, n, r0, rl) in segs}
    runs = []
    for bch in batches:
        rebased, rows = [], 0
        for (s0, n, sd, cid, _) in bch:  # outputs of a batch: its own rows, in launch order
            rebased.append((s0, n, sd, cid, rows))
            rows += n
        dcb = two_group.DeviceChains(model, rebased, rows, device=dev, workspace=ws)
        # final gather (aggregate_results.py:71-206): per-site posterior counts over
        # all trajectories of all seeds (one HIP kernel over the chains' trimmed
        # rows), summed over ranks by one all-reduce
        # (one call per seed: a seed's chains cover disjoint sites, so no atomics)
        runs.append((dcb, parallel.gather_tables(rebased, seg_of, dev)))
    stream = torch.cuda.Stream(device=dev)
    sp = stream.cuda_stream
    E = torch.empty((args.sites, 2 * K), dtype=torch.float64, device=dev)
    counts = torch.zeros((args.sites, 1 + 2 * K), dtype=torch.int32, device=dev)

    def step():
        kms = np.zeros(3)
        runs[0][0].emission(data["meth_control"], data["tot_control"], data["meth_case"], data["tot_case"], E=E,
                            stream=sp)
        ms3 = (ctypes.c_float * 3)()
        for i, (dcb, _) in enumerate(runs):
            dcb.run(E, stream=sp)
            _lib.check(L.hyg_tg_last_kernel_ms(ms3))
            kms += np.array(list(ms3)) * np.array([1.0 if i == 0 else 0.0, 1.0, 1.0])
        with torch.cuda.stream(stream):
            parallel.gather_counts(L, [(dcb.split_probs, dcb.regime_probs, tabs) for dcb, tabs in runs], B, counts,
                                   sp)
        return kms

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
        kms += step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    L.hyg_set_kernel_timing(0)
    status = np.concatenate([r[0].status.cpu().numpy() for r in runs])
    if (status != 0).any():
        raise RuntimeError(f"{int((status != 0).sum())} chains failed: {np.unique(status)}")
    # every site is counted once per trajectory of every seed of the job
    seeds_job = job_seeds(args)
    per_site = counts[:, 1:1 + K].sum(dim=1)
    if args.shard:  # this rank's trimmed sites, once per trajectory of their chains' seeds
        if int(per_site.sum().item()) != B * units:
            raise RuntimeError("posterior counts do not cover the shard's sites once per trajectory")
    elif not bool((per_site == B * seeds_job).all().item()):
        raise RuntimeError("posterior counts do not cover every site once per trajectory of every seed")
    total_units = units
    if dist:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = tt.item()
        uu = torch.tensor([units], dtype=torch.int64, device=dev)
        dist.all_reduce(uu, op=dist.ReduceOp.SUM)
        total_units = int(uu.item())
    ms_per_step = dt * 1000.0 / args.steps
    value = total_units / (ms_per_step / 1000.0)
    kavg = kms / args.steps  # emission, forward, backward (ms per launch)
    names = ["tg_emission_kernel", "tg_forward_kernel", "tg_backward_kernel"]
    dom = int(np.argmax(kavg))
    bpu = bytes_per_unit(args.samples, args.samples, K, M, B)
    achieved = bpu * units / (kavg[dom] / 1000.0) / 1e9
    cfg_name = {"c3": "C3", "c4": "C4", "c5": "C5"}[args.job]
    if args.job != "c4" and (args.sites, args.samples, K, args.seeds) != {"c3": (28_000_000, 4, 6, 2),
                                                                          "c5": (28_000_000, 50, 12, 4)}[args.job]:
        cfg_name = "custom"
    workload = (f"{cfg_name} two_group {args.sites} CpG (22 chromosomes, 100k segments + 5k buffers), "
                f"{args.samples}+{args.samples} samples, K={K}, M={M}, B={B}, "
                f"{job_seeds(args)} seeds in total, chains sharded over the GPUs (LPT)")
    # (the PMC records hold whole-job launches: none for a rank's share)
    whole = world == 1 and not args.shard
    tr = pmc_record("traffic", workload) if whole else None
    iss = pmc_record("issue", workload) if whole else None
    roof = {"bound": "hbm", "kernel": names[dom], "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": tr.get(names[dom]) if tr else None,
            "bytes_per_unit": bpu, "units_per_launch": units,
            "kernel_ms": {n: float(v) for n, v in zip(names, kavg)}}
    if iss and names[dom] in iss.get("valu_per_launch", {}):
        clk = iss["clock_hz"][names[dom]]
        rate = iss["valu_per_launch"][names[dom]] / (kavg[dom] / 1000.0)
        roof["issue"] = {"valu_wave_instr_per_s": rate, "peak": N_SIMD * clk / VALU_ISSUE_CYCLES,
                         "clock_hz": clk, "frac": rate / (N_SIMD * clk / VALU_ISSUE_CYCLES),
                         "source": f"profiles/pmc_issue.json (SQ_INSTS_VALU, GRBM_GUI_ACTIVE; build {iss['source_hash']})"}
    # one rank per GPU over RCCL (nccl: any number of nodes); only a gloo rehearsal
    # may put several ranks on one node's GPUs
    n_gpus = world if args.dist_backend == "nccl" or world == 1 else min(world, torch.cuda.device_count())
    line = {
        "metric": METRIC, "value": value, "unit": "CpG-sites*seeds/s", "n_gpus": n_gpus, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": workload, "chains_per_rank": len(chains), "launches_per_step": len(runs),
                   "threads_per_chain": int(L.hyg_tg_threads_per_chain(model.handle, len(batches[0]))),
                   "chains_per_cu_resident": int(L.hyg_tg_chains_per_cu(model.handle, len(batches[0]))),
                   "global_sites_x_seeds": total_units,
                   "parallelism": f"chains over {world} rank(s) on {n_gpus} GPU(s)"},
        "roofline": roof,
    }
    if args.shard:
        line["projection"] = (f"one GPU running rank {srank}'s chains of a {sworld}-rank job: value = that rank's "
                              f"units / its time, NOT the job's throughput")
    if world != n_gpus:
        line["ranks"] = world
        line["rehearsal"] = f"{world} {args.dist_backend} ranks on {n_gpus} GPU(s)"
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        host = {k: data[k].cpu().numpy().view(np.uint16) for k in
                ("meth_control", "tot_control", "meth_case", "tot_case")}
        line["cpu_baseline"] = cpu_baseline(args, host, [(ci, b, s0, n) for (ci, b, s0, n, r0, rl) in segs],
                                            args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
