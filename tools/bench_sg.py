"""Single-group throughput (BASELINE.json configs[1], "C2"): whole-genome
synthetic, 28M CpG over 22 chromosomes, 4 samples, K = 6, N_max = 250,
epsilon = 0.01, 1 seed on 1 GPU. One chain per chromosome, as the reference
runs one R process per (sample group, chromosome); one "step" = emission table
+ SMC / optimal resampling / online marginal smoothing of every chain, counts
resident in HBM. Prints one JSON line in bench.py's format (units = CpG sites).

    python tools/bench_sg.py [--config c1|c2] [--sites N] [--steps K] [--warmup W] [--per-sample]

--config c1 is BASELINE.json configs[0]: the chr21-sized chain of the same
genome (454 914 sites), 2 samples, K = 6, 1 seed; its CPU baseline times the
oracle/ restatement on ALL of C1 (one thread: the reference runs one R process
per chromosome), as BASELINE.md 3 asks. Both configs draw the data from the
single-group model of bin/simulate_data (per-regime omega) at the
reference's default coverage lambda = 100.

--estimate-parameters runs the two-group pipeline's actual stage 2
(2_estimate_parameters_and_regimes.nf: --estimate_regime_probabilities
--estimate_parameters): online parameter estimation with the
flag defaults (ADAM, an update every 200 steps), theta rows written per chain.

--per-sample runs the single-group pipeline's granularity instead
(modules/single_group/3_estimate_regimes.nf: one process per (case_id,
chromosome), one sample per chain): samples x 22 chains of S = 1, units = CpG
sites x samples. The default is the joint S-sample chain per chromosome (the
two-group pipeline's step 2 on the control group, 2_estimate_parameters_and_regimes.nf).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def bytes_per_site(S: int, K: int) -> int:
    """SURVEY.md 8(d) algorithmic bytes per site: uint16 counts (2 x S x 2 B),
    the position (4 B) and the f64 regime probabilities written (8K); the f64
    emission table between the two kernels is an intermediate and not counted
    (C2: 16 + 4 + 48 = 68 B)."""
    return 4 * S + 4 + 8 * K


def cpu_baseline(meth, tot, chains, params, seconds, threads, pe=False, refstruct=False):
    """Sites/s of the CPU restatement on `threads` threads over prefixes of the
    chains, sized to about `seconds`. refstruct: the reference's cost structure
    (oracle_sg_chain_refstruct: the Beta-Binomial from the counts at every use,
    9 lgamma per sample, K x N_prev of them per step for the fresh particles as in
    computeWeightsCp, Smc.h:563-573); else the optimised port (one
    emission table per site)."""
    from oracle import sg_binding as sb

    p = sb.SgParams.from_buffer_copy(bytes(params))
    ope = sb.make_pe()

    def run(sl, seed, cid):
        if refstruct:
            return sb.chain_refstruct(p, meth[sl], tot[sl], seed, cid)
        E = sb.emission(p, meth[sl], tot[sl])
        return sb.chain_pe(p, ope, E, seed, cid) if pe else sb.chain(p, E, seed, cid)

    s0 = chains[0][0]
    n_cal = 300 if refstruct else 2000
    t0 = time.perf_counter()
    run(slice(s0, s0 + n_cal), 0, 1)
    per_site = (time.perf_counter() - t0) / n_cal
    n = int(max(n_cal, min(400000, seconds / per_site)))
    n = min(n, min(c[1] for c in chains[:threads]))  # a prefix of every chain used
    res = [0] * threads

    def work(i):
        b = chains[i % len(chains)][0]
        out = run(slice(b, b + n), i, 7 + i)
        assert out["status"] == 0
        res[i] = n

    th = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    what = ("oracle_sg_chain_refstruct (the reference's emission structure: Beta-Binomial from the counts at "
            "every use; the backward-kernel rows factorised as in the port, not the reference's per-row exps) "
            if refstruct else "oracle/sg_oracle.c emission + ")
    return {"value": sum(res) / dt, "unit": "CpG-sites/s", "cores": threads, "kind": "port",
            "variant": "reference emission structure, factorised backward kernels" if refstruct else "optimised port",
            "sample": f"{threads} threads x {n}-site prefixes of the chromosome chains, each one "
                      f"{what}SMC + online smoothing"
                      f"{' + online parameter estimation' if pe else ''}; {sum(res)} sites in {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=("c1", "c2"), default="c2")
    ap.add_argument("--sites", type=int, default=None, help="default: 28M (c2), the chr21 share of 28M (c1)")
    ap.add_argument("--samples", type=int, default=None, help="default: 4 (c2), 2 (c1)")
    ap.add_argument("--K", type=int, default=6)
    ap.add_argument("--coverage", type=float, default=100.0, help="Poisson lambda (SURVEY.md 8d default 100)")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=0)
    ap.add_argument("--psi-capacity", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=None, help="default: the host cores usable (bench.host_cpus)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--per-sample", action="store_true", help="one chain per (sample, chromosome), S = 1")
    ap.add_argument("--estimate-parameters", action="store_true", help="online parameter estimation (8f-1)")
    args = ap.parse_args()

    import torch

    from hygeia_amd import _lib, synthetic

    c1 = args.config == "c1"
    chr21 = int(synthetic.chromosome_sizes(28_000_000)[20])
    if args.sites is None:
        args.sites = chr21 if c1 else 28_000_000
    if args.samples is None:
        args.samples = 2 if c1 else 4

    # the chain kernel runs for minutes: a heartbeat keeps the run visibly alive
    t_start = time.perf_counter()

    def beat():
        while True:
            time.sleep(20)
            print(f"[bench_sg] alive {time.perf_counter() - t_start:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()

    dev = torch.device("cuda", 0)
    L = _lib.load()
    K, S = args.K, args.samples
    d = synthetic.simulate_device(args.sites, S, 1, K=K, coverage=args.coverage, omega=synthetic.SG_OMEGA,
                                  device=dev)
    meth, tot = d["meth_control"], d["tot_control"]
    del d["meth_case"], d["tot_case"]
    sizes = np.array([args.sites]) if c1 else synthetic.chromosome_sizes(args.sites)
    begins = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    n_rows = args.sites  # rows of the emission / output tables
    if args.per_sample:  # sample-major [S][T][1]: sample s's chain rows start at s * T
        meth = meth.t().contiguous().reshape(S * args.sites, 1)
        tot = tot.t().contiguous().reshape(S * args.sites, 1)
        n_rows = S * args.sites
        cl = [(int(s * args.sites + b), int(n), s * 22 + i) for s in range(S)
              for i, (b, n) in enumerate(zip(begins, sizes))]
        S = 1
    else:
        cl = [(int(b), int(n), 20 if c1 else i) for i, (b, n) in enumerate(zip(begins, sizes))]
    chains = sorted(cl, key=lambda c: -c[1])
    arr = (_lib.SgChain * len(chains))()
    for i, (b, n, ci) in enumerate(chains):
        arr[i].site_begin, arr[i].n_sites, arr[i].seed, arr[i].chain_id, arr[i].out_begin = b, n, 1, ci, b
    max_reads = int(tot.to(torch.int32).max().item() & 0xFFFF)
    p = _lib.SgParams()
    L.hyg_sg_params_default(C.byref(p))  # pipeline defaults: K = 6, u = 3, N_max = 250, epsilon = 0.01
    if K != p.n_regimes:
        raise SystemExit("the C2 workload is K = 6")
    h = C.c_void_p()
    _lib.check(L.hyg_sg_model_create(C.byref(p), max_reads, int(max(sizes)), C.byref(h)))
    pe = None
    if args.estimate_parameters:
        pe = _lib.SgPeParams()
        L.hyg_sg_pe_params_default(C.byref(pe))
        n_theta = int(L.hyg_sg_pe_theta_rows(arr, len(chains), pe.n_steps_without_update))
        theta = torch.empty((n_theta, K * K), dtype=torch.float64, device=dev)
        wsb = int(L.hyg_sg_pe_workspace_bytes(h, arr, len(chains), args.psi_capacity))
    else:
        wsb = int(L.hyg_sg_workspace_bytes(h, len(chains), args.psi_capacity))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    E = torch.empty((n_rows, K), dtype=torch.float64, device=dev)
    probs = torch.empty((n_rows, K), dtype=torch.float64, device=dev)
    st = torch.zeros(len(chains), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = C.c_void_p(stream.cuda_stream)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    kms = np.zeros(2)

    def step(timed):
        ev[0].record(stream)
        _lib.check(L.hyg_sg_emission(h, meth.data_ptr(), tot.data_ptr(), S, n_rows, E.data_ptr(), sp))
        ev[1].record(stream)
        if pe is not None:
            _lib.check(L.hyg_sg_run_chains_pe(h, C.byref(pe), arr, len(chains), E.data_ptr(), ws.data_ptr(), wsb,
                                              args.psi_capacity, probs.data_ptr(), theta.data_ptr(), st.data_ptr(),
                                              sp))
        else:
            _lib.check(L.hyg_sg_run_chains(h, arr, len(chains), E.data_ptr(), ws.data_ptr(), wsb,
                                           args.psi_capacity, probs.data_ptr(), st.data_ptr(), sp))
        ev[2].record(stream)
        if timed:
            ev[2].synchronize()
            kms[0] += ev[0].elapsed_time(ev[1])
            kms[1] += ev[1].elapsed_time(ev[2])

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    status = st.cpu().numpy()
    if (status != 0).any():
        raise RuntimeError(f"chains failed: {np.unique(status)}")
    pr = probs.sum(dim=1)
    # the unnormalised log-weights reach ~-2 per site (-5e6 on chromosome 1), where an
    # f64 ulp is ~1e-9: normalisation by exp(lw - log Z) is exact only to a few ulps
    bad = ~((pr - 1.0).abs() < 1e-6)
    if bool(bad.any().item()):
        idx = torch.nonzero(bad).flatten().cpu().numpy()
        owner = [next(ci for (b, n, ci) in chains if b <= i < b + n) for i in idx[:10]]
        print("bad rows:", len(idx), "first:", idx[:10].tolist(), "chains:", owner,
              "values:", probs[torch.from_numpy(idx[:3]).to(dev)].cpu().numpy().tolist(), file=sys.stderr)
        raise RuntimeError("regime probabilities do not sum to one")
    if pe is not None and not bool(torch.isfinite(theta).all().item()):
        raise RuntimeError("non-finite theta estimates")
    ms = dt * 1000.0 / args.steps
    kavg = kms / args.steps
    bps = bytes_per_site(S, K)
    units = n_rows  # CpG sites (joint chains) or sites x samples (per-sample chains)
    line = {
        "metric": "CpG sites/sec through SMC + online smoothing (single group)"
                  + (" + online parameter estimation" if pe is not None else ""), "value": units / (ms / 1000.0),
        "unit": "CpG-site-samples/s" if args.per_sample else "CpG-sites/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": (f"C2 single_group {args.sites} CpG x {args.samples} samples, one chain per "
                                f"(sample, chromosome) = {len(chains)} chains of 1 sample" if args.per_sample else
                                f"C1 single_group chr21 {args.sites} CpG, one chain, {S} samples" if c1 else
                                f"C2 single_group {args.sites} CpG, 22 chromosome chains, {S} samples jointly")
                               + ", single-group model data (per-regime omega)"
                               + f", K={K}, N_max=250, epsilon=0.01, 1 seed, coverage {args.coverage}"
                               + (", online parameter estimation (ADAM, update every 200 steps)"
                                  if pe is not None else ""),
                   "chains": len(chains), "longest_chain": int(max(sizes)), "parallelism": "chains on 1 GPU"},
        "roofline": {"bound": "hbm", "kernel": "sg_chain_kernel",
                     "achieved": bps * units / (kavg[1] / 1000.0) / 1e9, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": bps * units / (kavg[1] / 1000.0) / 1e9 / HBM_PEAK_GBS,
                     "traffic": None, "bytes_per_unit": bps,
                     "kernel_ms": {"sg_emission_kernel": float(kavg[0]), "sg_chain_kernel": float(kavg[1])},
                     "us_per_step_longest_chain": float(kavg[1] * 1000.0 / max(sizes))},
    }
    if not args.no_cpu_baseline and c1:
        import bench
        from oracle import sg_binding as sb

        # C1 in full on the CPU: the restatement over the whole chain, one thread
        mh, th = meth.cpu().numpy().view(np.uint16), tot.cpu().numpy().view(np.uint16)
        pc = sb.SgParams.from_buffer_copy(bytes(p))
        t0 = time.perf_counter()
        out = sb.chain(pc, sb.emission(pc, mh, th), 1, 20)
        dt_cpu = time.perf_counter() - t0
        assert out["status"] == 0
        line["cpu_baseline"] = {"value": args.sites / dt_cpu, "unit": "CpG-sites/s", "cores": 1, "kind": "port",
                                "variant": "optimised port",
                                "sample": f"the whole C1 chain ({args.sites} sites) in full: oracle/sg_oracle.c "
                                          f"emission + SMC + online smoothing, {dt_cpu:.1f} s",
                                "host": bench.host_cpus()}
        # and the reference's cost structure on one thread, a bounded prefix of the chain
        line["cpu_baseline"]["reference_structure"] = cpu_baseline(mh, th, chains, p, args.cpu_seconds, 1,
                                                                   refstruct=True)
    elif not args.no_cpu_baseline:
        import bench

        host = bench.host_cpus()
        mh, th = meth.cpu().numpy().view(np.uint16), tot.cpu().numpy().view(np.uint16)
        nth = args.cpu_threads or host["usable"]
        if pe is None:
            # headline: the reference's cost structure; the optimised port beside it
            line["cpu_baseline"] = cpu_baseline(mh, th, chains, p, args.cpu_seconds, nth, refstruct=True)
            line["cpu_baseline"]["optimised_port"] = cpu_baseline(mh, th, chains, p, args.cpu_seconds, nth)
        else:
            line["cpu_baseline"] = cpu_baseline(mh, th, chains, p, args.cpu_seconds, nth, pe=True)
        line["cpu_baseline"]["unit"] = line["unit"]
        line["cpu_baseline"]["host"] = host
    L.hyg_sg_model_destroy(h)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
