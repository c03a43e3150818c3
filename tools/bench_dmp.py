"""Measurement of the aggregation / DMP-calling stage on MI355X.

Workload: the C3 layout -- 28M CpG sites in the reference's 100k-site segments
over 22 chromosomes, 2 seeds x B = 25 trajectories per site (P = 50), K = 6 --
with synthetic int16 trajectories resident in HBM (the hyg_tg_outputs layout,
segment blocks of both seeds interleaved as bench.py's chain order leaves them).
Timed: per-site counts (hyg_dmp_site_counts), FDR_procedure and
weighted_FDR_procedure on the split statistic t = 1 - #(r_ctrl != r_case) / P
at fdr 0.05, as get_dmps.py runs them. CPU baseline: the numpy restatement
(oracle/dmp_oracle.py, the reference's own numpy operations) on the same
statistics, and the reference's per-site numpy reductions (np.mean(merged == 0),
np.sum(r_ctrl != r_case)) on a 1M-site sample, scaled.

Prints one JSON line; `--out` also writes it to a file.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sites", type=int, default=28_000_000)
    ap.add_argument("--B", type=int, default=25)
    ap.add_argument("--seeds", type=int, default=2)
    ap.add_argument("--K", type=int, default=6)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-sample", type=int, default=1_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    import torch

    from hygeia_amd import dmp, synthetic
    from oracle import dmp_oracle as od

    dev = torch.device("cuda", 0)
    K, B, S = a.K, a.B, a.seeds
    P = B * S
    segs = synthetic.segment_chains(synthetic.chromosome_sizes(a.sites))
    # trajectory rows: every (segment, seed) block of untrimmed rows, seed-major like bench.py
    groups, block_rows, o = [], [], 0
    starts = {}
    for s in range(S):
        for gi, (ci, b, s0, n, r0, rl) in enumerate(segs):
            starts[(gi, s)] = o + r0
            o += n
    rows = o
    for gi, (ci, b, s0, n, r0, rl) in enumerate(segs):
        groups.append((s0 + r0, rl))
        block_rows.append([starts[(gi, s)] for s in range(S)])
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    merged = torch.randint(0, 2, (rows, B), dtype=torch.int16, device=dev, generator=g)
    control = torch.randint(0, K, (rows, B, 2), dtype=torch.int16, device=dev, generator=g)
    kase = control.clone()
    # ~5% differential sites (case regime differs in most trajectories), the rest rarely
    p_site = torch.where(torch.rand((rows, 1), device=dev, generator=g) < 0.05, 0.9, 0.01)
    flip = torch.rand((rows, B), device=dev, generator=g) < p_site
    kase[..., 1] = torch.where(flip, (control[..., 1] + 1) % K, control[..., 1])
    torch.cuda.synchronize()

    counts = torch.zeros((a.sites, 2 + 2 * K), dtype=torch.int32, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    stream = torch.cuda.current_stream(dev)
    dmp.site_counts(merged, control, kase, B, K, groups, block_rows, a.sites, counts=counts)  # warm-up
    torch.cuda.synchronize()
    t_counts = []
    for _ in range(a.reps):
        ev[0].record(stream)
        dmp.site_counts(merged, control, kase, B, K, groups, block_rows, a.sites, counts=counts)
        ev[1].record(stream)
        torch.cuda.synchronize()
        t_counts.append(ev[0].elapsed_time(ev[1]))
    ms_counts = min(t_counts)  # (the call synchronises on its descriptors: events bracket the kernel)
    n_rep = sum(r for _, r in groups)
    bytes_counts = n_rep * P * (2 + 4 + 4) + n_rep * (2 + 2 * K) * 4

    w_fp = torch.ones(a.sites, dtype=torch.float64, device=dev)
    pos = synthetic.positions(a.sites)
    w_fn_h = od.false_negative_weights(pos)
    w_fn = torch.from_numpy(w_fn_h).to(dev)
    dmp.fdr(counts, 1, P, 0.05)
    t0 = time.perf_counter()
    for _ in range(a.reps):
        fdr_res = dmp.fdr(counts, 1, P, 0.05)
    ms_fdr = (time.perf_counter() - t0) * 1000 / a.reps
    dmp.weighted_fdr(counts, 1, P, 0.05, w_fp, w_fn)
    t0 = time.perf_counter()
    for _ in range(a.reps):
        widx, wsum = dmp.weighted_fdr(counts, 1, P, 0.05, w_fp, w_fn)
    ms_w = (time.perf_counter() - t0) * 1000 / a.reps
    ms_total = ms_counts + ms_fdr + ms_w
    line = {
        "metric": "CpG sites/sec through aggregation + DMP calling (site counts, FDR, weighted FDR)",
        "value": a.sites / (ms_total / 1000.0), "unit": "CpG-sites/s", "n_gpus": 1, "higher_is_better": True,
        "data": "synthetic", "dtype": "int16/int32/f64",
        "config": {"workload": f"{a.sites} CpG, {len(groups)} segments, P = {B} x {S} seeds, K = {K}, fdr 0.05"},
        "ms": {"site_counts": ms_counts, "fdr": ms_fdr, "weighted_fdr": ms_w},
        "roofline": {"bound": "hbm", "kernel": "dmp_site_counts_kernel",
                     "achieved": bytes_counts / (ms_counts / 1000) / 1e9, "peak": 8000.0, "unit": "GB/s",
                     "frac": bytes_counts / (ms_counts / 1000) / 1e9 / 8000.0,
                     "bytes_per_site": bytes_counts / n_rep},
        "result": {"fdr_k": fdr_res[0], "fdr_threshold": fdr_res[2], "weighted_selected": int(widx.shape[0])},
    }
    if not a.no_cpu:
        c = counts[:, 1].cpu().numpy()
        t = od.statistics_from_counts(c, P)
        t0 = time.perf_counter()
        ref = od.fdr_procedure(t, 0.05)
        cpu_fdr = time.perf_counter() - t0
        t0 = time.perf_counter()
        ridx, rsum = od.weighted_fdr_procedure(t, 0.05, np.ones(a.sites), w_fn_h)
        cpu_w = time.perf_counter() - t0
        # per-site counts in numpy over a sample of the first segments' rows
        m_h, c_h, k_h, n_s = [], [], [], 0
        for gi, (s0, rl) in enumerate(groups):
            take = min(rl, a.cpu_sample - n_s)
            if take <= 0:
                break
            sl = lambda x, s: x[block_rows[gi][s]:block_rows[gi][s] + take].cpu().numpy()  # noqa: E731
            m_h.append(np.concatenate([sl(merged, s) for s in range(S)], 1))
            c_h.append(np.concatenate([sl(control, s)[..., 1] for s in range(S)], 1))
            k_h.append(np.concatenate([sl(kase, s)[..., 1] for s in range(S)], 1))
            n_s += take
        m_h, c_h, k_h = np.concatenate(m_h), np.concatenate(c_h), np.concatenate(k_h)
        t0 = time.perf_counter()  # what aggregate + get_dmps compute per site by default
        np.mean(m_h == 0, axis=1)  # aggregate_results.py:129
        1. - np.sum(c_h != k_h, axis=1) / P  # get_dmps.py:68-69
        cpu_counts = (time.perf_counter() - t0) * a.sites / n_s
        cpu_total = cpu_counts + cpu_fdr + cpu_w
        line["cpu_baseline"] = {"value": a.sites / cpu_total, "unit": "CpG-sites/s", "cores": 1, "kind": "port",
                                "sample": f"numpy restatement (oracle/dmp_oracle.py): FDR {cpu_fdr:.2f} s and "
                                          f"weighted FDR {cpu_w:.2f} s on all {a.sites} sites; per-site reductions "
                                          f"on {n_s} sites scaled x{a.sites / n_s:.1f} ({cpu_counts:.2f} s)"}
        line["parity"] = {"fdr": list(ref) == list(fdr_res),
                          "weighted": bool(np.array_equal(ridx, widx)) and rsum == wsum}
    print(json.dumps(line), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(json.dumps(line) + "\n")


if __name__ == "__main__":
    main()
