"""Throughput of the device stages either side of the inference path
(SURVEY.md 8f-3 and 8f-4), on synthetic genome-scale data resident in HBM:

* preprocess: hyg_pre_collapse (strand join + CpG-grid counts) for S samples
  on a 28 M-site grid, ~75 % of CpGs with a "+" record and ~75 % with a "-"
  record per sample; units = CpG sites x samples.
* BED labels: hyg_bed_labels on regime probabilities [28 M][6] f64.

Kernel times are HIP events on the launch stream; `achieved` = algorithmic
bytes (each input array read once, each output written once) / time, against
the 8 TB/s HBM peak. cpu_baseline: a vectorized numpy restatement on a bounded
prefix (single-threaded numpy, the reference's polars would use all cores).
Prints one JSON line per stage.

    python tools/bench_downstream.py [--sites N] [--samples S]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HBM_PEAK_GBS = 8000.0


def synth(T, seed):
    rng = np.random.default_rng(seed)
    pos0 = np.cumsum(rng.integers(2, 60, T, dtype=np.int64)) + 10_000
    has_p, has_m = rng.random(T) < 0.75, rng.random(T) < 0.75
    ps = pos0[has_p]
    pe = ps + 1
    pc = rng.integers(1, 40, ps.size).astype(np.float64)
    pp = np.round(rng.random(ps.size) * 100, 2)
    ms = pos0[has_m] + 1
    mc = rng.integers(1, 40, ms.size).astype(np.float64)
    mp = np.round(rng.random(ms.size) * 100, 2)
    return pos0, (ps, pe, pc, pp), (ms, mc, mp)


def cpu_collapse(pos0, plus, minus):
    """vectorized restatement (searchsorted joins) of the same computation"""
    ps, pe, pc, pp = plus
    ms, mc, mp = minus
    out = np.full((pos0.size, 2), np.nan)
    ip = np.searchsorted(ps, pos0)
    okp = (ip < ps.size) & (ps[np.minimum(ip, ps.size - 1)] == pos0)
    jn = np.searchsorted(ms, pe)
    okn = (jn < ms.size) & (ms[np.minimum(jn, ms.size - 1)] == pe)
    matched = np.zeros(ms.size, bool)
    matched[jn[okn]] = True
    jm = np.searchsorted(ms, pos0 + 1)
    okm = (jm < ms.size) & (ms[np.minimum(jm, ms.size - 1)] == pos0 + 1)
    minus_only = okm & ~matched[np.minimum(jm, ms.size - 1)]
    cp = np.where(okp, pc[np.minimum(ip, ps.size - 1)], 0.0)
    pcp = np.where(okp, pp[np.minimum(ip, ps.size - 1)], 0.0)
    jj = jn[np.minimum(ip, ps.size - 1)]
    pair = okp & okn[np.minimum(ip, ps.size - 1)]
    cn = np.where(pair, mc[np.minimum(jj, ms.size - 1)], np.where(~okp & minus_only, mc[np.minimum(jm, ms.size - 1)], 0.0))
    pn = np.where(pair, mp[np.minimum(jj, ms.size - 1)], np.where(~okp & minus_only, mp[np.minimum(jm, ms.size - 1)], 0.0))
    total = cp + cn
    have = (okp | minus_only) & (total > 0)
    with np.errstate(invalid="ignore", divide="ignore"):
        avg = ((cp * pcp) + (cn * pn)) / total
    r = lambda x: np.sign(x) * np.floor(np.abs(x) + 0.5)  # noqa: E731
    out[have, 0] = r((total * avg) / 100.0)[have]
    out[have, 1] = r((total * (100.0 - avg)) / 100.0)[have]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sites", type=int, default=28_000_000)
    ap.add_argument("--samples", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    from hygeia_amd import _lib

    L = _lib.load()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sp = C.c_void_p(stream.cuda_stream)
    T, S = args.sites, args.samples
    pos0, plus, minus = synth(T, 1)
    d_pos = torch.from_numpy(pos0).to(dev)
    dp = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in plus]
    dm = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in minus]
    scratch = torch.empty(minus[0].size, dtype=torch.uint8, device=dev)
    conf = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.empty((S, T, 2), dtype=torch.float64, device=dev)  # per-sample [T][2] blocks
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run():
        for s in range(S):  # the same synthetic sample in every column (layout and traffic are what is timed)
            _lib.check(L.hyg_pre_collapse(d_pos.data_ptr(), T, dp[0].data_ptr(), dp[1].data_ptr(), dp[2].data_ptr(),
                                          dp[3].data_ptr(), plus[0].size, dm[0].data_ptr(), dm[1].data_ptr(),
                                          dm[2].data_ptr(), minus[0].size, 1, scratch.data_ptr(), out[s].data_ptr(),
                                          2, 0, conf.data_ptr(), sp))

    run()
    torch.cuda.synchronize(dev)
    ev0.record(stream)
    for _ in range(args.reps):
        run()
    ev1.record(stream)
    ev1.synchronize()
    ms = ev0.elapsed_time(ev1) / args.reps
    # per sample: pos0 read, the records read once, the match flags written + read, the count pair written
    bytes_sample = 8 * T + 32 * plus[0].size + 24 * minus[0].size + 16 * T  # single-base: no match flags
    chk = out[0].cpu().numpy()
    n_cpu = min(T, 4_000_000)
    t0 = time.perf_counter()
    ref = cpu_collapse(pos0[:n_cpu], tuple(a[a_ok] for a, a_ok in zip(plus, [plus[0] <= pos0[n_cpu - 1]] * 4)),
                       tuple(a[m_ok] for a, m_ok in zip(minus, [minus[0] <= pos0[n_cpu - 1] + 1] * 3)))
    dt = time.perf_counter() - t0
    same = np.array_equal(np.nan_to_num(ref, nan=-1.0), np.nan_to_num(chk[:n_cpu], nan=-1.0))
    print(json.dumps({
        "metric": "CpG site-samples/sec through the preprocess strand collapse + CpG-grid counts",
        "value": T * S / (ms / 1000.0), "unit": "CpG-site-samples/s", "n_gpus": 1, "ms_per_step": ms,
        "dtype": "int64/f64", "data": "synthetic",
        "config": {"workload": f"{T} CpG grid x {S} samples, 75% + / 75% - strand records per sample"},
        "roofline": {"bound": "hbm", "kernel": "pre_grid_kernel",
                     "achieved": bytes_sample * S / (ms / 1000.0) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": bytes_sample * S / (ms / 1000.0) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                     "bytes_per_unit": bytes_sample / T},
        "cpu_baseline": {"value": n_cpu / dt, "unit": "CpG-site-samples/s", "cores": 1, "kind": "port",
                         "sample": f"numpy searchsorted restatement, {n_cpu} sites x 1 sample in {dt:.2f} s"},
        "parity_vs_cpu_restatement": bool(same)}), flush=True)
    del out, scratch
    # ---- BED labels
    K = 6
    probs = torch.rand((T, K), dtype=torch.float64, device=dev)
    probs /= probs.sum(dim=1, keepdim=True)
    lab = torch.empty(T, dtype=torch.int8, device=dev)
    sc = torch.empty(T, dtype=torch.float64, device=dev)
    _lib.check(L.hyg_bed_labels(probs.data_ptr(), K, T, lab.data_ptr(), sc.data_ptr(), sp))
    torch.cuda.synchronize(dev)
    ev0.record(stream)
    for _ in range(args.reps):
        _lib.check(L.hyg_bed_labels(probs.data_ptr(), K, T, lab.data_ptr(), sc.data_ptr(), sp))
    ev1.record(stream)
    ev1.synchronize()
    ms = ev0.elapsed_time(ev1) / args.reps
    b = (8 * K + 9) * T
    ph = probs[:2_000_000].cpu().numpy()
    t0 = time.perf_counter()
    mx = ph.max(axis=1)
    ties = (ph == mx[:, None]).sum(axis=1)
    rl = np.where(ties > 1, -1, ph.argmax(axis=1))
    dt = time.perf_counter() - t0
    same = np.array_equal(rl, lab[:2_000_000].cpu().numpy()) and np.array_equal(mx, sc[:2_000_000].cpu().numpy())
    print(json.dumps({
        "metric": "CpG sites/sec through the regime BED labels (max, first argmax, equiprobable ties)",
        "value": T / (ms / 1000.0), "unit": "CpG-sites/s", "n_gpus": 1, "ms_per_step": ms, "dtype": "f64",
        "data": "synthetic", "config": {"workload": f"{T} sites x K={K} regime probabilities in HBM"},
        "roofline": {"bound": "hbm", "kernel": "bed_label_kernel", "achieved": b / (ms / 1000.0) / 1e9,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": b / (ms / 1000.0) / 1e9 / HBM_PEAK_GBS,
                     "traffic": None, "bytes_per_unit": 8 * K + 9},
        "cpu_baseline": {"value": 2_000_000 / dt, "unit": "CpG-sites/s", "cores": 1, "kind": "port",
                         "sample": f"numpy restatement on 2000000 sites in {dt:.2f} s"},
        "parity_vs_cpu_restatement": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
