"""Why concurrent `hygeia infer` processes slow each other's chains (VERDICT r5
item 3b): the same N single-chain tasks of a 2.4M-site chromosome (100k-site
segments + 5k buffers, 4 + 4 samples, K = 6, M = 50, B = 25), in ONE process:

- ``alone``: one chain by itself (the single task's kernel time);
- ``streams``: N single-chain launches on N HIP streams of this process at once
  (one context; the GPU runs them side by side, as N processes could; HIP maps
  the streams onto GPU_MAX_HW_QUEUES hardware queues, 4 by default, each of
  which runs its kernels in order: run with GPU_MAX_HW_QUEUES=N to have all N
  at once);
- ``one_launch``: the N chains in one launch (infer_many's shape).

Per mode: the wall of the whole set and each chain's own span (HIP events on
its stream). Compare with tools/bench_pipeline.py --concurrent N, whose tasks
are N processes: if the processes' chains take longer than the streams' here,
the difference is the process level (HW-queue time slicing, host), not CU
contention. Prints one JSON line.

    python tools/bench_streams.py [--n 16] [--sites 2400000]
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
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--sites", type=int, default=2_400_000)
    a = ap.parse_args()

    import torch

    from hygeia_amd import _lib, synthetic, two_group

    L = _lib.load()
    dev = torch.device("cuda", 0)
    K, M, B, S = 6, 50, 25, 4
    d = synthetic.simulate_device(a.sites, S, S, K=K, coverage=100.0, device=dev)
    segs = synthetic.segment_chains(np.array([a.sites]))
    tasks = [(seg, sd) for sd in (0, 1) for seg in segs][:a.n]
    maxr = int(max(d["tot_control"].to(torch.int32).max().item() & 0xFFFF,
                   d["tot_case"].to(torch.int32).max().item() & 0xFFFF))
    mu, sg = synthetic.regime_params(K)
    model = two_group.CaseControlModel(mu, sg, two_group.uniform_theta(K, 0.8), num_resampled_ancestors=M,
                                       num_samples_backward=B, max_total_reads=maxr,
                                       max_duration=max(t[0][3] for t in tasks))
    E = torch.empty((a.sites, 2 * K), dtype=torch.float64, device=dev)
    two_group.DeviceChains(model, [(0, 10, 0, 0, 0)], 10, device=dev).emission(
        d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"], E=E)
    torch.cuda.synchronize()

    def chain(t):
        (ci, b, s0, n, r0, rl), sd = t
        return (s0, n, sd, (ci << 32) | b, 0)

    singles = [two_group.DeviceChains(model, [chain(t)], chain(t)[1], device=dev) for t in tasks]
    streams = [torch.cuda.Stream(device=dev) for _ in tasks]
    rows, allc = 0, []
    for t in tasks:
        c = chain(t)
        allc.append(c[:4] + (rows,))
        rows += c[1]
    many = two_group.DeviceChains(model, allc, rows, device=dev)

    def timed(fn_list):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in fn_list]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for (e0, e1), (dc, st) in zip(evs, fn_list):
            e0.record(st)
            dc.run(E, stream=st.cuda_stream)
            e1.record(st)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        spans = np.array([e0.elapsed_time(e1) / 1000.0 for e0, e1 in evs])
        for dc, _ in fn_list:
            if not bool((dc.status == 0).all().item()):
                raise RuntimeError("chain failed")
        return wall, spans

    timed([(singles[0], streams[0])])  # warm-up (module load, first launch)
    res = {}
    w, sp = timed([(singles[0], streams[0])])
    res["alone"] = {"wall_s": w, "chain_s": float(sp[0])}
    w, sp = timed(list(zip(singles, streams)))
    res["streams"] = {"wall_s": w, "chain_s": {"mean": float(sp.mean()), "min": float(sp.min()),
                                               "max": float(sp.max())}}
    w, sp = timed([(many, streams[0])])
    res["one_launch"] = {"wall_s": w}
    units = sum(t[0][5] for t in tasks)
    for k in res:
        res[k]["site_seeds_per_s"] = units / res[k]["wall_s"] if k != "alone" else tasks[0][0][5] / res[k]["wall_s"]
    line = {"what": f"{len(tasks)} single-chain tasks of a {a.sites}-site chromosome (110k-site chains, 4+4 samples, "
                    f"K={K}, M={M}, B={B}) in one process", "n": len(tasks),
            "env": {k: os.environ.get(k) for k in ("GPU_MAX_HW_QUEUES",)}, "modes": res}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
