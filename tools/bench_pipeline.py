"""Pipeline-level throughput of the two-group drop-in, gz-CSV parse and result
files included.

A synthetic chromosome (default 2.4M CpG, the size of chr1 in the 28M
workload; 4 + 4 samples) is written in the pipeline's input format
(preprocess_bed.py:463-470: gzip CSVs of float64 counts + theta_{chrom}.csv.gz),
then timed end to end:

- `hygeia infer_many --batches all --seeds 0,1`: every (segment, seed) task of
  the chromosome in one launch, the CSVs parsed once;
- `hygeia infer` for one task (batch 0, seed 0), the unit that
  modules/two_group/4_infer.nf fans out; its wall time x the number of tasks is
  the cost of running the fan-out task by task on one GPU.

Prints one JSON line: sites x seeds / s for both, and the split of the
batched run (parse, launch, writes).

--concurrent 1,4,8,16 (round 5) instead runs EVERY task of the chromosome as a
fresh `hygeia infer` process, N at once (a thread pool of subprocesses), the
way Nextflow's local executor runs the module's fan-out on a node
(nextflow.config:17-21), and reports per N the aggregate sites x seeds / s and
the per-task wall times; `infer_many` runs as a subprocess too, so the parent
never holds a GPU context (the GPU box admits at most 16 processes on its card,
which caps N there).
--server (round 6) runs the --concurrent tasks through the node chain server
(`hygeia serve`, hygeia_amd/serve.py), started before the sweep and stopped
after it: the tasks are unchanged processes; their chains share launches.
usage: python tools/bench_pipeline.py [--sites N] [--seeds 0,1] [--workdir DIR] [--concurrent LIST]
                                      [--server [--gather S]] [--task-env K=V]
"""
from __future__ import annotations

import argparse
import gzip
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def write_inputs(d: str, chrom: str, T: int, S: int = 4, K: int = 6):
    from hygeia_amd import synthetic as syn
    from hygeia_amd import two_group

    data = syn.simulate(T, S, S, K=K, seed=20251024, coverage=100.0)
    os.makedirs(os.path.join(d, "data"), exist_ok=True)
    os.makedirs(os.path.join(d, "sg"), exist_ok=True)

    def save(path, a):  # np.savetxt(fmt='%s') of float64, as preprocess_bed.py writes them
        with gzip.open(path, "wt", compresslevel=1) as fh:
            rows = a.astype(np.float64)
            if rows.ndim == 1:
                rows = rows[:, None]
            fh.write("\n".join(",".join(f"{v:.1f}" for v in r) for r in rows.tolist()) + "\n")

    save(os.path.join(d, "data", f"positions_{chrom}.txt.gz"), syn.positions(T))
    for g in ("control", "case"):
        save(os.path.join(d, "data", f"n_total_reads_{g}_{chrom}.txt.gz"), data[f"tot_{g}"])
        save(os.path.join(d, "data", f"n_methylated_reads_{g}_{chrom}.txt.gz"), data[f"meth_{g}"])
    theta = two_group.uniform_theta(K, 0.8)
    with gzip.open(os.path.join(d, "sg", f"theta_{chrom}.csv.gz"), "wt") as fh:
        fh.write("data\n" + "\n".join(repr(float(x)) for x in theta) + "\n")


# Runs one CLI command in a fresh process and prints its own phase split
# (cli.LAST_TIMINGS) and device (cli.LAST_DEVICE) after '@@'.
DRIVER = ("import json, sys, time; t0 = time.perf_counter(); from hygeia_amd import cli; t1 = time.perf_counter(); "
          "rc = cli.main(sys.argv[1:]); t2 = time.perf_counter(); "
          "print('@@' + json.dumps(dict(cli.LAST_TIMINGS, import_cli=t1 - t0, main=t2 - t1, rc=rc, "
          "device=cli.LAST_DEVICE.get('device', -1), slot=cli.LAST_DEVICE.get('slot', -1))), flush=True)")


def run_task(args, env=None, version=False) -> dict:
    """One task as a fresh process; version: then `hygeia --version` as
    4_infer.nf:54-57 runs it after every task, inside the task's wall."""
    t0 = time.perf_counter()
    e = dict(os.environ if env is None else env, PYTHONPATH=ROOT, HYGEIA_TASK_TIMING="1")
    r = subprocess.run([sys.executable, "-c", DRIVER] + list(args), cwd=ROOT, capture_output=True, text=True, env=e)
    t1 = time.perf_counter()
    if r.returncode != 0:
        raise RuntimeError(f"hygeia {' '.join(args[:5])} failed: {r.stderr[-2000:]}")
    split = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("@@")][-1][2:])
    if version:
        v = subprocess.run([os.path.join(ROOT, "bin", "hygeia"), "--version"], cwd=ROOT, capture_output=True,
                           text=True, env=e)
        if v.returncode != 0 or "Hygeia version" not in v.stdout:
            raise RuntimeError(f"hygeia --version failed: {v.stderr[-500:]}")
        split["version"] = time.perf_counter() - t1
    t2 = time.perf_counter()
    return {"start": t0, "end": t2, "wall_s": t2 - t0, "split": split}


def concurrent_sweep(wd, common, seeds, sites, n_batches, ns, env=None):
    """Every (batch, seed) task as a fresh `hygeia infer` process followed by
    `hygeia --version` (the module's script), N at a time."""
    from concurrent.futures import ThreadPoolExecutor

    units = sites * len(seeds)
    tasks = [(b, sd) for b in range(n_batches) for sd in seeds]
    out = []
    for n in ns:
        rdir = os.path.join(wd, f"conc{n}")
        pc = (env or {}).get("HYGEIA_PARSE_CACHE", "0")
        if pc != "0":  # every N starts with an empty parse cache (a fresh pipeline run)
            shutil.rmtree(pc, ignore_errors=True)

        def one(t):
            b, sd = t
            r = run_task(["infer", "--batch", str(b), "--seed", str(sd), "--results_dir", rdir] + common, env=env,
                         version=True)
            print(f"  N={n} batch {b} seed {sd}: {r['wall_s']:.2f} s", file=sys.stderr, flush=True)  # progress
            return r

        t0 = time.perf_counter()
        with ThreadPoolExecutor(max_workers=n) as ex:
            res = list(ex.map(one, tasks))
        wall = time.perf_counter() - t0
        walls = np.array([r["wall_s"] for r in res])
        chains = np.array([r["split"].get("chains", 0.0) for r in res])
        keys = sorted({k for r in res for k, v in r["split"].items() if isinstance(v, (int, float))} - {"rc", "slot"})
        split_mean = {k: float(np.mean([r["split"].get(k, 0.0) for r in res])) for k in keys}
        kern = np.array([r["split"].get("kernels", 0.0) for r in res])
        ver = np.array([r["split"].get("version", 0.0) for r in res])
        rec = {"concurrent": n, "tasks": len(tasks), "wall_s": wall, "value": units / wall,
               "task_wall_s": {"mean": float(walls.mean()), "min": float(walls.min()), "max": float(walls.max())},
               "task_chains_s": {"mean": float(chains.mean()), "max": float(chains.max())},
               "task_kernels_s": {"mean": float(kern.mean()), "max": float(kern.max())},
               "task_version_s": {"mean": float(ver.mean()), "max": float(ver.max())},
               "task_split_mean_s": split_mean,
               "devices": sorted({(r["split"]["device"], r["split"]["slot"]) for r in res})}
        out.append(rec)
        print(json.dumps(rec), flush=True)
        shutil.rmtree(rdir, ignore_errors=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sites", type=int, default=2_400_000)
    ap.add_argument("--seeds", default="0,1")
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--concurrent", default="", help="comma list of N: every task as a process, N at once")
    ap.add_argument("--task-env", action="append", default=[], metavar="KEY=VALUE",
                    help="extra environment of the task processes (e.g. GPU_MAX_HW_QUEUES=1)")
    ap.add_argument("--server", action="store_true",
                    help="--concurrent through the node chain server (`hygeia serve`, started and stopped here)")
    ap.add_argument("--gather", type=float, default=0.0, help="the server's gather window (s)")
    ap.add_argument("--parse-cache", action="store_true",
                    help="--concurrent tasks share a parse cache (HYGEIA_PARSE_CACHE, as inside a Nextflow run)")
    a = ap.parse_args()
    if a.concurrent:
        return main_concurrent(a)
    from hygeia_amd import cli

    wd = a.workdir or tempfile.mkdtemp(prefix="hyg_pipe_")
    chrom = "1"
    t0 = time.perf_counter()
    write_inputs(wd, chrom, a.sites)
    t_write = time.perf_counter() - t0
    print(f"inputs written in {t_write:.1f} s", flush=True)
    common = ["--chrom", chrom, "--data_dir", os.path.join(wd, "data"), "--single_group_dir", os.path.join(wd, "sg")]
    seeds = [int(x) for x in a.seeds.split(",")]
    n_batches = a.sites // 100000 + 1
    units = a.sites * len(seeds)  # every site is returned by exactly one segment per seed
    t0 = time.perf_counter()
    assert cli.main(["infer_many", "--batches", "all", "--seeds", a.seeds, "--results_dir",
                     os.path.join(wd, "many")] + common) == 0
    t_many = time.perf_counter() - t0
    print(f"infer_many done in {t_many:.1f} s", flush=True)
    many_split = dict(cli.LAST_TIMINGS)
    # The unchanged Nextflow module runs one `hygeia infer` PROCESS per (batch,
    # seed) (modules/two_group/4_infer.nf:42-48): each task below is a fresh
    # Python process (interpreter start, imports, HIP initialisation included),
    # timed from outside, with the command's own phase split printed by it.
    drv = ("import json, sys, time; t0 = time.perf_counter(); from hygeia_amd import cli; t1 = time.perf_counter(); "
           "rc = cli.main(sys.argv[1:]); t2 = time.perf_counter(); "
           "print('@@' + json.dumps(dict(cli.LAST_TIMINGS, import_cli=t1 - t0, main=t2 - t1, rc=rc)), flush=True)")
    one = []
    for b, sd in ((0, seeds[0]), (n_batches // 2, seeds[-1])):
        t0 = time.perf_counter()
        r = subprocess.run([sys.executable, "-c", drv, "infer", "--batch", str(b), "--seed", str(sd), "--results_dir",
                            os.path.join(wd, "one")] + common, cwd=ROOT, capture_output=True, text=True,
                           env=dict(os.environ, PYTHONPATH=ROOT))
        wall = time.perf_counter() - t0
        if r.returncode != 0:
            raise RuntimeError(f"hygeia infer --batch {b} failed: {r.stderr[-2000:]}")
        split = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("@@")][-1][2:])
        one.append({"batch": b, "seed": sd, "process_wall_s": wall,
                    "split_s": {k: split[k] for k in ("import_cli", "parse", "device", "chains", "writes", "main") if k in split}})
        print(f"task batch {b} seed {sd}: {wall:.1f} s {one[-1]['split_s']}", flush=True)
    t_one = sum(o["process_wall_s"] for o in one) / len(one)
    tasks = n_batches * len(seeds)
    line = {"metric": "pipeline CpG sites x seeds / s (hygeia infer, gz CSV in -> result files out)",
            "sites": a.sites, "seeds": seeds, "tasks": tasks,
            "infer_many": {"value": units / t_many, "wall_s": t_many, "split_s": many_split},
            "infer_task_by_task": {"value": units / (t_one * tasks), "wall_s_one_task": t_one,
                                   "extrapolated_s": t_one * tasks, "tasks_timed": one,
                                   "note": "each task a fresh process, as the Nextflow module runs it"},
            "input_write_s": t_write}
    print(json.dumps(line), flush=True)
    if a.workdir is None:
        shutil.rmtree(wd, ignore_errors=True)


def main_concurrent(a):
    wd = a.workdir or tempfile.mkdtemp(prefix="hyg_pipe_")
    chrom = "1"
    t0 = time.perf_counter()
    write_inputs(wd, chrom, a.sites)
    print(f"inputs written in {time.perf_counter() - t0:.1f} s", flush=True)
    common = ["--chrom", chrom, "--data_dir", os.path.join(wd, "data"), "--single_group_dir", os.path.join(wd, "sg")]
    seeds = [int(x) for x in a.seeds.split(",")]
    n_batches = a.sites // 100000 + 1
    units = a.sites * len(seeds)
    many = run_task(["infer_many", "--batches", "all", "--seeds", a.seeds, "--results_dir",
                     os.path.join(wd, "many")] + common)
    print(f"infer_many {many['wall_s']:.1f} s", flush=True)
    env = dict(os.environ)
    env.update(kv.split("=", 1) for kv in a.task_env)
    env.setdefault("HYGEIA_PARSE_CACHE", os.path.join(wd, "parse_cache") if a.parse_cache else "0")
    srv, server_status = None, None
    if a.server:  # the node chain server (`hygeia serve`), started and stopped here
        from hygeia_amd import serve

        lockd = os.path.join(wd, "locks")
        os.makedirs(lockd, exist_ok=True)
        env["HYGEIA_DEVICE_LOCK_DIR"] = lockd
        path = serve.socket_path(lockd)
        srv = subprocess.Popen([sys.executable, "-m", "hygeia_amd.serve", "--socket", path, "--gather",
                                str(a.gather)], env=dict(env, PYTHONPATH=ROOT), cwd=ROOT)
        t0 = time.perf_counter()
        while not serve.connectable(path):
            if srv.poll() is not None or time.perf_counter() - t0 > 120:
                raise RuntimeError("the chain server did not start")
            time.sleep(0.1)
        print(f"server up in {time.perf_counter() - t0:.1f} s", flush=True)
    try:
        sweep = concurrent_sweep(wd, common, seeds, a.sites, n_batches, [int(x) for x in a.concurrent.split(",")],
                                 env)
        if srv is not None:
            server_status = serve.Client(path).status()
            serve.Client(path).stop()
            srv.wait(timeout=300)
    finally:
        if srv is not None and srv.poll() is None:
            srv.kill()
            srv.wait()
    line = {"metric": "pipeline CpG sites x seeds / s (hygeia infer, gz CSV in -> result files out)",
            "sites": a.sites, "seeds": seeds, "tasks": n_batches * len(seeds),
            "infer_many": {"value": units / many["wall_s"], "wall_s": many["wall_s"], "split_s": many["split"]},
            "concurrent_tasks": sweep, "task_env": a.task_env, "parse_cache": a.parse_cache,
            "server": ({"gather_s": a.gather, "status": server_status} if a.server else None),
            "note": "each task a fresh `hygeia infer` process, N at once on one GPU (Nextflow local executor)"}
    print(json.dumps(line), flush=True)
    if a.workdir is None:
        shutil.rmtree(wd, ignore_errors=True)


if __name__ == "__main__":
    main()
