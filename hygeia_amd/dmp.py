"""Aggregation and DMP calling on the MI355X path.

Drop-ins for the two consumers of `hygeia infer`'s trajectories:

  hygeia aggregate  -> src/two_group/aggregate_results.py (5_aggregate_results.nf:51-53)
  hygeia get_dmps   -> src/two_group/get_dmps.py          (6_get_dmps.nf:22-23)

with the same flags, input files and output files, and the device-side
functions behind them (C ABI hyg_dmp_*, include/hygeia_amd.h):

  site_counts()   per-site counts over the P = B x seeds trajectories of every
                  site, straight from the trajectory buffers in HBM
                  (aggregate_results.py:125-129, get_dmps.py:68-74):
                  counts [T][2 + 2K] = (#merged==0, #(r_ctrl != r_case),
                  #(r_ctrl == r)_r, #(r_case == r)_r), pairs [T][K][K]
  fdr()           multiple_testing.FDR_procedure on t = 1 - c / P
  weighted_fdr()  multiple_testing.weighted_FDR_procedure on the same t

The statistics get_dmps tests are always t = 1 - c / P for integer counts c,
so the FDR sort is a counting sort on the device and the only sequential
piece -- numpy's float64 cumsum over the sorted statistics -- is replayed
exactly by the C ABI on the host. There is no CPU path: without the HIP
library or a GPU these functions raise.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
from pathlib import Path
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib


def _torch():
    import torch

    return torch


def _stream(device):
    torch = _torch()
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def site_counts(merged, control, kase, B: int, K: int, groups: Sequence[Tuple[int, int]],
                block_rows: Sequence[Sequence[int]], n_sites: int, pairs: bool = False, counts=None, stream=None):
    """Per-site trajectory counts (device tensors in, device tensors out).

    merged [rows][B], control / kase [rows][B][2] int16 (hyg_tg_outputs layout);
    groups[g] = (site_begin, n_rows) of a segment's reported rows and
    block_rows[g][s] = the trajectory row holding that segment's first reported
    row in seed s's block. Returns (counts [n_sites][2 + 2K] int32, pairs
    [n_sites][K][K] int32 or None); rows of sites outside the groups are 0."""
    torch = _torch()
    dev = merged.device
    for a in (merged, control, kase):
        if a.dtype != torch.int16 or not a.is_contiguous() or a.device != dev:
            raise ValueError("merged/control/kase must be contiguous int16 tensors on one device")
    if counts is None:
        counts = torch.zeros((n_sites, 2 + 2 * K), dtype=torch.int32, device=dev)
    pr = torch.zeros((n_sites, K, K), dtype=torch.int32, device=dev) if pairs else None
    n_groups = len(groups)
    n_seeds = len(block_rows[0]) if n_groups else 1
    g_arr = (_lib.DmpGroup * max(n_groups, 1))(*[_lib.DmpGroup(int(a), int(b)) for a, b in groups])
    br = np.ascontiguousarray(np.asarray(block_rows, dtype=np.int64).reshape(-1))
    s = stream if stream is not None else _stream(dev)
    L = _lib.load()
    _lib.check(L.hyg_dmp_site_counts(merged.data_ptr(), control.data_ptr(), kase.data_ptr(), B, K, g_arr,
                                     br.ctypes.data_as(C.POINTER(C.c_int64)), n_groups, n_seeds, n_sites,
                                     counts.data_ptr(), pr.data_ptr() if pr is not None else None,
                                     s if isinstance(s, C.c_void_p) else C.c_void_p(s)))
    return counts, pr


def fdr(counts, column: int, n_particles: int, fdr_threshold: float, stream=None):
    """FDR_procedure (multiple_testing.py:3-12) on t_i = 1 - counts[i, column] / P.
    counts: a 2-D int32 device tensor. Returns (k, Q_k, threshold)."""
    k, q, th = C.c_int64(), C.c_double(), C.c_double()
    s = stream if stream is not None else _stream(counts.device)
    _lib.check(_lib.load().hyg_dmp_fdr(counts.data_ptr(), counts.shape[1], column, counts.shape[0], n_particles,
                                       float(fdr_threshold), C.byref(k), C.byref(q), C.byref(th), s))
    return k.value, q.value, th.value


def weighted_fdr(counts, column: int, n_particles: int, fdr_threshold: float, w_fp, w_fn, stream=None):
    """weighted_FDR_procedure (multiple_testing.py:14-22) on the same t; w_fp /
    w_fn float64 device tensors. Returns (ranking_indices[:s] as numpy int64,
    Nsums[s-1]). Ties of the ranking keep ascending site order."""
    torch = _torch()
    n = counts.shape[0]
    ranked = torch.empty(n, dtype=torch.int64, device=counts.device)
    sel, ns = C.c_int64(), C.c_double()
    s = stream if stream is not None else _stream(counts.device)
    _lib.check(_lib.load().hyg_dmp_weighted_fdr(counts.data_ptr(), counts.shape[1], column, n, n_particles,
                                                float(fdr_threshold), w_fp.data_ptr(), w_fn.data_ptr(),
                                                ranked.data_ptr(), C.byref(sel), C.byref(ns), s))
    return ranked[:sel.value].cpu().numpy(), ns.value


def regime_frequencies(counts, K: int, n_particles: int, rows: np.ndarray):
    """np.bincount(row, minlength=K) / P for the selected sites (get_dmps.py:113-120)
    from the device counts: (control [n][K], case [n][K]) float64."""
    c = counts[:, 2:2 + 2 * K].cpu().numpy()[rows].astype(np.int64)
    return c[:, :K] / n_particles, c[:, K:] / n_particles


# ---------------------------------------------------------------- get_dmps
GET_DMPS_FLAGS = [
    ("fdr_thresholds", "multi_float", [.01, .05], "fdr threshold for selecting DMPs."),
    ("results_dir", "string", os.path.join(Path(os.getcwd()).parents[0], "test"),
     "Directory for the results of the two-group algorithms."),
    ("output_dir", "string", os.path.join(Path(os.getcwd()).parents[0], "test", "dmp"),
     "Directory for the outputs of this script."),
    ("n_regimes", "int", 6, "number of regimes."),
    ("chrom", "string", "21", "The chromosome to analyze (chr22, or 22, as per input file)"),
    ("test_regime_combinations", "bool", False, "whether to test for each possible regime configuration"),
]


def _upload_regimes(regimes: np.ndarray, device):
    """[T][P] regime labels -> a (d, r) int16 trajectory block [T][P][2]."""
    torch = _torch()
    T, P = regimes.shape
    st = np.zeros((T, P, 2), dtype=np.int16)
    st[:, :, 1] = regimes
    return torch.from_numpy(st).to(device)


def get_dmps_main(argv: Sequence[str]) -> int:
    """get_dmps.py:14-180 with the statistics, FDR selections and regime
    frequencies computed on the GPU."""
    import pandas as pd
    torch = _torch()
    from .cli import parse_flags

    f = parse_flags(argv, GET_DMPS_FLAGS)
    K = int(f["n_regimes"])
    out_dir = f["output_dir"]
    os.makedirs(out_dir, exist_ok=True)
    chrom, path = f["chrom"], f["results_dir"]
    ctrl = pd.read_csv(os.path.join(path, f"control_regimes_chrom_{chrom}.csv.gz"), sep="\t")
    ctrl = ctrl.set_index("pos").to_numpy()
    case = pd.read_csv(os.path.join(path, f"case_regimes_chrom_{chrom}.csv.gz"), sep="\t")
    case = case.set_index("pos").to_numpy()
    P = ctrl.shape[-1]
    T = ctrl.shape[0]
    dev = torch.device("cuda", 0)
    c_dev, k_dev = _upload_regimes(ctrl, dev), _upload_regimes(case, dev)
    m_dev = torch.ones((T, P), dtype=torch.int16, device=dev)  # merged states are not an input here
    counts, pairs = site_counts(m_dev, c_dev, k_dev, P, K, [(0, T)], [[0]], T,
                                pairs=bool(f["test_regime_combinations"]))
    del m_dev, c_dev, k_dev
    c_host = counts.cpu().numpy().astype(np.int64)
    t_split = 1. - c_host[:, 1] / P  # get_dmps.py:68-69

    split_probs_ = pd.read_csv(os.path.join(path, f"split_probs_{chrom}.csv.gz"), sep="\t").set_index("pos")
    idx = pd.DataFrame(split_probs_.index)
    position_diffs = 1 / 3 * (idx.diff(1) + idx.diff(2) + idx.diff(3))  # :79-80
    positions = pd.DataFrame(split_probs_.index)
    positions["chrom"] = chrom
    pos_np = positions.to_numpy()
    false_negative_weights = np.squeeze(1. / (position_diffs.fillna(1e+5).to_numpy()), -1)  # :101
    w_fp = torch.ones(T, dtype=torch.float64, device=dev)
    w_fn = torch.from_numpy(np.ascontiguousarray(false_negative_weights, dtype=np.float64)).to(dev)
    pair_flat = pairs.reshape(T, K * K) if pairs is not None else None

    def dmp_frame(sel_rows, stats, fn_weight):
        dmp_pos = pos_np[sel_rows]
        d = pd.DataFrame({"chrom": dmp_pos[:, 1], "position": dmp_pos[:, 0], "null_stats": stats})
        d["false_negative_weight"] = fn_weight
        return d

    def with_freqs(d, rows):
        fc, fk = regime_frequencies(counts, K, P, rows)
        dc = pd.DataFrame(fc, columns=["Control_METEOR_{}".format(i + 1) for i in range(K)])
        dk = pd.DataFrame(fk, columns=["Case_METEOR_{}".format(i + 1) for i in range(K)])
        return pd.concat([d, dc, dk], axis=1)

    for thr in f["fdr_thresholds"]:
        k, Qk, threshold = fdr(counts, 1, P, thr)
        ind = t_split < threshold
        rows = np.nonzero(ind)[0]
        d = with_freqs(dmp_frame(ind, t_split[ind], 1.), rows)
        d.to_csv(os.path.join(out_dir, "dmp_{}.csv".format(thr)), index=False, float_format="%.4f")
        if pair_flat is not None:
            for i in range(K):
                for j in range(K):
                    if i != j:
                        t_ij = 1 - pairs[:, i, j].cpu().numpy().astype(np.int64) / P
                        k, Qk, th = fdr(pair_flat, i * K + j, P, thr)
                        ind_ij = t_ij < th
                        dmp_frame(ind_ij, t_ij[ind_ij], 1.).to_csv(
                            os.path.join(out_dir, "dmp_{}_{}_{}.csv".format(i, j, thr)), index=False)
        # weighted versions (:142-166)
        dmp_index, Nk = weighted_fdr(counts, 1, P, thr, w_fp, w_fn)
        dmp_index = np.sort(dmp_index)
        d = dmp_frame(dmp_index, t_split[dmp_index], false_negative_weights[dmp_index])
        d = with_freqs(d, dmp_index)
        d.to_csv(os.path.join(out_dir, "weighted_dmp_{}.csv".format(thr)), index=False, float_format="%.4f")
        if pair_flat is not None:
            for i in range(K):
                for j in range(K):
                    if i != j:
                        t_ij = 1 - pairs[:, i, j].cpu().numpy().astype(np.int64) / P
                        di, _ = weighted_fdr(pair_flat, i * K + j, P, thr, w_fp, w_fn)
                        di = np.sort(di)
                        dmp_frame(di, t_ij[di], false_negative_weights[di]).to_csv(
                            os.path.join(out_dir, "weighted_dmp_{}_{}_{}.csv".format(i, j, thr)), index=False)
    return 0


# --------------------------------------------------------------- aggregate
AGGREGATE_FLAGS = [
    ("results_dir", "string", os.path.join(Path(os.getcwd()).parents[0], "test"),
     "Directory for the results of the two-group algorithms."),
    ("output_dir", "string", os.path.join(Path(os.getcwd()).parents[0], "test", "results"),
     "Directory for the outputs of this script."),
    ("seeds", "int", 10, "Number of seeds that algorithms have been run."),
    ("chrom", "string", "22", "The chromosome to analyze (chr22, or 22, as per input file)"),
    ("num_batches", "int", 30, "maximum number of batches"),
    ("num_particles", "int", 2400, "number of particles from backward smoothing"),
    ("compute_freqs", "bool", False, "whether to compute freqs of METEOR regimes (takes some time)"),
]


def aggregate_main(argv: Sequence[str]) -> int:
    """aggregate_results.py:14-215: per-batch trajectories of every seed are
    concatenated along the particle axis and written per chromosome; the split
    probabilities (mean over particles of merged == 0) come from the device
    counts kernel."""
    import pandas as pd
    torch = _torch()
    from .cli import parse_flags

    f = parse_flags(argv, AGGREGATE_FLAGS)
    N = f["num_particles"]
    out_dir = f["output_dir"]
    print(f"Results directory: {f['results_dir']}")
    print(f"Output directory: {out_dir}")
    os.makedirs(out_dir, exist_ok=True)
    chrom = f["chrom"]
    print(f"Processing chromosome: {chrom}")
    dev = torch.device("cuda", 0)
    lists = {k: [] for k in ("split", "pos", "merge", "creg", "kreg", "cdur", "kdur", "ntc", "ntk", "obc", "obk")}
    processed = 0
    for batch in range(0, f["num_batches"]):
        data_dir = os.path.join(f["results_dir"], "chrom_{}_{}".format(chrom, batch))
        print(f"\nProcessing batch {batch}")
        if not os.path.exists(data_dir):
            print(f"Directory does not exist: {data_dir}")
            break
        positions_file = os.path.join(data_dir, "positions.csv.gz")
        if not os.path.isfile(positions_file):
            print(f"positions.csv.gz not found in {data_dir}")
            break
        positions__ = pd.read_table(positions_file, sep=" ", header=None, dtype=np.int64)
        # aggregate_results.py:98-105 reads these with sep=' ', which cannot split
        # infer's comma-separated rows (run_inference_two_groups.py:245-252) once a
        # group has two or more samples (its .astype(np.int16) then raises); read
        # them with the delimiter they are written with (same frames for one sample)
        rd = lambda name: pd.read_table(os.path.join(data_dir, name), sep=",", header=None)  # noqa: E731
        ntc, ntk = rd("n_total_reads_control.csv.gz"), rd("n_total_reads_case.csv.gz")
        obc, obk = rd("observations_control.csv.gz"), rd("observations_case.csv.gz")
        m_, c_, k_ = [], [], []
        for seed in range(0, f["seeds"]):
            ld = lambda kind: np.load(os.path.join(  # noqa: E731
                data_dir, "optimal_backward_particles_{}_state_{}_{}.npz".format(kind, N, seed)))["arr_0"]
            m_.append(ld("merged"))
            c_.append(ld("control"))
            k_.append(ld("case"))
        print(f"Successfully processed {len(m_)} seeds out of {f['seeds']}")
        merged = np.concatenate(m_, -1)
        control = np.concatenate(c_, axis=1)
        case = np.concatenate(k_, axis=1)
        T, P = merged.shape
        K = int(max(control[..., 1].max(initial=0), case[..., 1].max(initial=0))) + 1
        to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int16)).to(dev)  # noqa: E731
        counts, _ = site_counts(to_dev(merged), to_dev(control), to_dev(case), P, min(K, 16), [(0, T)], [[0]], T)
        split = counts[:, 0].cpu().numpy().astype(np.int64) / P  # np.mean(merged == 0, axis=1) (:129)
        lists["split"].append(pd.DataFrame(split))
        lists["pos"].append(positions__.iloc[0:T])
        lists["merge"].append(pd.DataFrame(merged).astype(np.int8))
        lists["creg"].append(pd.DataFrame(control[:, :, 1]).astype(np.int8))
        lists["kreg"].append(pd.DataFrame(case[:, :, 1]).astype(np.int8))
        lists["cdur"].append(pd.DataFrame(control[:, :, 0]).astype(np.int16))
        lists["kdur"].append(pd.DataFrame(case[:, :, 0]).astype(np.int16))
        lists["ntc"].append(pd.DataFrame(ntc[0:T]).astype(np.int16))
        lists["ntk"].append(pd.DataFrame(ntk[0:T]).astype(np.int16))
        lists["obc"].append(pd.DataFrame(obc[0:T]).astype(np.int16))
        lists["obk"].append(pd.DataFrame(obk[0:T]).astype(np.int16))
        processed += 1
        print(f"Successfully processed batch {batch}")
    print(f"\nProcessing complete. Successfully processed {processed} batches")
    if not lists["pos"]:
        print("No data was processed. Check the input directories and file paths.")
        return 1
    pos = pd.concat(lists["pos"]).rename(columns={0: "pos"}).astype(np.int32)

    def write(key, name):
        d = pd.concat(lists[key]).set_index(pos["pos"])
        d.to_csv(os.path.join(out_dir, name.format(chrom)), sep="\t", compression="gzip")
        return d

    creg_chrom = write("creg", "control_regimes_chrom_{}.csv.gz")
    kreg_chrom = write("kreg", "case_regimes_chrom_{}.csv.gz")
    merge_chrom = write("merge", "merge_states_chrom_{}.csv.gz")
    # split_probs_chrom = np.mean(merge_states_chrom == 0, axis=1) (:181): from the device counts
    m = torch.from_numpy(np.ascontiguousarray(merge_chrom.to_numpy(), dtype=np.int16)).to(dev)
    Tc, Pc = m.shape
    z = torch.zeros((Tc, Pc, 2), dtype=torch.int16, device=dev)
    cnt, _ = site_counts(m, z, z, Pc, 1, [(0, Tc)], [[0]], Tc)
    split_chrom = pd.Series(cnt[:, 0].cpu().numpy().astype(np.int64) / Pc, index=merge_chrom.index)
    split_chrom.to_csv(os.path.join(out_dir, "split_probs_{}.csv.gz".format(chrom)), sep="\t", compression="gzip")
    write("ntc", "n_total_reads_control_chrom_{}.csv.gz")
    write("ntk", "n_total_reads_case_chrom_{}.csv.gz")
    write("obc", "n_meth_reads_control_chrom_{}.csv.gz")
    write("obk", "n_meth_reads_case_chrom_{}.csv.gz")
    write("cdur", "control_durations_chrom_{}.csv.gz")
    write("kdur", "case_durations_chrom_{}.csv.gz")
    if f["compute_freqs"]:
        # aggregate_results.py:208-215: per site, value_counts(normalize=True) of
        # the regimes over all particles; the frame pandas assembles has one
        # column per regime seen at any site (sorted labels), NaN where a row
        # has none. The regime histograms come from the device counts kernel.
        cr = torch.from_numpy(np.ascontiguousarray(creg_chrom.to_numpy(), dtype=np.int16)).to(dev)
        kr = torch.from_numpy(np.ascontiguousarray(kreg_chrom.to_numpy(), dtype=np.int16)).to(dev)
        Kf = int(max(int(cr.max().item()), int(kr.max().item()))) + 1
        if Kf > 16 or int(min(cr.min().item(), kr.min().item())) < 0:
            raise ValueError("regime labels outside [0, 16)")
        ctl = torch.stack([torch.zeros_like(cr), cr], dim=2).contiguous()
        cas = torch.stack([torch.zeros_like(kr), kr], dim=2).contiguous()
        cnt, _ = site_counts(torch.zeros_like(cr), ctl, cas, Pc, Kf, [(0, Tc)], [[0]], Tc)
        cnt = cnt.cpu().numpy().astype(np.int64)
        for g, name in ((1, "case_regimes_freq_{}.csv"), (0, "control_regimes_freq_{}.csv")):
            h = cnt[:, 2 + g * Kf:2 + (g + 1) * Kf]
            seen = [r for r in range(Kf) if h[:, r].any()]
            fr = pd.DataFrame({r: np.where(h[:, r] > 0, h[:, r] / Pc, np.nan) for r in seen},
                              index=creg_chrom.index)
            fr.to_csv(os.path.join(out_dir, name.format(chrom)), sep="\t")
    return 0
