"""`hygeia preprocess` on the MI355X path: a drop-in for
src/two_group/preprocess_bed.py as modules/two_group/1_preprocess.nf:39-41 runs
it. Same absl flags (:25-63), inputs (a tab-separated CpG file with `seqID`
and `start` columns; per-sample per-strand methylation BED files with a header
row and >= 14 columns, :128-149) and outputs in --output_path
(`{positions, cpg_sites_merged, n_methylated_reads_{control,case},
n_total_reads_{control,case}}_{chromosome}.txt.gz`, np.savetxt fmt '%s',
:420-456) -- the inputs of `hygeia infer`.

The text is parsed on the host (pandas; the reference uses polars 1.8.2,
absent here); the strand collapse and the counts on the CpG grid run on the
device (hyg_pre_collapse, hygeia_amd/csrc/pre_kernels.hip), one sample at a
time into its own [sites][2] block in HBM. Reference behaviours kept:
* sites of a sample that are not CpG sites of the CpG file are dropped (the
  full joins give them a null Pos0, :365-369), CpG sites a sample lacks are 0
  (np.nan_to_num, :384); a missing sample file gives 0 columns (:281-287);
* counts = round(total * avg / 100) half away from zero (polars f64 round);
* the count matrices print as floats ("12.0") when any site is missing in any
  sample (polars turns null-bearing Int64 columns into float64), else as ints.
Records longer than one base that make two collapsed rows share a key, and
duplicate starts within a strand, are rejected (the reference would multiply
rows in its joins).
"""
from __future__ import annotations

import ctypes as C
import logging
import os
import sys
from pathlib import Path
from typing import List, Sequence

import numpy as np

from . import _lib

logger = logging.getLogger("hygeia.preprocess")

FLAGS_SPEC = [
    ("cpg_file_path", "string", None, "Path to file containing all CpG sites."),
    ("output_path", "string", os.path.join(Path.cwd().parent, "test"), "Directory where to store the results."),
    ("case_data_path", "multi_string", [], "Paths for the methylation data of the case group (BED format)."),
    ("case_id_names", "multi_string", [], "Names of case IDs in methylation files."),
    ("control_data_path", "multi_string", [], "Paths for the methylation data of the control group (BED format)."),
    ("control_id_names", "multi_string", [], "Names of control IDs in methylation files."),
    ("chromosome", "string", "22", "The chromosome to analyze (chr22, or 22, as per input file)"),
    ("verbose", "bool", False, "Enable verbose logging"),
]

BED_COLUMNS = ["chr", "start", "end", "name", "score", "strand", "thickStart", "thickEnd", "itemRgb", "coverage",
               "percent_methylated", "ref_genotype", "sample_genotype", "quality_score"]


def load_cpg_positions(path: str, chromosome: str) -> np.ndarray:
    """load_cpg_sites (:94-121): rows with str(seqID) == chromosome; Pos0 = start - 1."""
    import pandas as pd

    df = pd.read_csv(path, sep="\t", dtype={"seqID": str})
    pos0 = df.loc[df["seqID"].astype(str) == chromosome, "start"].to_numpy(np.int64) - 1
    if pos0.size == 0:
        raise ValueError(f"No CpG sites found for chromosome {chromosome}")
    return pos0


def read_bed(path: str, chromosome: str):
    """read_bed_file (:123-181): header row skipped, the first 14 columns, rows of
    the chromosome with ref_genotype CG; returns the "+" and "-" records
    (start, end, coverage, percent) sorted by start."""
    import pandas as pd

    df = pd.read_csv(path, sep="\t", skiprows=1, header=None, usecols=range(14), names=BED_COLUMNS,
                     dtype={"chr": str, "strand": str, "ref_genotype": str})
    df = df[(df["chr"].astype(str) == chromosome) & (df["ref_genotype"] == "CG")]
    out = []
    for strand in ("+", "-"):
        s = df[df["strand"] == strand]
        start = s["start"].to_numpy(np.int64)
        order = np.argsort(start, kind="stable")
        start = start[order]
        if start.size > 1 and not np.all(np.diff(start) > 0):
            raise ValueError(f"{path}: duplicate {strand} strand starts on chromosome {chromosome}")
        out.append((start, s["end"].to_numpy(np.int64)[order], s["coverage"].to_numpy(np.float64)[order],
                    s["percent_methylated"].to_numpy(np.float64)[order]))
    return out, len(df)


def collapse_on_device(pos0_dev, strands, counts_dev, stream) -> None:
    """hyg_pre_collapse for one sample into its contiguous counts block [sites][2]."""
    import torch

    L = _lib.load()
    dev = pos0_dev.device
    (ps, pe, pc, pp), (ms, _me, mc, mp) = strands
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d = [t(x) for x in (ps, pe, pc, pp, ms, mc, mp)]
    single = int(bool(np.all(pe == ps + 1)))  # single-base "+" records: no marking pass
    scratch = torch.empty(max(len(ms), 1), dtype=torch.uint8, device=dev)
    conflicts = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.check(L.hyg_pre_collapse(pos0_dev.data_ptr(), pos0_dev.numel(), d[0].data_ptr(), d[1].data_ptr(),
                                  d[2].data_ptr(), d[3].data_ptr(), len(ps), d[4].data_ptr(), d[5].data_ptr(),
                                  d[6].data_ptr(), len(ms), single, scratch.data_ptr(), counts_dev.data_ptr(), 2, 0,
                                  conflicts.data_ptr(), stream))
    if int(conflicts.item()) != 0:
        raise ValueError(f"{int(conflicts.item())} CpG sites claimed by two collapsed rows (records longer "
                         "than one base are not supported)")


def process(cpg_file_path: str, output_path: str, chromosome: str, case_paths: List[str], case_ids: List[str],
            control_paths: List[str], control_ids: List[str]) -> int:
    """MethylationBEDProcessor.process (:477-543) + save_results (:405-456)."""
    import torch

    L = _lib.load()
    if L.hyg_device_count() < 1:
        raise RuntimeError("hygeia preprocess needs a HIP device (hygeia_amd has no CPU fallback)")
    out_dir = Path(output_path)
    out_dir.mkdir(parents=True, exist_ok=True)
    pos0 = np.sort(load_cpg_positions(cpg_file_path, chromosome), kind="stable")
    dev = torch.device("cuda", 0)
    stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    samples = [(p, i) for p, i in zip(control_paths, control_ids)] + [(p, i) for p, i in zip(case_paths, case_ids)]
    T = pos0.size
    pos0_dev = torch.from_numpy(pos0).to(dev)
    counts = torch.full((len(samples), T, 2), float("nan"), dtype=torch.float64, device=dev)  # per sample [T][2]
    for s, (path, sid) in enumerate(samples):
        logger.info(f"Processing sample: {sid}")
        if not Path(path).exists():
            logger.error(f"File not found: {path}")
            continue
        strands, n_rows = read_bed(path, chromosome)
        if n_rows == 0:
            logger.warning(f"No CpG data found for {sid} on chromosome {chromosome}")
            continue
        collapse_on_device(pos0_dev, strands, counts[s], stream)
    data = counts.permute(1, 0, 2).reshape(T, 2 * len(samples)).cpu().numpy()  # [T][(meth, unmeth) per sample]
    has_null = bool(np.isnan(data).any())
    data = np.nan_to_num(data, copy=False)
    if not has_null:  # polars hands out an Int64 matrix when no value is null
        data = data.astype(np.int64)
    n_ctrl = len(control_ids) if control_paths else 0
    files = {"positions": pos0, "cpg_sites_merged": np.array([T])}
    if n_ctrl:
        meth, unmeth = data[:, 0:2 * n_ctrl:2], data[:, 1:2 * n_ctrl:2]
        files["n_methylated_reads_control"] = meth
        files["n_total_reads_control"] = unmeth + meth
    if case_paths:
        meth, unmeth = data[:, 2 * n_ctrl::2], data[:, 2 * n_ctrl + 1::2]
        files["n_methylated_reads_case"] = meth
        files["n_total_reads_case"] = unmeth + meth
    for name, arr in files.items():
        np.savetxt(out_dir / f"{name}_{chromosome}.txt.gz", arr, delimiter=",", fmt="%s")
    return T


def main(argv: Sequence[str]) -> int:
    from .cli import parse_flags

    fl = parse_flags(argv, FLAGS_SPEC)
    logging.basicConfig(level=logging.DEBUG if fl["verbose"] else logging.INFO,
                        format="%(asctime)s - %(levelname)s - %(message)s")
    try:
        # validate_flags (:546-569)
        if not fl["cpg_file_path"]:
            raise ValueError("Required flag --cpg_file_path not provided")
        case_p, case_i = list(fl["case_data_path"]), list(fl["case_id_names"])
        ctrl_p, ctrl_i = list(fl["control_data_path"]), list(fl["control_id_names"])
        if not case_p and not ctrl_p:
            raise ValueError("Must provide either case samples, control samples, or both")
        if case_p:
            if case_i and len(case_p) != len(case_i):
                raise ValueError("Number of case data paths must match number of case ID names")
            case_i = case_i or [f"case_{i}" for i in range(len(case_p))]
        if ctrl_p:
            if ctrl_i and len(ctrl_p) != len(ctrl_i):
                raise ValueError("Number of control data paths must match number of control ID names")
            ctrl_i = ctrl_i or [f"control_{i}" for i in range(len(ctrl_p))]
        if not Path(fl["cpg_file_path"]).exists():
            raise FileNotFoundError(f"CpG file not found: {fl['cpg_file_path']}")
        n = process(fl["cpg_file_path"], fl["output_path"], fl["chromosome"], case_p, case_i, ctrl_p, ctrl_i)
        print(f"Successfully processed {n} CpG sites for chromosome {fl['chromosome']}")
    except Exception as e:  # the reference logs and returns 1 (:585-587)
        logger.error(f"Processing failed: {e}")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
