"""Downstream plumbing of SURVEY.md 8f-4 on the MI355X path.

* `hygeia make_bed_file --chr C --regimes_file F --output_file O`: drop-in for
  src/single_group/bin/make_bed_file (run by
  modules/single_group/4_generate_single_group_bed_files.nf:24-27). The regimes
  CSV (genomic_position, regime_1..K; bin/estimate_parameters_and_regimes:325-338)
  goes to the device, `hyg_bed_labels` finds per site the largest probability
  and its regime or "equiprobable" (make_bed_file:27-39), and the native
  formatter `hyg_bed_format` writes the 9-column BED lines in start order
  (:41-63): chrom, pos-1, pos+1, name, score, ".", pos-1, pos+1, itemRgb.
* `hygeia get_chrom_segments --input_file P --chromosome C --segment_size S
  --output_csv O`: drop-in for src/two_group/get_chrom_segments.py (run by
  modules/two_group/3_get_chrom_segments.nf:46-48): 1 + n // S segment rows
  `chrom,segment_index` (the batches `hygeia infer --batch` is called with).

Against R / data.table the BED text is parity unpinned (R is absent here):
tests/test_bed.py pins it against a restatement of the R logic, and the score
uses printf's %.15g (fwrite writes at most 15 significant digits).
"""
from __future__ import annotations

import ctypes as C
import gzip
import os
import sys
from typing import Sequence

import numpy as np

from . import _lib

# make_bed_file:45-48 (the reference's colours assume six regimes)
ITEM_RGB = ("248,118,109", "183,159,0", "0,186,56", "0,191,196", "97,156,255", "245,100,227", "128,128,128")


def _argparser_flags(argv: Sequence[str], names: Sequence[str]) -> dict:
    """argparser (R) style: --name value or --name=value; unknown flags are errors."""
    out, i = {}, 0
    argv = list(argv)
    while i < len(argv):
        a = argv[i]
        if not a.startswith("--"):
            raise ValueError(f"unexpected argument {a!r}")
        name, eq, val = a[2:].partition("=")
        if name not in names:
            raise ValueError(f"unknown flag --{name}")
        if not eq:
            if i + 1 >= len(argv):
                raise ValueError(f"--{name} needs a value")
            val = argv[i + 1]
            i += 1
        out[name] = val
        i += 1
    return out


def labels(probs: np.ndarray):
    """(label int8 [-1 = equiprobable], score f64) per row of probs [n][K], on the device."""
    import torch

    L = _lib.load()
    if L.hyg_device_count() < 1:
        raise RuntimeError("hyg_bed_labels needs a HIP device (hygeia_amd has no CPU fallback)")
    n, K = probs.shape
    dev = torch.device("cuda", 0)
    p = torch.from_numpy(np.ascontiguousarray(probs, np.float64)).to(dev)
    lab = torch.empty(n, dtype=torch.int8, device=dev)
    sc = torch.empty(n, dtype=torch.float64, device=dev)
    stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(L.hyg_bed_labels(p.data_ptr(), K, n, lab.data_ptr(), sc.data_ptr(), stream))
    torch.cuda.synchronize(dev)
    return lab.cpu().numpy(), sc.cpu().numpy()


def format_bed(chrom: str, positions: np.ndarray, label: np.ndarray, score: np.ndarray, names, rgb) -> bytes:
    """The BED text through the native formatter (hyg_bed_format)."""
    L = _lib.load()
    K = len(names) - 1
    pos = np.ascontiguousarray(positions, np.int64)
    lab = np.ascontiguousarray(label, np.int8)
    sc = np.ascontiguousarray(score, np.float64)
    nm = (C.c_char_p * (K + 1))(*[s.encode() for s in names])
    cl = (C.c_char_p * (K + 1))(*[s.encode() for s in rgb])
    ptr = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    need = L.hyg_bed_format(chrom.encode(), ptr(pos), ptr(lab), ptr(sc), len(pos), K, nm, cl, None, 0)
    if need < 0:
        raise RuntimeError(L.hyg_last_error().decode())
    buf = C.create_string_buffer(max(int(need), 1))
    got = L.hyg_bed_format(chrom.encode(), ptr(pos), ptr(lab), ptr(sc), len(pos), K, nm, cl, buf, need)
    if got != need:
        raise RuntimeError(L.hyg_last_error().decode())
    return buf.raw[:need]


def read_regimes(path: str):
    """regimes CSV of estimate_parameters_and_regimes (R format(): values may carry
    leading spaces): positions int64 [n], probabilities [n][K], the regime column names."""
    import pandas as pd

    df = pd.read_csv(path, skipinitialspace=True)
    cols = [c for c in df.columns if c != "genomic_position"]
    return (df["genomic_position"].to_numpy(np.int64), df[cols].to_numpy(np.float64), cols)


def make_bed_file_main(argv: Sequence[str]) -> int:
    try:
        f = _argparser_flags(argv, ("chr", "regimes_file", "output_file"))
    except ValueError as e:
        print(f"Error: {e}", file=sys.stderr)
        return 1
    for k in ("chr", "regimes_file", "output_file"):
        if k not in f:
            print(f"Error: missing --{k}", file=sys.stderr)
            return 1
    pos, probs, cols = read_regimes(f["regimes_file"])
    if len(cols) + 1 != len(ITEM_RGB):
        # data.table(regime = c(regime_cols, "equiprobable"), itemRgb = <7 colours>) (make_bed_file:45-48)
        print(f"Error: the BED colours are defined for {len(ITEM_RGB) - 1} regimes, not {len(cols)}",
              file=sys.stderr)
        return 1
    lab, sc = labels(probs)
    order = np.argsort(pos - 1, kind="stable")  # setkey(bed, chr, start)
    text = format_bed(f["chr"], pos[order], lab[order], sc[order], list(cols) + ["equiprobable"], ITEM_RGB)
    out_dir = os.path.dirname(f["output_file"])
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
    with open(f["output_file"], "wb") as fh:
        fh.write(text)
    print(f"Completed processing for chromosome {f['chr']}", file=sys.stderr)
    return 0


GET_CHROM_SEGMENTS_FLAGS = [
    ("input_file", "string", "positions.txt", "input (gzipped) chromosome positions"),
    ("chromosome", "string", "22", "the chromosome to analyze"),
    ("segment_size", "int", 100000, "size of the selected chromosome segment (in CpG sites)"),
    ("output_csv", "string", "chrom_segments.csv", "output CSV with the segment information"),
]


def get_chrom_segments_main(argv: Sequence[str]) -> int:
    """get_chrom_segments.py:23-43: num_segments = 1 + n_positions // segment_size."""
    from .cli import parse_flags

    fl = parse_flags(argv, GET_CHROM_SEGMENTS_FLAGS)
    with gzip.open(fl["input_file"], "rb") as fh:
        n = sum(1 for line in fh if line.strip())
    num_segments = 1 + n // int(fl["segment_size"])
    out_dir = os.path.dirname(fl["output_csv"])
    if out_dir and not os.path.exists(out_dir):
        os.makedirs(out_dir)
    with open(fl["output_csv"], "w") as fh:
        fh.write("chrom,segment_index\n")
        for i in range(num_segments):
            fh.write(f"{fl['chromosome']},{i}\n")
    print(f"Segment information saved to {fl['output_csv']}")
    return 0
