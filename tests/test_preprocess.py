"""SURVEY.md 8f-3 on CPU: a restatement of src/two_group/preprocess_bed.py's
join semantics (polars 1.8.2 full joins, strand collapse, rounding) written
here with pandas, checked on hand-computed cases; the flag validation of
`hygeia preprocess`. The device path is compared with this restatement in
tests/test_gpu_preprocess.py. polars is absent, so against the reference
itself the outputs are parity unpinned (the restatement follows its source)."""
import gzip
import math
import os

import numpy as np
import pandas as pd
import pytest

from hygeia_amd import cli

COLS = ["chr", "start", "end", "name", "score", "strand", "thickStart", "thickEnd", "itemRgb", "coverage",
        "percent_methylated", "ref_genotype", "sample_genotype", "quality_score"]


def polars_round(x):
    """Rust f64::round (half away from zero)"""
    return np.sign(x) * np.floor(np.abs(x) + 0.5)


def ref_collapse(bed: pd.DataFrame, chrom: str) -> pd.DataFrame:
    """read_bed_file filter (:160-168) + collapse_strands (:183-259)"""
    b = bed[(bed["chr"].astype(str) == chrom) & (bed["ref_genotype"] == "CG")]
    pos, neg = b[b["strand"] == "+"], b[b["strand"] == "-"]
    m = pos.merge(neg, left_on=["chr", "end"], right_on=["chr", "start"], how="outer", suffixes=("", "_neg"))
    cp = m["coverage"].fillna(0).astype(float)
    cn = m["coverage_neg"].fillna(0).astype(float)
    pp = m["percent_methylated"].fillna(0).astype(float)
    pn = m["percent_methylated_neg"].fillna(0).astype(float)
    total = cp + cn
    start = m["start"].where(m["start"].notna(), m["start_neg"] - 1)
    keep = total > 0
    avg = ((cp * pp) + (cn * pn)) / total
    return pd.DataFrame({"start": start[keep].astype(np.int64), "total": total[keep], "avg": avg[keep]})


def ref_counts(cpg_pos0, beds, chrom):
    """process_sample_data + the Pos0 joins + extract_count_arrays: per sample
    (meth, unmeth) on the CpG grid, NaN where the sample has no collapsed row."""
    out = np.full((len(cpg_pos0), 2 * len(beds)), np.nan)
    idx = {int(p): i for i, p in enumerate(cpg_pos0)}
    for s, bed in enumerate(beds):
        if bed is None:
            continue
        c = ref_collapse(bed, chrom)
        meth = polars_round((c["total"] * c["avg"]) / 100.0)
        unmeth = polars_round((c["total"] * (100.0 - c["avg"])) / 100.0)
        for k, a, b in zip(c["start"], meth, unmeth):
            if int(k) in idx:
                out[idx[int(k)], 2 * s] = a
                out[idx[int(k)], 2 * s + 1] = b
    return out


def bed_rows(rows):
    """rows of (chr, start, end, strand, coverage, percent, ref)"""
    return pd.DataFrame([[c, s, e, ".", 0, st, s, e, "0,0,0", cov, pct, ref, "CG", 30]
                         for c, s, e, st, cov, pct, ref in rows], columns=COLS)


def test_restatement_hand_cases():
    bed = bed_rows([
        ("22", 100, 101, "+", 3, 50.0, "CG"),    # paired with the "-" at 101: total 5, avg 40 -> 2, 3
        ("22", 101, 102, "-", 2, 25.0, "CG"),
        ("22", 200, 201, "+", 5, 50.0, "CG"),    # "+" only: 2.5 -> 3 (half away from zero), 2.5 -> 3
        ("22", 301, 302, "-", 4, 100.0, "CG"),   # "-" only: key 300
        ("22", 400, 401, "+", 0, 0.0, "CG"),     # coverage 0: dropped (null -> 0, NaN here)
        ("22", 500, 501, "+", 9, 10.0, "CH"),    # not CG
        ("21", 600, 601, "+", 9, 10.0, "CG"),    # other chromosome
        ("22", 700, 701, "+", 7, 30.0, "CG"),    # not a CpG site of the grid: dropped
    ])
    got = ref_counts(np.array([100, 200, 300, 400, 500, 600, 900]), [bed], "22")
    exp = [[2, 3], [3, 3], [4, 0], [np.nan, np.nan], [np.nan, np.nan], [np.nan, np.nan], [np.nan, np.nan]]
    np.testing.assert_array_equal(got, np.array(exp, float))
    assert polars_round(np.array([0.5, 1.5, 2.5, -0.5]))[2] == 3.0


def test_flag_validation(tmp_path, capsys):
    assert cli.main(["preprocess", "--chromosome", "22"]) == 1  # no --cpg_file_path
    assert cli.main(["preprocess", "--cpg_file_path", str(tmp_path / "x.tsv")]) == 1  # no samples
    assert cli.main(["preprocess", "--cpg_file_path", str(tmp_path / "x.tsv"), "--case_data_path", "a.bed",
                     "--case_id_names", "a", "--case_id_names", "b"]) == 1  # names != paths
    assert cli.main(["preprocess", "--cpg_file_path", str(tmp_path / "missing.tsv"),
                     "--control_data_path", "a.bed"]) == 1  # CpG file not found
    assert cli.main(["preprocess", "--bogus", "1"]) == 1
