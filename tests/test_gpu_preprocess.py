"""SURVEY.md 8f-3 on the GPU: `hygeia preprocess` end to end (host parse,
hyg_pre_collapse on the device, np.savetxt outputs) against the restatement of
preprocess_bed.py in tests/test_preprocess.py, file by file, on synthetic
per-strand BED files: paired and single-strand CpGs, zero coverage, non-CG and
other-chromosome rows, sites outside the CpG grid, half-integer roundings,
extra columns, a missing sample file, and the all-covered case (int output)."""
import gzip

import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from tests.test_preprocess import COLS, ref_counts  # noqa: E402


@pytest.fixture(scope="module")
def lib():
    from hygeia_amd import _lib

    L = _lib.load()
    if L.hyg_device_count() <= 0:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X (gpurun)")
    return L


def synth(n_cpg, seed, chrom="22", full=False):
    rng = np.random.default_rng(seed)
    cpg1 = np.cumsum(rng.integers(2, 40, n_cpg)) + 1000  # 1-based C positions
    beds = []
    for s in range(3):
        rows = []
        for p in cpg1 - 1:  # 0-based C
            r = rng.random()
            cov_p, cov_n = int(rng.integers(0, 30)), int(rng.integers(0, 30))
            pct_p, pct_n = float(rng.choice([0.0, 50.0, 100.0, round(rng.random() * 100, 2)])), \
                float(round(rng.random() * 100, 2))
            if full:
                cov_p = max(cov_p, 1)
                r = 0.0
            if r < 0.6:
                rows += [(chrom, p, p + 1, "+", cov_p, pct_p, "CG"), (chrom, p + 1, p + 2, "-", cov_n, pct_n, "CG")]
            elif r < 0.75:
                rows.append((chrom, p, p + 1, "+", cov_p, pct_p, "CG"))
            elif r < 0.9:
                rows.append((chrom, p + 1, p + 2, "-", cov_n, pct_n, "CG"))
            elif r < 0.95:
                rows.append((chrom, p, p + 1, "+", cov_p, pct_p, "CHG"))
        if not full:
            rows += [("21", 5, 6, "+", 4, 50.0, "CG"), (chrom, int(cpg1[-1]) + 100, int(cpg1[-1]) + 101, "+", 3, 50.0,
                                                          "CG")]
        beds.append(pd.DataFrame([[c, a, b, ".", 0, st, a, b, "0,0,0", cv, pc, rf, "CG", 30, "extra"]
                                  for c, a, b, st, cv, pc, rf in rows], columns=COLS + ["x"]))
    return cpg1, beds


def write_inputs(tmp, cpg1, beds, chrom):
    cpg = pd.DataFrame({"seqID": [chrom] * len(cpg1) + ["21"], "start": list(cpg1) + [6], "end": 0})
    cpg.to_csv(tmp / "cpg.tsv", sep="\t", index=False)
    paths = []
    for s, b in enumerate(beds):
        p = tmp / f"s{s}.bed"
        with open(p, "w") as fh:
            fh.write("track header\n")
            b.to_csv(fh, sep="\t", index=False, header=False)
        paths.append(str(p))
    return paths


def read_out(path):
    with gzip.open(path, "rt") as fh:
        return fh.read()


@pytest.mark.parametrize("full", [False, True])
def test_preprocess_end_to_end(lib, tmp_path, full):
    from hygeia_amd import cli

    chrom = "22"
    cpg1, beds = synth(3000, 7 + full, chrom, full=full)
    paths = write_inputs(tmp_path, cpg1, beds, chrom)
    ctrl = [paths[0], str(tmp_path / "missing.bed")] if not full else [paths[0]]
    case = [paths[1], paths[2]]
    argv = ["preprocess", "--cpg_file_path", str(tmp_path / "cpg.tsv"), "--output_path", str(tmp_path / "out"),
            "--chromosome", chrom]
    for p in ctrl:
        argv += ["--control_data_path", p]
    for i, p in enumerate(case):
        argv += ["--case_data_path", p, "--case_id_names", f"k{i}"]
    assert cli.main(argv) == 0
    pos0 = np.sort(cpg1 - 1)
    ref = ref_counts(pos0, [beds[0]] + ([None] if not full else []) + [beds[1], beds[2]], chrom)
    has_null = np.isnan(ref).any()
    assert has_null != full
    ref = np.nan_to_num(ref)
    if not has_null:
        ref = ref.astype(np.int64)
    nc = len(ctrl)
    exp = {"positions": pos0, "cpg_sites_merged": np.array([len(pos0)]),
           "n_methylated_reads_control": ref[:, 0:2 * nc:2],
           "n_total_reads_control": ref[:, 1:2 * nc:2] + ref[:, 0:2 * nc:2],
           "n_methylated_reads_case": ref[:, 2 * nc::2], "n_total_reads_case": ref[:, 2 * nc + 1::2] + ref[:, 2 * nc::2]}
    for name, arr in exp.items():
        np.savetxt(tmp_path / f"exp_{name}.txt.gz", arr, delimiter=",", fmt="%s")
        assert read_out(tmp_path / "out" / f"{name}_{chrom}.txt.gz") == read_out(tmp_path / f"exp_{name}.txt.gz"), name
    txt = read_out(tmp_path / "out" / f"n_total_reads_case_{chrom}.txt.gz")
    assert (".0" in txt) == (not full)


def test_marking_pass_equals_single_base_path(lib):
    """hyg_pre_collapse with plus_single_base = 0 (the pre_mark_kernel pass)
    and = 1 (pairing through the grid's own lookup) agree on single-base data."""
    from hygeia_amd import _lib
    from hygeia_amd.preprocess import read_bed
    import ctypes as C

    cpg1, beds = synth(5000, 11)
    dev = torch.device("cuda", 0)
    pos0 = torch.from_numpy(np.sort(cpg1 - 1)).to(dev)
    import tempfile, os
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "s.bed")
        with open(p, "w") as fh:
            fh.write("h\n")
            beds[0].to_csv(fh, sep="\t", index=False, header=False)
        (ps, pe, pc, pp), (ms, _, mc, mp) = read_bed(p, "22")[0]
    t = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (ps, pe, pc, pp, ms, mc, mp)]
    outs = []
    for single in (0, 1):
        out = torch.full((pos0.numel(), 2), -7.0, dtype=torch.float64, device=dev)
        scratch = torch.empty(max(len(ms), 1), dtype=torch.uint8, device=dev)
        conf = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.check(lib.hyg_pre_collapse(pos0.data_ptr(), pos0.numel(), t[0].data_ptr(), t[1].data_ptr(),
                                        t[2].data_ptr(), t[3].data_ptr(), len(ps), t[4].data_ptr(), t[5].data_ptr(),
                                        t[6].data_ptr(), len(ms), single, scratch.data_ptr(), out.data_ptr(), 2, 0,
                                        conf.data_ptr(), None))
        torch.cuda.synchronize()
        assert int(conf.item()) == 0
        outs.append(out.cpu().numpy())
    np.testing.assert_array_equal(np.nan_to_num(outs[0], nan=-1), np.nan_to_num(outs[1], nan=-1))
    assert np.isfinite(outs[0]).any() and np.isnan(outs[0]).any()
