"""SURVEY.md 8f-4 on CPU: `hygeia get_chrom_segments` (get_chrom_segments.py:23-43)
and the native BED formatter hyg_bed_format (host code of the C ABI) against a
restatement of src/single_group/bin/make_bed_file:19-66 (data.table) written
here; the per-site labels come from the device (tests/test_gpu_bed.py). Against
R itself the text is parity unpinned (R is absent)."""
import gzip
import os

import numpy as np
import pytest

from hygeia_amd import bed, cli


def r_make_bed(chrom, pos, probs, cols):
    """make_bed_file:19-63: score = pmax, tie_count = rowSums(.SD == score),
    name = "equiprobable" or max.col(ties.method = "first"); setkey(chr, start)."""
    score = probs.max(axis=1)
    ties = (probs == score[:, None]).sum(axis=1)
    name = np.where(ties > 1, "equiprobable", np.asarray(cols, dtype=object)[probs.argmax(axis=1)])
    rgb = dict(zip(list(cols) + ["equiprobable"], bed.ITEM_RGB))
    order = np.argsort(pos - 1, kind="stable")
    out = []
    for i in order:
        p = int(pos[i])
        out.append(f"{chrom}\t{p - 1}\t{p + 1}\t{name[i]}\t{score[i]:.15g}\t.\t{p - 1}\t{p + 1}\t{rgb[name[i]]}\n")
    return "".join(out).encode()


def r_labels(probs):
    score = probs.max(axis=1)
    ties = (probs == score[:, None]).sum(axis=1)
    return np.where(ties > 1, -1, probs.argmax(axis=1)).astype(np.int8), score


def regimes_probs(n, K, seed):
    rng = np.random.default_rng(seed)
    p = rng.dirichlet(np.ones(K) * 0.3, size=n)
    p = np.round(p, 7)  # R format(): 7 significant digits
    p[::7, :2] = p[::7, :2].max(axis=1, keepdims=True)  # planted ties of the maximum
    p[::11] = 1.0 / K                                    # all equal
    p[5::13, 0] = 1.0
    p[5::13, 1:] = 0.0
    return p


def test_bed_format_matches_restatement():
    K, n = 6, 5000
    probs = regimes_probs(n, K, 1)
    pos = np.cumsum(np.random.default_rng(2).integers(1, 300, n)) + 10_000
    cols = [f"regime_{r + 1}" for r in range(K)]
    lab, sc = r_labels(probs)
    got = bed.format_bed("21", pos, lab, sc, cols + ["equiprobable"], bed.ITEM_RGB)
    assert got == r_make_bed("21", pos, probs, cols)
    lines = got.decode().splitlines()
    assert len(lines) == n and all(len(x.split("\t")) == 9 for x in lines)
    assert any("\tequiprobable\t" in x and x.endswith("128,128,128") for x in lines)
    assert "\t1\t.\t" in lines[5]  # score 1.0 written as "1" (fwrite drops trailing zeros)


def test_bed_format_sizes_and_errors():
    from hygeia_amd import _lib

    L = _lib.load()
    pos, lab, sc = np.array([5], np.int64), np.array([7], np.int8), np.array([0.5])
    names = ["regime_1", "equiprobable"]
    with pytest.raises(RuntimeError):  # label beyond K
        bed.format_bed("1", pos, lab, sc, names, bed.ITEM_RGB[:2])
    assert bed.format_bed("1", pos[:0], lab[:0], sc[:0], names, bed.ITEM_RGB[:2]) == b""
    assert L.hyg_bed_labels(None, 0, 10, None, None, None) == -1


def test_make_bed_file_rejects_non_six_regimes(tmp_path):
    f = tmp_path / "regimes.csv"
    f.write_text("genomic_position,regime_1,regime_2\n10,0.5,0.5\n")
    rc = cli.main(["make_bed_file", "--chr", "1", "--regimes_file", str(f), "--output_file", str(tmp_path / "o.bed")])
    assert rc == 1


@pytest.mark.parametrize("n,size,expect", [(250_001, 100_000, 3), (200_000, 100_000, 3), (5, 100_000, 1),
                                           (0, 10, 1)])
def test_get_chrom_segments(tmp_path, capsys, n, size, expect):
    inp = tmp_path / "positions_22.txt.gz"
    with gzip.open(inp, "wt") as fh:
        for i in range(n):
            fh.write(f"{100 + 3 * i}\n")
    out = tmp_path / "sub" / "chrom_segments_22.csv"
    rc = cli.main(["get_chrom_segments", f"--input_file={inp}", "--chromosome", "22", "--output_csv", str(out),
                   "--segment_size", str(size)])
    assert rc == 0
    assert out.read_text() == "chrom,segment_index\n" + "".join(f"22,{i}\n" for i in range(expect))
    assert f"Segment information saved to {out}" in capsys.readouterr().out
