"""`hygeia infer` host logic (hygeia_amd/cli.py) against run_inference_two_groups.py:
flags (:19-72), segment slicing and early exit (:194-218), file layout (:101-108,
246-322). CPU only: the compute call itself must refuse without a GPU.
"""
import gzip
import math
import os
import time

import numpy as np
import pytest

from hygeia_amd import cli


def test_flag_defaults_match_reference():
    f = cli.parse_flags([])
    assert f["mu"] == ["0.95", "0.05", "0.80", "0.20", "0.50", "0.50"]
    assert f["sigma"] == ["0.05", "0.05", "0.1", "0.1", "0.1", "0.2886751"]
    assert f["minimum_duration"] == 3 and f["omega_case"] == 0.8
    assert f["merge_log_prob"] == pytest.approx(math.log(0.1)) and f["split_prob"] == 0.01
    assert f["num_resampled_particles"] == [50] and f["num_samples_backward"] == 25
    assert f["multinomial"] is False and f["chrom"] == "22"
    assert (f["seed"], f["batch"], f["segment_size"], f["buffer_size"]) == (0, 0, 100000, 5000)


def test_flag_forms():
    f = cli.parse_flags(["--mu", "0.9,0.1", "--sigma=0.05,0.05", "--chrom", "chr7", "--seed=3", "--batch", "2",
                         "--num_resampled_particles=20", "--num_resampled_particles", "30", "--multinomial",
                         "--segment_size", "1000", "--results_dir", "/tmp/x"])
    assert f["mu"] == ["0.9", "0.1"] and f["sigma"] == ["0.05", "0.05"]
    assert f["chrom"] == "chr7" and f["seed"] == 3 and f["batch"] == 2
    assert f["num_resampled_particles"] == [20, 30] and f["multinomial"] is True
    assert cli.parse_flags(["--nomultinomial"])["multinomial"] is False
    with pytest.raises(cli.FlagError):
        cli.parse_flags(["--not_a_flag=1"])
    with pytest.raises(cli.FlagError):
        cli.parse_flags(["--seed"])


def test_serialized_flags_roundtrip():
    f = cli.parse_flags(["--num_resampled_particles=20", "--num_resampled_particles=30", "--chrom=5"])
    s = cli.serialize_flags(f)
    assert "--num_resampled_particles=20\n--num_resampled_particles=30" in s
    assert "--nomultinomial" in s and "--chrom=5" in s
    assert cli.parse_flags(s.split("\n")) == f


@pytest.mark.parametrize("n,batch,S,B,want", [
    (250000, 0, 100000, 5000, ((0, 105000), (0, 100000))),
    (250000, 1, 100000, 5000, ((95000, 205000), (5000, 105000))),
    (250000, 2, 100000, 5000, ((195000, 250000), (5000, 55000))),
    (200000, 2, 100000, 5000, ((195000, 200000), (5000, 5000))),   # b*S == n: an empty return range
    (250000, 3, 100000, 5000, None),                                # b*S > n: exit 0
    (50, 0, 100000, 5000, ((0, 50), (0, 50))),
])
def test_segment_index(n, batch, S, B, want):
    assert cli.segment_index(n, batch, S, B) == want


def test_segments_cover_the_chromosome_once():
    n, S, B = 123457, 10000, 500
    covered = np.zeros(n, int)
    b = 0
    while True:
        seg = cli.segment_index(n, b, S, B)
        if seg is None:
            break
        (lo, hi), (r0, r1) = seg
        covered[lo + r0:lo + r1] += 1
        b += 1
    assert np.all(covered == 1)


def _write_inputs(d, chrom, T, S=2, K=6, seed=4):
    from hygeia_amd import synthetic as syn
    from hygeia_amd import two_group

    data = syn.simulate(T, S, S, K=K, seed=seed, coverage=30.0)
    os.makedirs(os.path.join(d, "data"), exist_ok=True)
    os.makedirs(os.path.join(d, "sg"), exist_ok=True)
    pos = syn.positions(T, seed)
    np.savetxt(os.path.join(d, "data", f"positions_{chrom}.txt.gz"), pos.astype(np.float64), fmt="%s")
    for g in ("control", "case"):
        np.savetxt(os.path.join(d, "data", f"n_total_reads_{g}_{chrom}.txt.gz"),
                   data[f"tot_{g}"].astype(np.float64), fmt="%s", delimiter=",")
        np.savetxt(os.path.join(d, "data", f"n_methylated_reads_{g}_{chrom}.txt.gz"),
                   data[f"meth_{g}"].astype(np.float64), fmt="%s", delimiter=",")
    theta = two_group.uniform_theta(K, 0.8)
    with gzip.open(os.path.join(d, "sg", f"theta_{chrom}.csv.gz"), "wt") as fh:
        fh.write("data\n" + "\n".join(repr(float(x)) for x in theta) + "\n")
    return data


def test_infer_too_large_batch_exits_zero(tmp_path):
    _write_inputs(str(tmp_path), "21", 300)
    rc = cli.main(["infer", "--chrom", "21", "--batch", "5", "--segment_size", "100",
                   "--data_dir", str(tmp_path / "data"), "--single_group_dir", str(tmp_path / "sg"),
                   "--results_dir", str(tmp_path / "res")])
    assert rc == 0
    assert os.path.exists(tmp_path / "res" / "chrom_21_5" / "flags0.txt")


def test_infer_writes_inputs_then_refuses_without_gpu(tmp_path):
    from hygeia_amd import _lib

    if _lib.load().hyg_device_count() > 0:
        pytest.skip("host without a GPU only")
    data = _write_inputs(str(tmp_path), "21", 300)
    args = ["infer", "--chrom", "21", "--batch", "1", "--segment_size", "100", "--buffer_size", "10",
            "--data_dir", str(tmp_path / "data"), "--single_group_dir", str(tmp_path / "sg"),
            "--results_dir", str(tmp_path / "res"), "--seed", "7"]
    with pytest.raises(_lib.HygError) as e:
        cli.main(args)
    assert e.value.code == _lib.HYG_EDEVICE
    out = tmp_path / "res" / "chrom_21_1"
    obs = np.loadtxt(out / "observations_control.csv.gz", delimiter=",")
    np.testing.assert_array_equal(obs, data["meth_control"][100:200])  # rows [90, 210), returned [10, 110)
    assert (out / "flags7.txt").read_text().startswith("--mu=")


def test_infer_many_writes_inputs_then_refuses_without_gpu(tmp_path):
    """infer_many parses the chromosome once, writes every task's flags and
    input files, then needs the HIP library and a device (no CPU path)."""
    _write_inputs(str(tmp_path), "3", 2500)
    args = ["infer_many", "--chrom", "3", "--segment_size", "1000", "--buffer_size", "50", "--seeds", "1,2",
            "--data_dir", str(tmp_path / "data"), "--single_group_dir", str(tmp_path / "sg"),
            "--results_dir", str(tmp_path / "res")]
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible: covered by tests/test_gpu_two_group.py")
    with pytest.raises(Exception):
        cli.main(args)
    for b in (0, 1, 2):
        d = tmp_path / "res" / f"chrom_3_{b}"
        assert (d / "flags1.txt").read_text().splitlines()[-4:-2] == [f"--seed=1", f"--batch={b}"]
        assert (d / "flags2.txt").exists() and (d / "positions.csv.gz").exists()


@pytest.mark.parametrize("shape,dtype", [((300, 4), np.int16), ((257,), np.int64), ((5, 1), np.int16)])
def test_fast_savetxt_matches_numpy(tmp_path, shape, dtype):
    """The table formatter writes np.savetxt(delimiter=',')'s exact text."""
    a = np.random.default_rng(3).integers(-5, 30000, size=shape).astype(dtype)
    cli._savetxt(str(tmp_path / "a.csv.gz"), a)
    np.savetxt(str(tmp_path / "b.csv.gz"), a, delimiter=",")
    assert gzip.open(tmp_path / "a.csv.gz").read() == gzip.open(tmp_path / "b.csv.gz").read()
    cli._savetxt(str(tmp_path / "c.csv"), a)
    np.savetxt(str(tmp_path / "d.csv"), a, delimiter=",")
    assert (tmp_path / "c.csv").read_bytes() == (tmp_path / "d.csv").read_bytes()


@pytest.mark.parametrize("form", ["repr", "%.18e", "%.6g", "quoted_header", "index_col", "int", "odd"])
def test_read_theta_equals_pandas(tmp_path, form):
    """read_theta gives pandas' values, the reference's reader
    (run_inference_two_groups.py:76-79), on every text form; on 17-digit repr
    text those differ from Python's correctly rounded float()."""
    import pandas as pd

    v = np.random.default_rng(7).normal(0.0, 3.0, size=42) * 10.0 ** np.random.default_rng(8).integers(-12, 12, 42)
    fmt = {"repr": repr, "%.18e": lambda x: "%.18e" % x, "%.6g": lambda x: "%.6g" % x}.get(form, repr)
    body = [fmt(float(x)) for x in v]
    if form == "quoted_header":
        text = '"data"\n' + "\n".join(body) + "\n"
    elif form == "index_col":
        text = ",data\n" + "\n".join(f"{i},{b}" for i, b in enumerate(body)) + "\n"
    elif form == "int":
        text = "data\n" + "\n".join(str(i - 20) for i in range(42)) + "\n"
    elif form == "odd":  # a blank, a NaN spelling and an empty line: the pandas path
        text = "data\n" + "\n".join(body[:5]) + "\n 1.5\nNA\n\n" + "\n".join(body[5:]) + "\n"
    else:
        text = "data\n" + "\n".join(body) + "\n"
    d = tmp_path / "sg"
    d.mkdir()
    with gzip.open(d / "theta_7.csv.gz", "wt") as fh:
        fh.write(text)
    got = cli.read_theta(str(d), "7")
    want = pd.to_numeric(pd.read_table(d / "theta_7.csv.gz", sep=",")["data"]).to_numpy(dtype=np.float64)
    np.testing.assert_array_equal(got, want)
    if form == "repr":  # why the reader stays pandas: its converter is not float()'s on such text
        assert not np.array_equal(want, np.array([float(b) for b in body]))


def test_sci18_table_matches_format():
    """The array-built '%.18e' text equals Python's for every digit count and
    sign, up to 2**53 - 1 (positions, counts, negative sentinels)."""
    edge = [0, 1, -1, 9, 10, -10, 99, 100, 2 ** 31 - 1, -2 ** 31, 2 ** 53 - 1, -(2 ** 53 - 1)]
    edge += [s * (10 ** k + d) for k in range(16) for d in (-1, 0, 1) for s in (1, -1)]
    rnd = np.random.default_rng(5).integers(-2 ** 53 + 1, 2 ** 53, size=20000)
    vals = np.concatenate([np.array(edge, np.int64), rnd, (rnd % 1000003)])
    t = cli._sci18_table(vals)
    got = [bytes(r[r != 0]).decode() for r in t]
    assert got == ["%.18e" % float(v) for v in vals]


@pytest.mark.parametrize("dtype", [np.int64, np.uint64, np.uint8])
def test_fast_savetxt_wide_and_unsigned(tmp_path, dtype):
    """Values at the 2**53 edge and unsigned types: the same text as np.savetxt."""
    info = np.iinfo(dtype)
    a = np.array([[0, 1], [info.max, 7], [min(info.max, 2 ** 53 - 1), 3]], dtype=dtype)
    cli._savetxt(str(tmp_path / "c.csv"), a)
    np.savetxt(str(tmp_path / "d.csv"), a, delimiter=",")
    assert (tmp_path / "c.csv").read_bytes() == (tmp_path / "d.csv").read_bytes()


def test_read_matrix_equals_pandas(tmp_path):
    """cli._read_matrix (pyarrow, pandas re-read for non-integral input) gives
    pandas' values (the reference's parser, run_inference_two_groups.py:177-191)
    on plain and '%.18e' integer text, gzip or not, and on non-integral text."""
    import pandas as pd

    rng = np.random.default_rng(5)
    a = rng.poisson(40, (3000, 3)).astype(np.int64)
    cases = {
        "plain.txt.gz": "\n".join(",".join(str(x) for x in r) for r in a) + "\n",
        "sci.txt.gz": "\n".join(",".join("%.18e" % x for x in r) for r in a) + "\n",
        "frac.txt": "0.1,2\n3.3333333333333333,1e-300\n",
        "one.txt": "7\n",
    }
    for name, text in cases.items():
        p = str(tmp_path / name)
        if name.endswith(".gz"):
            with gzip.open(p, "wt") as fh:
                fh.write(text)
        else:
            with open(p, "w") as fh:
                fh.write(text)
        got = cli._read_matrix(p)
        ref = pd.read_csv(p, sep=",", header=None, dtype=np.float64).to_numpy()
        assert got.dtype == np.float64 and got.shape == ref.shape
        assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), name


@pytest.mark.parametrize("group", ["case", "control"])
@pytest.mark.parametrize("cmd", ["infer", "infer_many"])
def test_methylated_above_total_is_rejected(tmp_path, group, cmd):
    """A site whose methylated count exceeds its total count stops the task with
    an AssertionError before any chain runs, in either group.

    The reference asserts this for the case group only: its control assertion
    compares n_total_reads_control with itself (run_inference_two_groups.py:
    210-211) and can never fail. That input has no defined emission
    (Beta-Binomial with k > n: TFP returns -inf or NaN from its lgamma terms),
    so the build applies the check the assertion evidently means to both groups
    -- a deliberate divergence at the boundary."""
    _write_inputs(str(tmp_path), "21", 300)
    f = tmp_path / "data" / f"n_methylated_reads_{group}_21.txt.gz"
    tot = np.loadtxt(tmp_path / "data" / f"n_total_reads_{group}_21.txt.gz", delimiter=",")
    meth = np.loadtxt(f, delimiter=",")
    meth[150, 1] = tot[150, 1] + 1  # inside batch 1's rows [90, 210)
    np.savetxt(f, meth, fmt="%s", delimiter=",")
    args = [cmd, "--chrom", "21", "--segment_size", "100", "--buffer_size", "10",
            "--data_dir", str(tmp_path / "data"), "--single_group_dir", str(tmp_path / "sg"),
            "--results_dir", str(tmp_path / "res")]
    args += ["--batch", "1"] if cmd == "infer" else ["--batches", "1"]
    with pytest.raises(AssertionError, match="methylated reads exceed total reads"):
        cli.main(args)
    # a batch whose rows do not hold the site runs on (up to the device call)
    args_ok = [a if a != "1" else "2" for a in args]
    try:
        cli.main(args_ok)  # runs on a GPU host; stops at the device call without one
    except AssertionError:
        raise
    except Exception:
        pass


def test_single_task_does_not_import_torch(tmp_path):
    """A `hygeia infer` task runs its chain through the host-pointer C entry, so
    its process never imports torch (about 2 s of every fresh task, which is
    how modules/two_group/4_infer.nf runs it). Here, without a GPU, the task
    stops at the device call; the check is on the process's modules."""
    import subprocess
    import sys

    _write_inputs(str(tmp_path), "21", 300)
    code = ("import sys\nfrom hygeia_amd import cli\n"
            "try:\n    cli.main(sys.argv[1:])\nexcept Exception as e:\n    print('stopped:', type(e).__name__)\n"
            "print('torch imported:', 'torch' in sys.modules)\n")
    args = ["infer", "--chrom", "21", "--batch", "1", "--segment_size", "100", "--buffer_size", "10",
            "--data_dir", str(tmp_path / "data"), "--single_group_dir", str(tmp_path / "sg"),
            "--results_dir", str(tmp_path / "res")]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code] + args, capture_output=True, text=True, cwd=root,
                       env=dict(os.environ, PYTHONPATH=root), timeout=300)
    assert "torch imported: False" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("fmt", ["%d", "%.18e", "%.1f"])
def test_partial_read_equals_whole_file_prefix(tmp_path, fmt):
    """A task reads its count files only up to its last row
    ((batch + 1) * segment + buffer): the rows read equal the whole file's
    first rows, across the streaming reader's blocks and at the end of the
    file, for the pipeline's number formats; a non-integral value falls back to
    pandas (nrows) with the same result."""
    rng = np.random.default_rng(3)
    a = rng.integers(0, 400, (130_000, 4)).astype(np.float64)
    p = str(tmp_path / "m.txt.gz")
    np.savetxt(p, a, fmt=fmt, delimiter=",")
    whole = cli._read_matrix(p)
    np.testing.assert_array_equal(whole, a)
    for n in (1, 999, 65_536, 100_001, 129_999, 130_000, 130_001, 10 ** 9):
        got = cli._read_matrix(p, max_rows=n)
        np.testing.assert_array_equal(got, a[:n])
    b = a.copy()
    b[5, 1] = 0.5  # not a count: the pandas path
    q = str(tmp_path / "f.txt.gz")
    np.savetxt(q, b, fmt="%.18e", delimiter=",")
    np.testing.assert_array_equal(cli._read_matrix(q, max_rows=70_000), b[:70_000])


def test_segment_of_partial_read_equals_whole(tmp_path):
    """segment_index on the rows a task reads gives the slice and the early exit
    it gives on the whole chromosome, for every batch."""
    for n in (1, 999, 1000, 1001, 2600, 5000):
        for b in range(0, n // 1000 + 3):
            need = (b + 1) * 1000 + 60
            assert cli.segment_index(min(n, max(need, 1)), b, 1000, 60) == cli.segment_index(n, b, 1000, 60)


def test_version_answer_of_the_wrapper_equals_the_cli(capsys):
    """bin/hygeia answers --version itself (every 4_infer.nf task runs it); the
    text equals hygeia_amd.cli's, which equals the library's hyg_version()
    (tests/test_capi_cpu.py)."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for arg in ("--version", "-v", "version"):
        env = dict(os.environ, HYGEIA_VERSION="9.9")
        out = subprocess.run([os.path.join(root, "bin", "hygeia"), arg], capture_output=True, text=True, env=env)
        assert out.returncode == 0
        os.environ["HYGEIA_VERSION"] = "9.9"
        try:
            assert cli.main([arg]) == 0
        finally:
            del os.environ["HYGEIA_VERSION"]
        assert out.stdout == capsys.readouterr().out == "Hygeia version 9.9 (hygeia_amd 0.1.0 (gfx950))\n"


def test_pandas_float_equals_pandas():
    """cli.pandas_float (read_theta's converter) against pandas' C parser on
    100 000 numbers: repr, %.18e, %.17g, 25-decimal fixed, long fractions with
    leading zeros, many-digit integers and fractions; bit for bit."""
    import io

    import pandas as pd

    rng = np.random.default_rng(1)
    strs = []
    for i in range(100_000):
        x = float(rng.normal() * 10.0 ** rng.integers(-30, 30))
        f = i % 6
        if f == 0:
            s = repr(x)
        elif f == 1:
            s = "%.18e" % x
        elif f == 2:
            s = "%.17g" % x
        elif f == 3:
            s = "%.25f" % x if abs(x) < 1e5 else repr(x)
        elif f == 4:
            s = "0.000" + str(rng.integers(0, 10 ** 18))
        else:
            s = str(rng.integers(-10 ** 6, 10 ** 6)) + "." + str(rng.integers(0, 10 ** 12)).zfill(12)
        strs.append(s)
    want = pd.to_numeric(pd.read_table(io.StringIO("data\n" + "\n".join(strs) + "\n"), sep=",")["data"]).to_numpy(
        dtype=np.float64)
    got = np.array([cli.pandas_float(s) for s in strs])
    assert np.array_equal(got.view(np.int64), want.view(np.int64))
    assert not np.array_equal(got, np.array([float(s) for s in strs]))  # not Python's float()


def test_parse_cache(tmp_path):
    """The parse cache returns the parse's values (int32-stored counts, float64
    positions beyond int32, a float matrix kept as float64), is filled once under
    concurrent readers, follows a rewritten file, and is placed by
    parse_cache_dir (env, Nextflow workDir, or off)."""
    from concurrent.futures import ThreadPoolExecutor

    rng = np.random.default_rng(5)
    a = rng.integers(0, 500, (20_000, 3)).astype(np.float64)
    big = (rng.integers(0, 2 ** 40, (3000, 1))).astype(np.float64)
    p, q = str(tmp_path / "a.txt.gz"), str(tmp_path / "b.txt.gz")
    np.savetxt(p, a, fmt="%.18e", delimiter=",")
    np.savetxt(q, big, fmt="%d", delimiter=",")
    cache = str(tmp_path / "cache")
    with ThreadPoolExecutor(8) as ex:
        outs = list(ex.map(lambda n: cli._cached_matrix(p, cache, n), [None, 5, 19_999, 20_000, 10 ** 6] * 4))
    for o, n in zip(outs, [None, 5, 19_999, 20_000, 10 ** 6] * 4):
        assert o.dtype == np.float64
        np.testing.assert_array_equal(o, a if n is None else a[:n])
    npys = [f for f in os.listdir(cache) if f.endswith(".npy")]
    assert len(npys) == 1 and np.load(os.path.join(cache, npys[0])).dtype == np.int32
    np.testing.assert_array_equal(cli._cached_matrix(q, cache, 100), big[:100])
    assert sorted(np.load(os.path.join(cache, f)).dtype.str for f in os.listdir(cache) if f.endswith(".npy")) == [
        "<f8", "<i4"]
    time.sleep(0.01)
    np.savetxt(p, a[:7] + 1, fmt="%d", delimiter=",")  # rewritten: a new key
    np.testing.assert_array_equal(cli._cached_matrix(p, cache), a[:7] + 1)
    # where it lives
    assert cli.parse_cache_dir({"HYGEIA_PARSE_CACHE": "/x"}) == "/x"
    assert cli.parse_cache_dir({"HYGEIA_PARSE_CACHE": "0"}, cwd=str(tmp_path)) is None
    assert cli.parse_cache_dir({}, cwd=str(tmp_path)) is None
    task = tmp_path / "work" / "ab" / "cdef"
    task.mkdir(parents=True)
    (task / ".command.sh").write_text("hygeia infer\n")
    assert cli.parse_cache_dir({}, cwd=str(task)) == str(tmp_path / "work" / ".hygeia_parse_cache")


def test_partial_read_of_a_multi_member_gzip(tmp_path):
    """A gzip file of several members (concatenated gzip streams, as `cat a.gz
    b.gz` makes) reads the same whole and by prefix, across the member joins."""
    rng = np.random.default_rng(9)
    a = rng.integers(0, 300, (9_000, 2)).astype(np.float64)
    p = tmp_path / "m.txt.gz"
    with open(p, "wb") as fh:
        for part in (a[:4000], a[4000:4001], a[4001:]):
            fh.write(gzip.compress(("\n".join(",".join(str(int(v)) for v in r) for r in part) + "\n").encode()))
    np.testing.assert_array_equal(cli._read_matrix(str(p)), a)
    for n in (3999, 4000, 4001, 4002, 8999, 9000, 20_000):
        np.testing.assert_array_equal(cli._read_matrix(str(p), max_rows=n), a[:n])


def test_control_theta_slices_as_the_reference():
    """get_estimated_control_group_param (run_inference_two_groups.py:76-89):
    P from the first K (K - 1) entries, omega's logits from the last K -- for a
    K (K + 1) theta (kappa estimated) those are the log kappa entries."""
    K = 6
    th = np.arange(42, dtype=np.float64)
    np.testing.assert_array_equal(cli.control_theta(th[:36], K), th[:36])
    np.testing.assert_array_equal(cli.control_theta(th, K), np.concatenate([th[:30], th[36:]]))
    with pytest.raises(ValueError):
        cli.control_theta(th[:40], K)


def test_parallel_reads_after_module_import(tmp_path):
    """_read_inputs parses its five files on worker threads. With pyarrow 25 /
    numpy 2.2 a process whose first `import pyarrow` happened on a worker
    thread segfaults in ChunkedArray.to_numpy under concurrent conversions;
    importing hygeia_amd.cli imports pyarrow on the main thread first. A fresh
    interpreter runs many concurrent reads and must exit cleanly."""
    import subprocess
    import sys

    rng = np.random.default_rng(5)
    p = str(tmp_path / "a.txt.gz")
    np.savetxt(p, rng.integers(0, 500, (20_000, 3)).astype(np.float64), fmt="%.18e", delimiter=",")
    code = (
        "import sys\n"
        "from concurrent.futures import ThreadPoolExecutor\n"
        "from hygeia_amd import cli\n"
        "for _ in range(20):\n"
        "    with ThreadPoolExecutor(8) as ex:\n"
        "        list(ex.map(lambda n: cli._read_matrix(sys.argv[1], n), [None, 5, 19999, 20000, 10 ** 6] * 4))\n"
    )
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code, p], cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
