"""`hygeia infer` on the MI355X path: a drop-in for src/two_group/run_inference_two_groups.py.

Same flags (absl spellings and defaults, run_inference_two_groups.py:19-72), same
input files (B.1 of SURVEY.md: whole-chromosome gzip CSVs in --data_dir and
theta_{chrom}.csv.gz in --single_group_dir), same segment slicing and exit
behaviour (:194-218), same output directory and files (:101-108, 246-322):

    results_dir/chrom_{chrom}_{batch}/
        flags{seed}.txt
        observations_{control,case}.csv.gz, n_total_reads_{control,case}.csv.gz, positions.csv.gz
        optimal_backward_particles_{merged,control,case}_state_{N}_{seed}.npz   (int16, trimmed)
        optimal_split_probs_{N}_{seed}.npz, optimal_regime_probs_{N}_{seed}.npz (float32, untrimmed)
        log_normalizing_constants_optimal_{seed}.txt, optimal_time_{seed}.txt,
        optimal_time_backward_{seed}.txt

so modules/two_group/4_infer.nf runs it unchanged (through bin/hygeia). The
filter and the backward simulation run in the HIP kernels behind the C ABI
(include/hygeia_amd.h); there is no CPU path.

The random streams are Philox4x64-10 keyed by (seed, chain id) with
chain id = crc32(chrom) << 32 | batch, so a (chrom, batch, seed) task gives the
same trajectories here, in a batched multi-chain run, and on any GPU count.
"""
from __future__ import annotations

import gzip
import math
import os
import re
import sys
import threading
import time
import zlib
from typing import Dict, List, Sequence

import numpy as np

try:  # on the importing (main) thread, before any reader thread: see _import_parsers
    import pyarrow  # noqa: F401
except ImportError:  # pragma: no cover -- the readers then fall back to pandas
    pass

# (name, kind, default, help) in the reference's definition order (:19-72)
FLAGS_SPEC = [
    ("mu", "list", "0.95,0.05,0.80,0.20,0.50,0.50", "mu of the beta distribution"),
    ("sigma", "list", "0.05,0.05,0.1,0.1,0.1,0.2886751", "sigma of the beta distribution"),
    ("minimum_duration", "int", 3, "minimum duration between change points"),
    ("omega_case", "float", 0.8, "omega parameter for duration of case group"),
    ("merge_log_prob", "float", math.log(0.1), "value for merge probability"),
    ("split_prob", "float", 0.01, "value for split probability"),
    ("num_resampled_particles", "multi_int", [50], "number M of particles that are resampled"),
    ("num_samples_backward", "int", 25, "number of particles used for backward sampling"),
    ("multinomial", "bool", False, "multinomial or residual resampling"),
    ("chrom", "string", "22", "The chromosome to analyze"),
    ("results_dir", "string", os.path.join(os.path.dirname(os.getcwd()), "test"), "Directory for the results"),
    ("data_dir", "string", "data", "Directory of the read data"),
    ("single_group_dir", "string", os.path.join("test_data", "single_group_results"),
     "Directory of the single group estimation results"),
    ("seed", "int", 0, "seed used for sampling random variables"),
    ("batch", "int", 0, "index of the selected chromosome segment"),
    ("segment_size", "int", 100000, "size of the selected chromosome segment (in CpG sites)"),
    ("buffer_size", "int", 5000, "size of the buffer segment (in CpG sites)"),
]


class FlagError(ValueError):
    pass


def parse_flags(argv: Sequence[str], flags_spec=None) -> Dict[str, object]:
    """absl-style parsing: --name=value, --name value, --bool / --nobool, list
    flags comma separated, multi flags repeated (FLAGS_SPEC unless given)."""
    spec = {n: (k, d) for n, k, d, _ in (FLAGS_SPEC if flags_spec is None else flags_spec)}
    out: Dict[str, object] = {}
    multi: Dict[str, List[object]] = {}
    i = 0
    argv = list(argv)
    while i < len(argv):
        a = argv[i]
        if a == "--":
            break
        if not a.startswith("-"):
            raise FlagError(f"unexpected argument {a!r}")
        body = a.lstrip("-")
        name, eq, val = body.partition("=")
        if name not in spec and name.startswith("no") and name[2:] in spec and spec[name[2:]][0] == "bool":
            if eq:
                raise FlagError(f"--{name} takes no value")
            out[name[2:]] = False
            i += 1
            continue
        if name not in spec:
            raise FlagError(f"Unknown command line flag '{name}'")
        kind = spec[name][0]
        if kind == "bool":
            if eq:
                v = val.lower()
                if v not in ("true", "false", "1", "0"):
                    raise FlagError(f"invalid boolean value for --{name}: {val}")
                out[name] = v in ("true", "1")
            else:
                out[name] = True
            i += 1
            continue
        if not eq:
            if i + 1 >= len(argv):
                raise FlagError(f"Flag --{name} must have a value other than None.")
            val = argv[i + 1]
            i += 2
        else:
            i += 1
        try:
            if kind == "int":
                out[name] = int(val)
            elif kind == "float":
                out[name] = float(val)
            elif kind == "list":
                out[name] = [x for x in val.split(",") if x != ""]
            elif kind == "multi_int":
                multi.setdefault(name, []).extend(int(x) for x in val.split(","))
            elif kind == "multi_string":
                multi.setdefault(name, []).append(val)
            elif kind == "multi_float":
                multi.setdefault(name, []).extend(float(x) for x in val.split(","))
            else:
                out[name] = val
        except ValueError as e:
            raise FlagError(f"invalid value for --{name}: {val!r} ({e})")
    for n, v in multi.items():
        out[n] = v
    for n, (k, d) in spec.items():
        if n not in out:
            out[n] = d.split(",") if k == "list" else d
    return out


def serialize_flags(f: Dict[str, object]) -> str:
    """The flags file content (absl FlagValues serialisation, definition order)."""
    lines = []
    for n, k, _, _ in FLAGS_SPEC:
        v = f[n]
        if k == "bool":
            lines.append(f"--{n}" if v else f"--no{n}")
        elif k == "list":
            lines.append(f"--{n}={','.join(v)}")
        elif k == "multi_int":
            lines.extend(f"--{n}={x}" for x in v)
        else:
            lines.append(f"--{n}={v}")
    return "\n".join(lines)


# Wall-clock phase split of the last infer / infer_many call in this process
# (seconds): parse (the chromosome's input files), device (model, chains, copies
# back), of which chains (the launches alone), writes (joining the result-file
# writes after the last chain). Read by tools/bench_pipeline.py; nothing in the
# command's behaviour depends on it.
LAST_TIMINGS: Dict[str, float] = {}


def chain_id(chrom: str, batch: int) -> int:
    return (zlib.crc32(str(chrom).encode()) << 32) | (int(batch) & 0xFFFFFFFF)


def _gz_prefix(path: str, max_rows: int):
    """(the bytes of the first max_rows lines of a (multi-member) gzip file,
    whether the file goes on past them). Decompression is most of a parse."""
    out, lines = [], 0
    with open(path, "rb") as fh:
        d = zlib.decompressobj(wbits=47)  # gzip or zlib header, auto-detected
        while True:
            c = fh.read(1 << 20)
            if not c:
                break
            while c:
                x = d.decompress(c)
                if x:
                    k = x.count(b"\n")
                    if lines + k >= max_rows:
                        nl = np.flatnonzero(np.frombuffer(x, np.uint8) == 10)
                        cut = int(nl[max_rows - lines - 1]) + 1
                        out.append(x[:cut])
                        return b"".join(out), True
                    lines += k
                    out.append(x)
                c = d.unused_data  # the next gzip member
                if c:
                    d = zlib.decompressobj(wbits=47)
        out.append(d.flush())
    return b"".join(out), False


_IMPORT_LOCK = threading.Lock()


def _import_parsers(pandas: bool = False):
    """pyarrow.csv (or pandas) for the readers, which run on worker threads
    (_read_inputs), imported under one process-wide lock. pyarrow itself must
    already have been imported by the main thread (this module's import does
    it): with pyarrow 25 / numpy 2.2 a process whose first `import pyarrow`
    ran on a worker thread segfaults inside ChunkedArray.to_numpy when several
    threads convert at once (tests/test_cli.py::
    test_parallel_reads_after_module_import)."""
    with _IMPORT_LOCK:
        if pandas:
            import pandas as pd

            return pd
        import pyarrow.csv as pacsv

        return pacsv


def _read_matrix(path: str, max_rows: int = None) -> np.ndarray:
    """A whole-chromosome count matrix (run_inference_two_groups.py:177-191 reads
    it with pd.read_table(sep=",", header=None)) as float64; with max_rows, only
    its first max_rows rows (the file is decompressed no further).

    Parsed by pyarrow's multi-threaded CSV reader (about 2.7x pandas on a chr1
    matrix, most of a single `hygeia infer` task's host time). The pipeline's
    files hold integer counts (plain or '%.18e' text), which every correct
    parser reads exactly, so the values equal pandas'; a matrix with any
    non-integral or non-finite value (or one pyarrow cannot read) is re-read
    with pandas, the reference's parser, so such input keeps its exact values.
    (pandas is imported on that path only.)"""
    import io

    try:
        pacsv = _import_parsers()
        ro = pacsv.ReadOptions(autogenerate_column_names=True)
        po = pacsv.ParseOptions(delimiter=",")
        if max_rows is None or not path.endswith(".gz"):
            tb = pacsv.read_csv(path, read_options=ro, parse_options=po)
        else:
            raw, more = _gz_prefix(path, max_rows)
            tb = pacsv.read_csv(io.BytesIO(raw), read_options=ro, parse_options=po)
            if more and tb.num_rows < max_rows:  # blank lines were among the lines cut: read it all
                tb = pacsv.read_csv(path, read_options=ro, parse_options=po)
        if max_rows is not None:
            tb = tb.slice(0, max_rows)
        cols = [c.to_numpy(zero_copy_only=False) for c in tb.columns]
        if tb.num_columns > 0 and all(c.dtype.kind in "iuf" for c in cols):
            a = np.column_stack(cols).astype(np.float64)
            if np.all(np.isfinite(a)) and np.all(a == np.rint(a)) and np.all(np.abs(a) < 2.0 ** 53):
                return a
    except Exception:  # noqa: BLE001 -- any pyarrow failure (ArrowInvalid, ArrowNotImplementedError,
        pass  # ArrowTypeError, ...) falls back to pandas, the reference's parser
    pd = _import_parsers(pandas=True)
    return pd.read_csv(path, sep=",", header=None, dtype=np.float64, nrows=max_rows).to_numpy()


PARSE_CACHE_VAR = "HYGEIA_PARSE_CACHE"


def parse_cache_dir(environ=None, cwd: str = None):
    """Where parsed input matrices are kept for the next task of the same
    chromosome: $HYGEIA_PARSE_CACHE ("0": none), else inside a Nextflow task
    (.command.sh in the working directory <workDir>/<xx>/<hash>) the run's
    <workDir>/.hygeia_parse_cache, else none. Every (batch, seed) task of a
    chromosome reads the same five gzip files (4_infer.nf:28); with the cache
    one of them decompresses and parses each file and the others map the
    result."""
    env = os.environ if environ is None else environ
    v = env.get(PARSE_CACHE_VAR, "").strip()
    if v == "0":
        return None
    if v:
        return v
    cwd = cwd or os.getcwd()
    task = env.get("NXF_TASK_WORKDIR") or (cwd if os.path.exists(os.path.join(cwd, ".command.sh")) else None)
    if task:
        return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(task))), ".hygeia_parse_cache")
    return None


def _cached_matrix(path: str, cache: str, max_rows: int = None) -> np.ndarray:
    """_read_matrix through the parse cache: the whole file's matrix is parsed
    once (under an exclusive lock, so concurrent tasks wait for it rather than
    parse it too) and kept as an .npy keyed by the file's path, size, mtime and
    inode (int32 when every value fits, else float64: the values are those of
    the parse); a task maps it and copies its rows out. Any cache failure reads
    the file directly."""
    import fcntl
    import hashlib

    try:
        st = os.stat(path)
        key = hashlib.sha1(f"{os.path.realpath(path)}|{st.st_size}|{st.st_mtime_ns}|{st.st_ino}".encode()).hexdigest()
        os.makedirs(cache, exist_ok=True)
        npy = os.path.join(cache, key + ".npy")
        if not os.path.exists(npy):
            with open(os.path.join(cache, key + ".lock"), "a") as lk:
                fcntl.flock(lk, fcntl.LOCK_EX)
                if not os.path.exists(npy):
                    a = _read_matrix(path)
                    small = a.size == 0 or (a.min() >= -2 ** 31 and a.max() < 2 ** 31)
                    tmp = npy + f".{os.getpid()}.tmp.npy"
                    np.save(tmp, a.astype(np.int32) if small else a)
                    os.replace(tmp, npy)
                    return a if max_rows is None else a[:max_rows]
        m = np.load(npy, mmap_mode="r")
        return np.asarray(m if max_rows is None else m[:max_rows], dtype=np.float64)
    except OSError:
        return _read_matrix(path, max_rows)


def _read_inputs(data_dir: str, chrom: str, max_rows: int = None):
    """positions, n_total_reads_control, n_methylated_reads_control,
    n_total_reads_case, n_methylated_reads_case of one chromosome
    (run_inference_two_groups.py:177-191), the five files read concurrently
    (each file's gzip stream decompresses on one thread); with max_rows, the
    first max_rows rows of each; through the parse cache when there is one
    (parse_cache_dir)."""
    from concurrent.futures import ThreadPoolExecutor

    names = ["positions", "n_total_reads_control", "n_methylated_reads_control", "n_total_reads_case",
             "n_methylated_reads_case"]
    paths = [os.path.join(data_dir, f"{n}_{chrom}.txt.gz") for n in names]
    cache = parse_cache_dir()
    read = (lambda p: _cached_matrix(p, cache, max_rows)) if cache else (lambda p: _read_matrix(p, max_rows))
    with ThreadPoolExecutor(max_workers=len(paths)) as ex:
        return list(ex.map(read, paths))


_POW10F = [float(f"1e{k}") for k in range(309)]
_FLOAT_RE = re.compile(r"[+-]?(?:[0-9]+\.?[0-9]*|\.[0-9]+)(?:[eE][+-]?[0-9]+)?")
_INT_RE = re.compile(r"[+-]?[0-9]{1,15}")


def pandas_float(s: str) -> float:
    """pandas' default float converter for the C parser (precise_xstrtod, the
    'high' float_precision) on one plain decimal / scientific number: at most
    17 significant characters of the mantissa are accumulated in double
    arithmetic (leading zeros count, later integer digits only raise the
    exponent, later fraction digits are dropped), then the value is scaled by
    one correctly rounded power of ten (a multiply, or divides below 1e-308).
    tests/test_cli.py::test_pandas_float_equals_pandas compares it with pandas
    on 100 000 numbers of many forms."""
    p, n = 0, len(s)
    neg = False
    if p < n and s[p] in "+-":
        neg = s[p] == "-"
        p += 1
    number, exponent, nd, ndec = 0.0, 0, 0, 0
    while p < n and "0" <= s[p] <= "9":
        if nd < 17:
            number = number * 10.0 + (ord(s[p]) - 48)
            nd += 1
        else:
            exponent += 1
        p += 1
    if p < n and s[p] == ".":
        p += 1
        while nd < 17 and p < n and "0" <= s[p] <= "9":
            number = number * 10.0 + (ord(s[p]) - 48)
            p += 1
            nd += 1
            ndec += 1
        while p < n and "0" <= s[p] <= "9":
            p += 1
        exponent -= ndec
    if neg:
        number = -number
    if p < n and s[p] in "eE":
        p += 1
        eneg = False
        if p < n and s[p] in "+-":
            eneg = s[p] == "-"
            p += 1
        k = m = 0
        while k < 17 and p < n and "0" <= s[p] <= "9":
            m = m * 10 + (ord(s[p]) - 48)
            k += 1
            p += 1
        exponent += -m if eneg else m
    if exponent > 308:  # pandas flags ERANGE here: left to pandas itself
        raise ValueError("exponent out of range")
    if exponent > 0:
        return number * _POW10F[exponent]
    if exponent < -308:
        if exponent < -616:
            return 0.0 * number
        return number / _POW10F[-308 - exponent] / _POW10F[308]
    return number / _POW10F[-exponent]


def control_theta(theta: np.ndarray, K: int, chrom: str = "") -> np.ndarray:
    """get_estimated_control_group_param (run_inference_two_groups.py:76-89):
    P's rows from the first K (K - 1) entries, omega's logits from the LAST K.
    A theta of the single-group step with kappa estimated (K (K + 1) entries,
    model_functions.R:65-78) therefore gives log kappa as omega's logits, as
    the reference reads it. Other lengths are refused."""
    n = theta.shape[0]
    if n not in (K * K, K * (K + 1)):
        raise ValueError(f"theta_{chrom}.csv.gz holds {n} values, expected K^2 = {K * K} (or K(K+1) = {K * (K + 1)})")
    return np.concatenate([theta[:K * (K - 1)], theta[n - K:]])


def read_theta(single_group_dir: str, chrom: str) -> np.ndarray:
    """theta_{chrom}.csv.gz, column 'data' (run_inference_two_groups.py:76-79),
    with pandas' values, the reference's reader: pandas' default float
    converter is not Python's float() (it drops digits past the 17th character
    of the mantissa, leading zeros included: tests/test_cli.py::
    test_read_theta_equals_pandas), and theta's bits set every transition
    probability. A file of the single-group step's form (readr::write_csv of
    one 'data' column, input_output_functions.R:4-7: a header line, then one
    plain number per line) is converted here by pandas_float, without
    importing pandas (half a second of every task); any other text goes to
    pandas itself."""
    with gzip.open(os.path.join(single_group_dir, f"theta_{chrom}.csv.gz"), "rt") as fh:
        lines = fh.read().split("\n")
    if lines and lines[-1] == "":
        lines.pop()
    if len(lines) >= 2 and lines[0] in ("data", '"data"'):
        vals = lines[1:]
        if all(_INT_RE.fullmatch(v) for v in vals):  # pandas reads an integer column as int64
            return np.array([float(int(v)) for v in vals], dtype=np.float64)
        if all(_FLOAT_RE.fullmatch(v) for v in vals):
            try:
                return np.array([pandas_float(v) for v in vals], dtype=np.float64)
            except ValueError:
                pass
    import pandas as pd

    df = pd.read_table(os.path.join(single_group_dir, f"theta_{chrom}.csv.gz"), sep=",")
    return pd.to_numeric(df["data"]).to_numpy(dtype=np.float64)


def segment_index(n_sites: int, batch: int, segment_size: int, buffer_size: int):
    """Rows of the batch (run_inference_two_groups.py:194-218): (slice, return range) or None."""
    if batch * segment_size > n_sites:
        return None
    lo = max(0, batch * segment_size - buffer_size)
    hi = min((batch + 1) * segment_size + buffer_size, n_sites)
    T = hi - lo
    if batch == 0:
        ret = (0, min(T, segment_size))
    else:
        ret = (buffer_size, min(T, buffer_size + segment_size))
    return (lo, hi), ret


def _cpu_budget() -> int:
    """CPUs this process may use: its affinity, capped by a cgroup-v2 CPU quota
    (a container's affinity can list every core of the host)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            quota, period = fh.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return n


_POW10 = 10 ** np.arange(19, dtype=np.uint64)


def _sci18_table(v: np.ndarray) -> np.ndarray:
    """'%.18e' % float(x) of each integer x with |x| < 2**53, as an (n, 25)
    uint8 table (a NUL in column 0 where there is no sign). float(x) is exact,
    so its 19 significant digits are x's own digits followed by zeros and the
    exponent is (number of digits - 1): built with array arithmetic, no Python
    format call per value."""
    v = v.astype(np.int64)
    m = np.abs(v).astype(np.uint64)
    e = (m[:, None] >= _POW10[None, 1:]).sum(axis=1)  # digits - 1 (0 for x == 0)
    shift = e[:, None] - np.arange(19)[None, :]  # digit i (0 = leading) = m // 10**(e - i) % 10
    dig = np.where(shift >= 0, (m[:, None] // _POW10[np.clip(shift, 0, 18)]) % np.uint64(10), 0).astype(np.uint8)
    t = np.empty((v.shape[0], 25), np.uint8)
    t[:, 0] = np.where(v < 0, ord("-"), 0)
    t[:, 1] = 48 + dig[:, 0]
    t[:, 2] = ord(".")
    t[:, 3:21] = 48 + dig[:, 1:]
    t[:, 21], t[:, 22] = ord("e"), ord("+")
    t[:, 23], t[:, 24] = 48 + e // 10, 48 + e % 10
    return t


def _savetxt(path: str, a: np.ndarray) -> None:
    """np.savetxt(path, a, delimiter=",") (default fmt '%.18e', gzip by
    extension, as the reference writes these files) for integer-valued arrays:
    the same text, built as bytes by array operations (_sci18_table of the
    distinct values, gathered, separators added, sign padding dropped). The
    batch input copies are written on a thread pool while the chains run: a
    formatter that held the GIL per value or per row (np.savetxt, str.join)
    starved the launching thread (11 s of a 14 s infer_many, profiles r04j)."""
    a = np.asarray(a)
    if (a.ndim not in (1, 2) or a.dtype.kind not in "iu" or a.size == 0
            or int(a.max()) >= 2 ** 53 or int(a.min()) <= -2 ** 53):
        np.savetxt(path, a, delimiter=",")
        return
    a2 = a.reshape(a.shape[0], -1)
    vals, inv = np.unique(a2, return_inverse=True)
    buf = np.empty(a2.shape + (26,), np.uint8)
    buf[..., :25] = _sci18_table(vals)[inv.reshape(a2.shape)]
    buf[..., 25] = ord(",")
    buf[:, -1, 25] = ord("\n")
    flat = buf.reshape(-1)
    body = flat[flat != 0].tobytes()
    if path.endswith(".gz"):
        with gzip.open(path, "wb", compresslevel=3) as fh:  # same text; numpy's gzip level 9 is ~5x slower here
            fh.write(body)
    else:
        with open(path, "wb") as fh:
            fh.write(body)


def infer(argv: Sequence[str]) -> int:
    f = parse_flags(argv)
    seed, chrom, batch = int(f["seed"]), str(f["chrom"]), int(f["batch"])
    s = serialize_flags(f)
    print("specified flags:\n{}".format(s))
    path = os.path.join(str(f["results_dir"]), "chrom_{}_{}".format(chrom, batch))
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, f"flags{seed}.txt"), "w") as fh:
        fh.write(s)

    mu = np.array([float(x) for x in f["mu"]], dtype=np.float32)
    sigma = np.array([float(x) for x in f["sigma"]], dtype=np.float32)
    K = mu.shape[0]
    theta = control_theta(read_theta(str(f["single_group_dir"]), chrom), K, chrom)

    LAST_TIMINGS.clear()
    t_parse = time.perf_counter()
    # The task's rows end at min((batch + 1) * segment + buffer, n): the files are
    # read that far and no further. segment_index gives the same slice and the
    # same early exit from the rows read as from the whole chromosome (either
    # the file holds at least that many rows, or all of it was read), so the
    # task reads half the chromosome on average instead of all of it.
    need = (batch + 1) * int(f["segment_size"]) + int(f["buffer_size"])
    positions, tot_c, meth_c, tot_k, meth_k = _read_inputs(str(f["data_dir"]), chrom, max_rows=max(need, 1))
    LAST_TIMINGS["parse"] = time.perf_counter() - t_parse

    seg = segment_index(positions.shape[0], batch, int(f["segment_size"]), int(f["buffer_size"]))
    if seg is None:
        print("Batch index is too large for the chromosome")
        return 0
    (lo, hi), (r0, r1) = seg
    ob_c, ob_k = meth_c[lo:hi].astype(np.float32), meth_k[lo:hi].astype(np.float32)
    nt_c, nt_k = tot_c[lo:hi].astype(np.float32), tot_k[lo:hi].astype(np.float32)
    pos = positions[lo:hi].astype(np.int64)
    if np.sum(nt_k < ob_k) != 0 or np.sum(nt_c < ob_c) != 0:
        raise AssertionError("methylated reads exceed total reads")
    ret = slice(r0, r1)

    from concurrent.futures import ThreadPoolExecutor

    T = hi - lo
    max_reads = int(max(nt_c.max(initial=0), nt_k.max(initial=0)))
    log_z: Dict[int, float] = {}
    times: Dict[int, float] = {}
    # The result files are written by a small pool (gzip / zlib release the GIL):
    # the batch's input copies while the chain runs on the GPU, each run's
    # arrays while the next one runs; every write is joined (and its error
    # raised) before the timing files, as the reference writes those last.
    with ThreadPoolExecutor(max_workers=5) as pool:
        writes = _write_batch_inputs(path, ob_c, ob_k, nt_c, nt_k, pos, ret, pool)

        t_dev = time.perf_counter()
        try:
            _infer_runs(f, mu, sigma, theta, K, T, seed, chrom, batch, ob_c, ob_k, nt_c, nt_k, max_reads, ret, path,
                        pool, writes, log_z, times)
        except BaseException:
            _report_write_errors(writes)
            raise
        t_w = time.perf_counter()
        LAST_TIMINGS["device"] = t_w - t_dev
        for w in writes:
            w.result()
        LAST_TIMINGS["writes"] = time.perf_counter() - t_w
    with open(os.path.join(path, f"log_normalizing_constants_optimal_{seed}.txt"), "w") as fh:
        print(log_z, file=fh)
    with open(os.path.join(path, f"optimal_time_{seed}.txt"), "w") as fh:
        print(times, file=fh)
    with open(os.path.join(path, f"optimal_time_backward_{seed}.txt"), "w") as fh:
        print({}, file=fh)
    return 0


# (device, slot) the last infer / infer_many call in this process ran on
# (parallel.task_device); read by tests and tools/bench_pipeline.py.
LAST_DEVICE: Dict[str, int] = {}


def _use_task_device(L) -> None:
    """Selects this task's GPU by the node policy of parallel.task_device (the
    executor's device variables, else a per-node slot over every visible GPU)."""
    from . import _lib, parallel

    dev, slot = parallel.task_device(L)
    if dev != 0 or slot >= 0:
        _lib.check(L.hyg_set_device(dev))
    LAST_DEVICE.clear()
    LAST_DEVICE.update(device=dev, slot=slot)


def _report_write_errors(writes) -> None:
    """On a failed run: wait for the result writes already submitted and report
    any of them that failed too (the run's own exception is the one raised)."""
    from concurrent.futures import wait

    done, _ = wait(writes)
    for w in done:
        e = w.exception()
        if e is not None:
            print(f"hygeia: a result-file write failed as well: {e!r}", file=sys.stderr)


def _infer_runs(f, mu, sigma, theta, K, T, seed, chrom, batch, ob_c, ob_k, nt_c, nt_k, max_reads, ret, path, pool,
                writes, log_z, times) -> None:
    """The chain runs of one `hygeia infer` task, one per --num_resampled_particles
    value (run_inference_two_groups.py:263-322); result writes go to `pool`.
    The chain runs through the host-pointer entry, so this process never needs
    torch: the library is loaded without it (a fresh task saves its import)."""
    from . import _lib, serve, two_group

    # a running node chain server (`hygeia serve`, serve.py: concurrent tasks'
    # chains share launches), else this process runs its chain on its device
    client = serve.task_client()
    timing = os.environ.get("HYGEIA_TASK_TIMING") == "1"  # tools/bench_pipeline.py: the kernels' own time
    L = None

    def local():
        L = _lib.load(import_torch=False)  # (raises without the HIP library)
        _use_task_device(L)
        if timing:
            L.hyg_set_kernel_timing(1)
        return L

    if client is None:
        L = local()
    for M in f["num_resampled_particles"]:
        print(M)
        N = int(M) * (2 * K + K * K)
        pkw = dict(minimum_duration=int(f["minimum_duration"]), omega_case=float(f["omega_case"]),
                   merge_log_prob=float(f["merge_log_prob"]), split_prob=float(f["split_prob"]),
                   num_resampled_ancestors=int(M), num_samples_backward=int(f["num_samples_backward"]),
                   multinomial=bool(f["multinomial"]))
        t0 = time.time()
        res = None
        if client is not None:
            try:
                res, _final_w, ex = client.run_chain(_lib.make_params(mu, sigma, theta, **pkw), max_reads,
                                                     ob_c, nt_c, ob_k, nt_k, seed, chain_id(chrom, batch))
                LAST_TIMINGS["server_batch"] = client.last.get("batch", 0)
                LAST_TIMINGS["server_wait"] = client.last.get("wait_s", 0.0)
                LAST_TIMINGS["kernels"] = LAST_TIMINGS.get("kernels", 0.0) + client.last.get("run_s", 0.0)
            except serve.ServerUnavailable as e:
                print(f"hygeia: chain server unavailable ({e}); running the chain in this process", file=sys.stderr)
                client, res = None, None
                L = local()
                t0 = time.time()
        if res is None:
            model = two_group.CaseControlModel(mu, sigma, theta, max_total_reads=max_reads, max_duration=T + 1,
                                               **pkw)
            try:
                res, _final_w, ex = two_group.run({"control": ob_c, "case": ob_k}, {"control": nt_c, "case": nt_k},
                                                  model, seed, chain_id(chrom, batch))
            finally:
                model.close()
        times[N] = time.time() - t0
        LAST_TIMINGS["chains"] = LAST_TIMINGS.get("chains", 0.0) + times[N]  # (inside "device")
        if timing and L is not None:
            import ctypes as C

            ms3 = (C.c_float * 3)()
            if L.hyg_tg_last_kernel_ms(ms3) == 0:
                LAST_TIMINGS["kernels"] = LAST_TIMINGS.get("kernels", 0.0) + sum(x for x in ms3 if x > 0) / 1000.0
        log_z[N] = float(ex["log_z"])
        pr = res.particle
        for name, arr in ((f"optimal_backward_particles_merged_state_{N}_{seed}",
                           pr["merged_state"].astype(np.int16)[ret]),
                          (f"optimal_backward_particles_control_state_{N}_{seed}",
                           pr["control_state"].astype(np.int16)[ret]),
                          (f"optimal_backward_particles_case_state_{N}_{seed}",
                           pr["case_state"].astype(np.int16)[ret]),
                          (f"optimal_split_probs_{N}_{seed}", ex["split_probs"]),
                          (f"optimal_regime_probs_{N}_{seed}", ex["regime_probs"])):
            writes.append(pool.submit(np.savez_compressed, os.path.join(path, name), arr))


def _write_batch_inputs(path: str, ob_c, ob_k, nt_c, nt_k, pos, ret, pool=None):
    """The batch's input copies (run_inference_two_groups.py:246-254); with a
    pool, submitted to it (returns the futures), else written here."""
    jobs = [("observations_control.csv.gz", ob_c.astype(np.int16)[ret]),
            ("observations_case.csv.gz", ob_k.astype(np.int16)[ret]),
            ("n_total_reads_control.csv.gz", nt_c.astype(np.int16)[ret]),
            ("n_total_reads_case.csv.gz", nt_k.astype(np.int16)[ret]),
            ("positions.csv.gz", pos[ret])]
    if pool is None:
        for name, a in jobs:
            _savetxt(os.path.join(path, name), a)
        return []
    return [pool.submit(_savetxt, os.path.join(path, name), a) for name, a in jobs]


MANY_FLAGS = FLAGS_SPEC + [
    ("batches", "string", "all", "segments to run: 'all' (get_chrom_segments.py: 1 + n // segment_size) or a "
                                 "comma list"),
    ("seeds", "string", "0", "inference seeds, a comma list"),
]


def infer_many(argv: Sequence[str]) -> int:
    """Multi-task `hygeia infer`: every (batch, seed) task of one chromosome in
    ONE batched launch (hyg_tg_run_chains_host, one workgroup per chain, no torch), writing
    the same results_dir/chrom_{chrom}_{batch}/ files as the single-task runs
    `hygeia infer --batch b --seed s` that modules/two_group/4_infer.nf:42-48
    fans out (flags{seed}.txt as that run's flags, identical trajectories,
    probabilities and log Z: the chain id is crc32(chrom) << 32 | batch).
    The chromosome's CSVs are parsed once instead of once per task."""
    f = parse_flags(argv, MANY_FLAGS)
    chrom = str(f["chrom"])
    seeds = [int(x) for x in str(f["seeds"]).split(",") if x != ""]
    S, buf = int(f["segment_size"]), int(f["buffer_size"])
    mu = np.array([float(x) for x in f["mu"]], dtype=np.float32)
    sigma = np.array([float(x) for x in f["sigma"]], dtype=np.float32)
    K = mu.shape[0]
    theta = control_theta(read_theta(str(f["single_group_dir"]), chrom), K, chrom)
    LAST_TIMINGS.clear()
    t_parse = time.perf_counter()
    positions, tot_c, meth_c, tot_k, meth_k = _read_inputs(str(f["data_dir"]), chrom)
    tot_c, meth_c, tot_k, meth_k = (a.astype(np.float32) for a in (tot_c, meth_c, tot_k, meth_k))
    LAST_TIMINGS["parse"] = time.perf_counter() - t_parse
    n = positions.shape[0]
    batches = (list(range(0, n // S + 1)) if str(f["batches"]) == "all"
               else [int(x) for x in str(f["batches"]).split(",") if x != ""])
    tasks = []  # (batch, lo, hi, r0, r1)
    for b in batches:
        seg = segment_index(n, b, S, buf)
        if seg is None:
            print(f"Batch index is too large for the chromosome (batch {b})")
            continue
        (lo, hi), (r0, r1) = seg
        if np.sum(tot_k[lo:hi] < meth_k[lo:hi]) != 0 or np.sum(tot_c[lo:hi] < meth_c[lo:hi]) != 0:
            raise AssertionError("methylated reads exceed total reads")
        tasks.append((b, lo, hi, r0, r1))
    if not tasks:
        return 0
    from concurrent.futures import ThreadPoolExecutor

    # one core stays with the thread that launches the chains (ctypes) and collects their outputs
    pool = ThreadPoolExecutor(max_workers=max(1, min(16, _cpu_budget() - 1)))
    writes, input_jobs = [], []
    for (b, lo, hi, r0, r1) in tasks:
        path = os.path.join(str(f["results_dir"]), "chrom_{}_{}".format(chrom, b))
        os.makedirs(path, exist_ok=True)
        for sd in seeds:
            fs = dict(f, batch=b, seed=sd)
            with open(os.path.join(path, f"flags{sd}.txt"), "w") as fh:
                fh.write(serialize_flags(fs))
        input_jobs.append((_write_batch_inputs, path, meth_c[lo:hi], meth_k[lo:hi], tot_c[lo:hi], tot_k[lo:hi],
                           positions[lo:hi].astype(np.int64), slice(r0, r1)))

    def submit_inputs():  # called just before the launch: the copies compress while the chains run
        while input_jobs:
            writes.append(pool.submit(*input_jobs.pop(0)))

    t_dev = time.perf_counter()
    try:
        return _infer_many_run(f, chrom, seeds, K, mu, sigma, theta, tasks, meth_c, tot_c, meth_k, tot_k, pool,
                               writes, submit_inputs)
    finally:
        t_w = time.perf_counter()
        LAST_TIMINGS["device"] = t_w - t_dev  # (includes submitting the result writes)
        submit_inputs()  # (no-op unless the device phase failed before its launch)
        for w in writes:  # zlib releases the GIL: the files compress in parallel
            w.result()
        pool.shutdown()
        LAST_TIMINGS["writes"] = time.perf_counter() - t_w


def _infer_many_run(f, chrom, seeds, K, mu, sigma, theta, tasks, meth_c, tot_c, meth_k, tot_k, pool, writes,
                    submit_inputs) -> int:
    from . import _lib, two_group

    # the batched host-pointer entry needs no torch (its import is ~2 s of a fresh process)
    _use_task_device(_lib.load(import_torch=False))  # (raises without the HIP library)
    lo_all, hi_all = min(t[1] for t in tasks), max(t[2] for t in tasks)
    counts = {k: a[lo_all:hi_all] for k, a in (("mc", meth_c), ("tc", tot_c), ("mk", meth_k), ("tk", tot_k))}
    max_reads = int(max(tot_c[lo_all:hi_all].max(initial=0), tot_k[lo_all:hi_all].max(initial=0)))
    chains, out = [], 0
    for (b, lo, hi, r0, r1) in tasks:
        for sd in seeds:
            chains.append((lo - lo_all, hi - lo, sd, chain_id(chrom, b), out))
            out += hi - lo
    log_z: Dict[tuple, Dict[int, float]] = {}
    times: Dict[tuple, Dict[int, float]] = {}
    for M in f["num_resampled_particles"]:
        print(M)
        N = int(M) * (2 * K + K * K)
        model = two_group.CaseControlModel(
            mu, sigma, theta, minimum_duration=int(f["minimum_duration"]), omega_case=float(f["omega_case"]),
            merge_log_prob=float(f["merge_log_prob"]), split_prob=float(f["split_prob"]),
            num_resampled_ancestors=int(M), num_samples_backward=int(f["num_samples_backward"]),
            max_total_reads=max_reads, max_duration=max(c[1] for c in chains) + 1,
            multinomial=bool(f["multinomial"]))
        submit_inputs()  # the copies compress on the pool while the chains run (ctypes drops the GIL)
        t0 = time.time()
        try:
            r = two_group.run_chains_host({"control": counts["mc"], "case": counts["mk"]},
                                          {"control": counts["tc"], "case": counts["tk"]}, model, chains, out)
        finally:
            model.close()
        dt = time.time() - t0
        LAST_TIMINGS["chains"] = LAST_TIMINGS.get("chains", 0.0) + dt  # (inside "device")
        status = r["status"]
        if (status != 0).any():
            raise _lib.HygError(int(status[status != 0][0]), "chains failed")
        mg, ct, cs = r["merged"], r["control"], r["case"]
        sp, rp, lz = r["split_probs"], r["regime_probs"], r["log_z"]
        i = 0
        for (b, lo, hi, r0, r1) in tasks:
            path = os.path.join(str(f["results_dir"]), "chrom_{}_{}".format(chrom, b))
            for sd in seeds:
                o, T = chains[i][4], chains[i][1]
                rows, ret = slice(o, o + T), slice(o + r0, o + r1)
                for name, arr in ((f"optimal_backward_particles_merged_state_{N}_{sd}", mg[ret]),
                                  (f"optimal_backward_particles_control_state_{N}_{sd}", ct[ret]),
                                  (f"optimal_backward_particles_case_state_{N}_{sd}", cs[ret]),
                                  (f"optimal_split_probs_{N}_{sd}", sp[rows]),
                                  (f"optimal_regime_probs_{N}_{sd}", rp[rows])):
                    writes.append(pool.submit(np.savez_compressed, os.path.join(path, name), arr))
                log_z.setdefault((b, sd), {})[N] = float(lz[i])
                times.setdefault((b, sd), {})[N] = dt * T / out  # the launch's wall time, pro rata
                i += 1
    for (b, sd), v in log_z.items():
        path = os.path.join(str(f["results_dir"]), "chrom_{}_{}".format(chrom, b))
        with open(os.path.join(path, f"log_normalizing_constants_optimal_{sd}.txt"), "w") as fh:
            print(v, file=fh)
        with open(os.path.join(path, f"optimal_time_{sd}.txt"), "w") as fh:
            print(times[(b, sd)], file=fh)
        with open(os.path.join(path, f"optimal_time_backward_{sd}.txt"), "w") as fh:
            print({}, file=fh)
    return 0


COMMANDS = "preprocess get_chrom_segments infer infer_many aggregate get_dmps"


def main(argv: Sequence[str] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        print("Usage: hygeia [command] [arguments...]")
        return 1
    cmd, rest = argv[0], argv[1:]
    if cmd in ("infer", "infer_many"):
        try:
            return infer(rest) if cmd == "infer" else infer_many(rest)
        except FlagError as e:
            print(f"FATAL Flags parsing error: {e}", file=sys.stderr)
            return 1
    if cmd in ("aggregate", "get_dmps"):
        from . import dmp
        try:
            return dmp.aggregate_main(rest) if cmd == "aggregate" else dmp.get_dmps_main(rest)
        except FlagError as e:
            print(f"FATAL Flags parsing error: {e}", file=sys.stderr)
            return 1
    if cmd == "preprocess":
        from . import preprocess
        try:
            return preprocess.main(rest)
        except FlagError as e:
            print(f"FATAL Flags parsing error: {e}", file=sys.stderr)
            return 1
    if cmd == "get_chrom_segments":
        from . import bed
        try:
            return bed.get_chrom_segments_main(rest)
        except FlagError as e:
            print(f"FATAL Flags parsing error: {e}", file=sys.stderr)
            return 1
    if cmd == "make_bed_file":  # the single-group container's subcommand
        from . import bed
        return bed.make_bed_file_main(rest)
    if cmd == "estimate_parameters_and_regimes":  # the single-group container's subcommand (pipeline step 2)
        from . import single_group
        try:
            return single_group.main(rest)
        except FlagError as e:
            print(f"Error: {e}", file=sys.stderr)
            return 1
    if cmd == "serve":  # the operator-run node chain server for concurrent `infer` tasks (serve.py)
        from . import serve
        return serve.main(rest)
    if cmd in ("version", "-v", "--version"):
        # every 4_infer.nf task runs this for versions.yml (:54-57): no torch
        # import, no HIP library load (_lib.VERSION equals hyg_version())
        from ._lib import VERSION
        print("Hygeia version {} ({})".format(os.environ.get("HYGEIA_VERSION", ""), VERSION))
        return 0
    if cmd in ("help", "-h", "--help"):
        print("Usage: hygeia [command] [arguments...]\n  preprocess - Preprocess BED methylation files (MI355X)\n"
              "  get_chrom_segments - Get chromosome segments\n"
              "  infer     - Run inference on two groups (MI355X)\n"
              "  infer_many - Every (batch, seed) task of a chromosome in one launch (MI355X)\n"
              "  serve     - Node chain server: concurrent infer tasks share launches (MI355X)\n"
              "  aggregate - Aggregate results\n  get_dmps  - Get DMPs (Differentially Methylated Positions)\n"
              "  make_bed_file - Regime BED track of a single-group regimes CSV (MI355X)\n"
              "  estimate_parameters_and_regimes - Single-group regimes and parameters (MI355X)")
        return 0
    if cmd in COMMANDS.split():
        print(f"Error: '{cmd}' is not part of the MI355X inference path; use the reference pipeline step",
              file=sys.stderr)
        return 2
    print(f"Error: Invalid command '{cmd}'\nValid commands are: {COMMANDS}\nUse 'hygeia help' for more information")
    return 2


if __name__ == "__main__":
    sys.exit(main())
