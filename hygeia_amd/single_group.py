"""`hygeia estimate_parameters_and_regimes` on the MI355X path: a drop-in for the
single-group container's R script src/single_group/bin/estimate_parameters_and_regimes,
which the two-group pipeline's step 2 runs per chromosome
(modules/two_group/2_estimate_parameters_and_regimes.nf:38-52) to produce the
theta_{chrom}.csv.gz that `hygeia infer` reads.

Same flags (R argparser spellings and defaults, :10-204), same inputs and
outputs (:216-379); the engine is the C ABI's single-group SMC with optimal
finite-state resampling, online marginal smoothing and (--estimate_parameters)
online parameter estimation (hyg_sg_run_chain_host[_pe], the HIP kernels of
libhygeia_amd.so; no CPU path). Reproduced quirks:

- read_csv with a header (input_output_functions.R:10-20): the pipeline's count
  files have none, so their first CpG site becomes the header and is dropped;
- convert_model_parameters_to_theta takes p[p != -1] column-major
  (model_functions.R:62-76) while the engine reads theta blocks as rows: a p
  from --p_input_csv_file enters transposed, and convert_theta_to_model_parameters
  (:78-111) writes p back row-major;
- the default p (:243-247) has 1/5 off the diagonal whatever the number of
  regimes (the engine's softmax normalises the rows);
- --estimate_parameters starts theta from the prior, K^2 standard normal draws
  (sampleFromParameterPriorCpp, singleGroup.cpp:18-35, singleGroup.h:480-483),
  not from --p / --omega;
- --randomise_rng_seed defaults to TRUE (:191-197): runs are not reproducible
  unless it is FALSE (then --rng_seed seeds every draw);
- the regimes CSV holds R format(scientific = FALSE) strings (:326-338):
  fixed notation, 7 significant digits, one width and one number of decimals
  per column (`r_format_column`).

Parity unpinned where R is the reference: R's RNG (arma::randn / the engine's
streams) is not reproduced, and readr's number writer is replaced by Python's
shortest round-trip text (the same values), except in the theta file, written
with 17 significant digits in exponent form so that `hygeia infer`'s pandas
parser reads it within 3 ulp (write_vector).
"""
from __future__ import annotations

import gzip
import math
import os
import sys
from typing import Dict, Sequence

import numpy as np

from .cli import FlagError

# (name, kind, default) in the R script's definition order
# (bin/estimate_parameters_and_regimes:12-204); kinds: str, int, double,
# logical (a value: TRUE / FALSE / T / F ...), flag (no value: TRUE if present)
FLAGS = [
    ("mu", "str", "0.99,0.01,0.80,0.20,0.50,0.50"),
    ("sigma", "str", "0.05,0.05,0.20,0.20,0.20,0.2886751"),
    ("u", "int", 2),
    ("kappa", "str", "2,2,2,2,2,2"),
    ("omega", "str", "0.995,0.975,0.950,0.925,0.900,0.900"),
    ("p_input_csv_file", "str", None),
    ("kappa_input_csv_file", "str", None),
    ("omega_input_csv_file", "str", None),
    ("n_methylated_reads_csv_file", "str", None),
    ("genomic_positions_csv_file", "str", None),
    ("n_total_reads_csv_file", "str", None),
    ("regime_probabilities_csv_file", "str", None),
    ("theta_trace_csv_file", "str", None),
    ("omega_csv_file", "str", "omega.csv"),
    ("kappa_csv_file", "str", "kappa.csv"),
    ("p_csv_file", "str", "p.csv"),
    ("theta_file", "str", "p.csv"),
    ("is_kappa_fixed", "logical", True),
    ("n_particles", "int", 250),
    ("estimate_regime_probabilities", "flag", False),
    ("estimate_parameters", "flag", False),
    ("epsilon", "double", 0.01),
    ("normalise_gradients", "logical", False),
    ("use_adam", "logical", True),
    ("n_steps_without_parameter_update", "int", 200),
    ("learning_rate_exponent", "double", 0.1),
    ("learning_rate_factor", "double", 0.01),
    ("root_dir", "str", "./src/r"),
    ("randomise_rng_seed", "logical", True),
    ("rng_seed", "int", -73),
]

_TRUE = {"TRUE", "T", "true", "True"}
_FALSE = {"FALSE", "F", "false", "False"}


def parse_flags(argv: Sequence[str]) -> Dict[str, object]:
    """argparser-style parsing: `--name value` or `--name=value`; logical values
    as R's as.logical reads them; flags take no value."""
    spec = {n: (k, d) for n, k, d in FLAGS}
    out = {n: d for n, _, d in FLAGS}
    argv = list(argv)
    i = 0
    while i < len(argv):
        a = argv[i]
        if not a.startswith("--"):
            raise FlagError(f"unexpected argument {a!r}")
        name, eq, val = a[2:].partition("=")
        if name not in spec:
            raise FlagError(f"unknown argument --{name}")
        kind = spec[name][0]
        if kind == "flag":
            if eq:
                raise FlagError(f"--{name} is a flag and takes no value")
            out[name] = True
            i += 1
            continue
        if not eq:
            if i + 1 >= len(argv):
                raise FlagError(f"--{name} needs a value")
            val = argv[i + 1]
            i += 2
        else:
            i += 1
        try:
            if kind == "int":  # as.integer: "3" and "3.0" read as 3
                v = float(val)
                if v != int(v):
                    raise ValueError("not an integer")
                out[name] = int(v)
            elif kind == "double":
                out[name] = float(val)
            elif kind == "logical":
                if val in _TRUE:
                    out[name] = True
                elif val in _FALSE:
                    out[name] = False
                else:
                    raise ValueError("not a logical")
            else:
                out[name] = val
        except ValueError as e:
            raise FlagError(f"invalid value for --{name}: {val!r} ({e})")
    return out


def _numbers(s: str) -> np.ndarray:
    return np.array([float(x) for x in str(s).split(",") if x.strip() != ""], dtype=np.float64)


# ------------------------------------------------------------------- inputs
def _open(path: str, mode: str = "rt"):
    return gzip.open(path, mode) if path.endswith(".gz") else open(path, mode)


def read_csv_matrix(path: str) -> np.ndarray:
    """readr::read_csv(file) as a numeric matrix (read_from_csv_file,
    input_output_functions.R:10-20): the FIRST LINE IS THE HEADER, whatever it
    holds, so a headerless count file loses its first CpG site (Appendix B.3)."""
    with _open(path) as fh:
        header = fh.readline()
        ncol = len(header.rstrip("\r\n").split(","))
        rows = fh.read()
    if not rows.strip():
        return np.zeros((0, ncol))
    a = np.loadtxt(rows.splitlines(), delimiter=",", dtype=np.float64, ndmin=2)
    if a.shape[1] != ncol:
        raise ValueError(f"{path}: {a.shape[1]} columns, header has {ncol}")
    return a


def default_p(K: int) -> np.ndarray:
    """The initial transition matrix of the R script (:243-247):
    matrix(c(rep(c(0, rep(1/5, K)), K - 1), 0), K, K), filled column-major."""
    v = np.concatenate([np.tile(np.concatenate([[0.0], np.full(K, 1 / 5)]), K - 1), [0.0]])
    return v.reshape(K, K, order="F")


def theta_from_model(p: np.ndarray, omega: np.ndarray, kappa=None) -> np.ndarray:
    """convert_model_parameters_to_theta (model_functions.R:65-78):
    diag(p) <- -1; c(log(p[p != -1]), logit(omega)) -- p[p != -1] in R's
    column-major order -- and log(kappa) appended when kappa is estimated
    (kappa given)."""
    p = np.array(p, dtype=np.float64)
    np.fill_diagonal(p, -1.0)
    flat = p.flatten(order="F")
    off = flat[flat != -1.0]
    with np.errstate(divide="ignore"):
        parts = [np.log(off), np.log(omega) - np.log(1.0 - omega)]
        if kappa is not None:
            parts.append(np.log(np.asarray(kappa, dtype=np.float64)))
        return np.concatenate(parts)


def model_from_theta(theta: np.ndarray, K: int):
    """convert_theta_to_model_parameters (model_functions.R:81-111): row r of p
    = exp(normalise_exp(theta block r)) off the diagonal (row-major), omega =
    inverse_logit(theta[K(K-1):K^2]) and, when theta carries the K log kappa
    entries (kappa estimated), kappa = exp(theta[K^2:K(K+1)]) (else None)."""
    p = np.zeros((K, K))
    for r in range(K):
        blk = theta[r * (K - 1):(r + 1) * (K - 1)]
        m = blk.max()
        lz = m + math.log(np.exp(blk - m).sum())
        p[r, [c for c in range(K) if c != r]] = np.exp(blk - lz)
    omega = 1.0 / (1.0 + np.exp(-theta[K * (K - 1):K * K]))
    kappa = np.exp(theta[K * K:K * (K + 1)]) if theta.shape[0] >= K * (K + 1) else None
    return p, omega, kappa


# ------------------------------------------------------------------ outputs
def r_format_column(x: np.ndarray, digits: int = 7) -> np.ndarray:
    """R's format(x, scientific = FALSE) of a double vector (formatReal in fixed
    notation): every element needs the fewest significant digits (<= `digits`)
    that show it to `digits` significant digits; the column takes the largest
    number of decimals any element needs and the widest integer part, and every
    element is printed "%*.*f" with that width and those decimals (right
    aligned, spaces). Returns an array of str. (R's own digit search uses long
    double arithmetic; here it is Python's correctly rounded '%.6e', so a value
    within an ulp of a rounding tie may choose one digit differently: parity
    unpinned, R is absent.)"""
    x = np.asarray(x, dtype=np.float64)
    if x.size == 0:
        return np.array([], dtype=str)
    fin = np.isfinite(x)
    rgt, left = 0, 1
    # distinct values decide the column's decimals (a column of probabilities or
    # positions has far fewer distinct values than rows)
    for v in np.unique(x[fin]):
        if v == 0.0:
            continue
        m, e = ("%.*e" % (digits - 1, abs(v))).split("e")
        kp = int(e)
        sig = len(m.replace(".", "").rstrip("0")) or 1
        rgt = max(rgt, sig - kp - 1)
        left = max(left, kp + 1)
    neg = bool(np.any(x[fin] < 0))
    out = np.array(["%.*f" % (rgt, v) for v in x.tolist()], dtype=object)
    width = max(len(s) for s in out) if out.size else 0
    width = max(width, neg + left + rgt + (rgt != 0))
    return np.array([s.rjust(width) for s in out])


def _shortest(v: float) -> str:
    """A double as the shortest text that reads back to the same value."""
    if v == int(v) and abs(v) < 1e15:
        return str(int(v))
    return repr(float(v))


def write_csv(path: str, header: Sequence[str], columns: Sequence[Sequence[str]], level: int = 6) -> None:
    """readr::write_csv of string columns (gzip by extension, as readr)."""
    body = "\n".join(",".join(row) for row in zip(*columns))
    text = ",".join(header) + "\n" + (body + "\n" if body else "")
    with (gzip.open(path, "wt", compresslevel=level) if path.endswith(".gz") else open(path, "w")) as fh:
        fh.write(text)


def write_vector(path: str, name: str, values: Sequence[float], exp17: bool = False) -> None:
    """write_to_csv_file(tibble(name = values)) (input_output_functions.R:4-7).
    exp17: 17 significant digits in exponent form ('%.16e'), which pandas'
    default parser -- `hygeia infer` reads the theta file with it, as
    run_inference_two_groups.py:76-79 does -- reads within 3 ulp; the shortest
    text of a small value ('0.00123...') has up to 21 mantissa characters, of
    which it keeps 17 (errors of thousands of ulp, tests/test_single_group_cli.py)."""
    write_csv(path, [name], [["%.16e" % v if exp17 else _shortest(v) for v in values]])


def write_theta_trace(path: str, theta_rows: np.ndarray, n_sites: int, every: int) -> None:
    """The thetaEstimates of every SMC step (OnlineParameterEstimation.h:42-61:
    theta_0 at t = 0, then theta after step t's update, which changes it only
    when t % every == 0), columns theta_1 .. theta_dim: row t is the engine's
    row t // every. Each distinct row is formatted once and repeated."""
    dim = theta_rows.shape[1]
    head = (",".join(f"theta_{j + 1}" for j in range(dim)) + "\n").encode()
    opener = gzip.open(path, "wb", compresslevel=1) if path.endswith(".gz") else open(path, "wb")
    with opener as fh:
        fh.write(head)
        for i in range(theta_rows.shape[0]):
            reps = min(every, n_sites - i * every) if i > 0 else min(every, n_sites)
            if reps <= 0:
                break
            line = (",".join(_shortest(v) for v in theta_rows[i].tolist()) + "\n").encode()
            fh.write(line * reps)


def write_regimes(path: str, positions: np.ndarray, probs: np.ndarray) -> None:
    """regimes CSV (:326-338): genomic_position, regime_1 .. regime_K, each column
    R format(scientific = FALSE) text."""
    K = probs.shape[1]
    cols = [r_format_column(positions)] + [r_format_column(probs[:, r]) for r in range(K)]
    write_csv(path, ["genomic_position"] + [f"regime_{r + 1}" for r in range(K)], cols)


# ------------------------------------------------------------------- engine
def run_engine(L, K: int, u: int, alpha, beta, kappa, theta_init, epsilon: float, n_particles: int,
               meth: np.ndarray, tot: np.ndarray, seed: int, chain_id: int, estimate_parameters: bool, pe_flags=None,
               is_kappa_fixed: bool = True):
    """runOnlineCombinedInferenceCpp (singleGroup.cpp:76-189) through the C ABI:
    regime probabilities [T][K] and, with parameter estimation, the engine's
    theta rows [1 + (T - 1) / every][dim] (dim = K^2, or K (K + 1) with kappa
    estimated: then theta_init carries log kappa and `kappa` is unused, as
    vartheta has no kappa, model_functions.R:48-54)."""
    import ctypes as C

    from . import _lib

    dim = K * K if is_kappa_fixed else K * (K + 1)
    if len(theta_init) != dim:
        raise ValueError(f"theta has {len(theta_init)} entries, the model {dim}")
    p = _lib.SgParams()
    L.hyg_sg_params_default(C.byref(p))
    p.n_regimes, p.minimum_duration, p.num_particles_max = K, int(u), int(n_particles)
    p.resample_type, p.is_kappa_fixed, p.theta_len = 2, int(bool(is_kappa_fixed)), dim
    for r in range(K):
        p.alpha[r], p.beta[r] = float(alpha[r]), float(beta[r])
        p.kappa[r] = float(kappa[r]) if is_kappa_fixed else 0.0
    for i, v in enumerate(theta_init):
        p.theta[i] = float(v)
    p.epsilon = float(epsilon)
    T, S = tot.shape
    meth = np.ascontiguousarray(meth, dtype=np.uint16)
    tot = np.ascontiguousarray(tot, dtype=np.uint16)
    h = C.c_void_p()
    _lib.check(L.hyg_sg_model_create(C.byref(p), max(int(tot.max(initial=0)), 1), T + 10, C.byref(h)))
    ptr = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    try:
        probs = np.empty((T, K), np.float64)
        if not estimate_parameters:
            _lib.check(L.hyg_sg_run_chain_host(h, ptr(meth), ptr(tot), S, T, seed, chain_id, ptr(probs)))
            return probs, None
        pe = _lib.SgPeParams()
        L.hyg_sg_pe_params_default(C.byref(pe))
        pe.use_adam = int(pe_flags["use_adam"])
        pe.normalise_gradients = int(pe_flags["normalise_gradients"])
        pe.n_steps_without_update = int(pe_flags["n_steps_without_parameter_update"])
        pe.learning_rate_exponent = float(pe_flags["learning_rate_exponent"])
        pe.learning_rate_factor = float(pe_flags["learning_rate_factor"])
        ch = _lib.SgChain(0, T, 0, seed, chain_id, 0)
        rows = int(L.hyg_sg_pe_theta_rows(C.byref(ch), 1, pe.n_steps_without_update))
        theta = np.empty((rows, dim), np.float64)
        _lib.check(L.hyg_sg_run_chain_host_pe(h, C.byref(pe), ptr(meth), ptr(tot), S, T, seed, chain_id, ptr(probs),
                                              ptr(theta)))
        return probs, theta
    finally:
        L.hyg_sg_model_destroy(h)


def main(argv: Sequence[str]) -> int:
    f = parse_flags(argv)
    # the seed of every draw: --rng_seed when --randomise_rng_seed FALSE (:208-210)
    seed = int(f["rng_seed"]) & (2 ** 64 - 1) if not f["randomise_rng_seed"] else \
        int.from_bytes(os.urandom(8), "little")
    u = int(f["u"])
    kappa = (read_csv_matrix(f["kappa_input_csv_file"])[:, 0] if f["kappa_input_csv_file"]
             else _numbers(f["kappa"]))
    omega = (read_csv_matrix(f["omega_input_csv_file"])[:, 0] if f["omega_input_csv_file"]
             else _numbers(f["omega"]))
    sigma, mu = _numbers(f["sigma"]), _numbers(f["mu"])
    K = mu.shape[0]
    p = read_csv_matrix(f["p_input_csv_file"]) if f["p_input_csv_file"] else default_p(K)
    fixed = bool(f["is_kappa_fixed"])
    dim_theta = K * K if fixed else K * (K + 1)  # get_known_parameters (model_functions.R:48-54)
    for path in (f["n_methylated_reads_csv_file"], f["genomic_positions_csv_file"], f["n_total_reads_csv_file"],
                 f["regime_probabilities_csv_file"], f["theta_trace_csv_file"], f["p_csv_file"],
                 f["omega_csv_file"], f["kappa_csv_file"], f["theta_file"]):  # create_dirs_for_file (:250-262)
        if isinstance(path, str) and os.path.dirname(path):
            os.makedirs(os.path.dirname(path), exist_ok=True)
    # get_known_parameters (model_functions.R:36-59)
    nu = mu * (1 - mu) / sigma ** 2 - 1
    alpha, beta = mu * nu, (1 - mu) * nu
    if f["estimate_parameters"]:  # sampleFromParameterPriorCpp: theta ~ N(0, I) (singleGroup.h:480-483)
        theta_init = np.random.default_rng(seed).standard_normal(dim_theta)
    else:
        theta_init = theta_from_model(p, omega, None if fixed else kappa)
    positions = read_csv_matrix(f["genomic_positions_csv_file"])[:, 0]
    tot = read_csv_matrix(f["n_total_reads_csv_file"])
    meth = read_csv_matrix(f["n_methylated_reads_csv_file"])
    if tot.shape != meth.shape or tot.shape[0] != positions.shape[0]:
        raise ValueError(f"inconsistent inputs: positions {positions.shape}, totals {tot.shape}, "
                         f"methylated {meth.shape}")
    if np.any(meth > tot) or np.any(tot < 0) or np.any(tot != np.rint(tot)) or np.any(tot > 65535):
        raise ValueError("read counts must be integers with 0 <= methylated <= total <= 65535")

    from . import _lib
    from .cli import _use_task_device

    L = _lib.load(import_torch=False)
    _use_task_device(L)
    probs, theta = run_engine(L, K, u, alpha, beta, kappa, theta_init, f["epsilon"], f["n_particles"], meth, tot,
                              seed, 0, bool(f["estimate_parameters"]), f, is_kappa_fixed=fixed)
    if f["estimate_regime_probabilities"]:
        write_regimes(f["regime_probabilities_csv_file"], positions, probs)
    if f["estimate_parameters"]:
        T = positions.shape[0]
        every = int(f["n_steps_without_parameter_update"])
        write_theta_trace(f["theta_trace_csv_file"], theta, T, every)
        last = theta[(T - 1) // every]
        p_hat, omega_hat, kappa_hat = model_from_theta(last, K)
        write_csv(f["p_csv_file"], [f"regime_{r + 1}" for r in range(K)],
                  [[_shortest(v) for v in p_hat[:, c]] for c in range(K)])
        write_vector(f["omega_csv_file"], "omega", omega_hat)
        # the final estimate when kappa is estimated, else the given kappa (:363-369)
        write_vector(f["kappa_csv_file"], "kappa", kappa if fixed else kappa_hat)
        write_vector(f["theta_file"], "data", last, exp17=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
