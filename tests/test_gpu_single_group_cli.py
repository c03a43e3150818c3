"""GPU: `hygeia estimate_parameters_and_regimes` end to end, as the two-group
pipeline's step 2 runs it (modules/two_group/2_estimate_parameters_and_regimes.nf:38-52:
--estimate_regime_probabilities --estimate_parameters on the preprocessed
control files), then its theta_{chrom}.csv.gz into `hygeia infer` (step 4).

- the regime probabilities in the regimes CSV are the CPU oracle's
  (oracle/sg_oracle.c:oracle_sg_chain_pe) on the same data -- the files' first
  site consumed as a header, as the R script's read_csv does -- formatted as
  R's format(scientific = FALSE): string for string;
- the theta trace is the oracle's theta rows repeated between updates, the theta
  file its last row, p / omega its conversion (model_functions.R:78-111);
- `hygeia infer` reads that theta file back (with pandas, as the reference:
  within a few ulp) and runs.
"""
import gzip
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MU = "0.95,0.05,0.80,0.20,0.50,0.50"
SIGMA = "0.05,0.05,0.1,0.1,0.1,0.2886751"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    from hygeia_amd import _lib

    if _lib.load().hyg_device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X (gpurun)")


def _write(path, a):  # preprocess_bed.py:463-470: np.savetxt(fmt='%s') of float64, no header
    np.savetxt(path, np.asarray(a, np.float64), fmt="%s", delimiter=",")


def _read_csv(path):
    with gzip.open(path, "rt") as fh:
        lines = fh.read().splitlines()
    return lines[0].split(","), [ln.split(",") for ln in lines[1:]]


@pytest.mark.timeout(300)
def test_estimate_parameters_and_regimes_then_infer(tmp_path):
    from hygeia_amd import cli
    from hygeia_amd import single_group as sgc
    from hygeia_amd import synthetic as syn
    from oracle import sg_binding as sg

    chrom, T, S, every, seed = "7", 2401, 4, 100, 11
    d = syn.simulate(T, S, S, K=6, seed=71, coverage=30.0)
    data = tmp_path / "data"
    data.mkdir()
    pos = syn.positions(T)
    _write(str(data / f"positions_{chrom}.txt.gz"), pos)
    for g in ("control", "case"):
        _write(str(data / f"n_total_reads_{g}_{chrom}.txt.gz"), d[f"tot_{g}"])
        _write(str(data / f"n_methylated_reads_{g}_{chrom}.txt.gz"), d[f"meth_{g}"])
    out = tmp_path / "sg"
    argv = ["estimate_parameters_and_regimes", "--mu", MU, "--sigma", SIGMA, "--u", "3",
            "--n_methylated_reads_csv_file", str(data / f"n_methylated_reads_control_{chrom}.txt.gz"),
            "--genomic_positions_csv_file", str(data / f"positions_{chrom}.txt.gz"),
            "--n_total_reads_csv_file", str(data / f"n_total_reads_control_{chrom}.txt.gz"),
            "--regime_probabilities_csv_file", str(out / f"regimes_{chrom}.csv.gz"),
            "--theta_trace_csv_file", str(out / f"theta_trace_{chrom}.csv.gz"),
            "--p_csv_file", str(out / f"p_{chrom}.csv.gz"), "--kappa_csv_file", str(out / f"kappa_{chrom}.csv.gz"),
            "--omega_csv_file", str(out / f"omega_{chrom}.csv.gz"), "--theta_file", str(out / f"theta_{chrom}.csv.gz"),
            "--estimate_regime_probabilities", "--estimate_parameters", "--randomise_rng_seed", "FALSE",
            "--rng_seed", str(seed), "--n_steps_without_parameter_update", str(every)]
    assert cli.main(argv) == 0

    # the oracle on the same data: the first site is consumed as the header
    meth, tot = d["meth_control"][1:], d["tot_control"][1:]
    p = sg.make_params(K=6, mu=[float(x) for x in MU.split(",")], sigma=[float(x) for x in SIGMA.split(",")], u=3)
    theta0 = np.random.default_rng(seed).standard_normal(36)  # the prior draw of the command
    for i, v in enumerate(theta0):
        p.theta[i] = v
    ref = sg.chain_pe(p, sg.make_pe(every=every), sg.emission(p, meth, tot), seed, 0)
    assert ref["status"] == 0
    n = T - 1

    head, rows = _read_csv(str(out / f"regimes_{chrom}.csv.gz"))
    assert head == ["genomic_position"] + [f"regime_{r + 1}" for r in range(6)]
    assert len(rows) == n
    cols = list(zip(*rows))
    assert list(cols[0]) == list(sgc.r_format_column(pos[1:].astype(np.float64)))
    for r in range(6):
        assert list(cols[1 + r]) == list(sgc.r_format_column(ref["regime_probs"][:, r])), r

    head, rows = _read_csv(str(out / f"theta_trace_{chrom}.csv.gz"))
    assert head == [f"theta_{j + 1}" for j in range(36)] and len(rows) == n
    trace = np.array(rows, dtype=np.float64)
    np.testing.assert_array_equal(trace, ref["theta"][np.arange(n) // every])
    last = ref["theta"][(n - 1) // every]
    assert not np.array_equal(last, theta0)  # the parameters moved

    _, rows = _read_csv(str(out / f"theta_{chrom}.csv.gz"))
    np.testing.assert_array_equal(np.array([float(v[0]) for v in rows]), last)
    p_hat, om_hat, _ = sgc.model_from_theta(last, 6)
    head, rows = _read_csv(str(out / f"p_{chrom}.csv.gz"))
    assert head == [f"regime_{r + 1}" for r in range(6)]
    np.testing.assert_array_equal(np.array(rows, dtype=np.float64), p_hat)
    _, rows = _read_csv(str(out / f"omega_{chrom}.csv.gz"))
    np.testing.assert_array_equal(np.array([float(v[0]) for v in rows]), om_hat)
    _, rows = _read_csv(str(out / f"kappa_{chrom}.csv.gz"))
    assert [float(v[0]) for v in rows] == [2.0] * 6

    # step 4: `hygeia infer` reads the theta file as the reference does, with pandas'
    # default float parser (run_inference_two_groups.py:76-89), which is not
    # correctly rounded for 17-digit text: within 3 ulp of the engine's theta
    th_inf = cli.read_theta(str(out), chrom)
    assert np.all(np.abs(th_inf - last) <= 3 * np.spacing(np.abs(last))), np.max(np.abs(th_inf - last))
    res = tmp_path / "res"
    assert cli.main(["infer", "--chrom", chrom, "--data_dir", str(data), "--single_group_dir", str(out),
                     "--results_dir", str(res), "--seed", "0", "--batch", "0", "--mu", MU, "--sigma", SIGMA]) == 0
    assert os.path.exists(str(res / f"chrom_{chrom}_0" / "optimal_regime_probs_2400_0.npz"))


@pytest.mark.timeout(300)
def test_estimate_parameters_with_kappa_estimated(tmp_path):
    """--is_kappa_fixed FALSE (bin/estimate_parameters_and_regimes:104-107):
    theta of K (K + 1) entries drawn from the prior, the trace and the oracle's
    rows equal, kappa.csv = exp(final log kappa) (:363-365), and `hygeia
    infer` reads the 42-entry theta file as the reference does (omega's logits
    from the last K entries, run_inference_two_groups.py:88)."""
    from hygeia_amd import cli
    from hygeia_amd import single_group as sgc
    from hygeia_amd import synthetic as syn
    from oracle import sg_binding as sg

    chrom, T, S, every, seed = "9", 1201, 2, 50, 5
    d = syn.simulate(T, S, S, K=6, seed=73, coverage=25.0)
    data = tmp_path / "data"
    data.mkdir()
    pos = syn.positions(T)
    _write(str(data / f"positions_{chrom}.txt.gz"), pos)
    for g in ("control", "case"):
        _write(str(data / f"n_total_reads_{g}_{chrom}.txt.gz"), d[f"tot_{g}"])
        _write(str(data / f"n_methylated_reads_{g}_{chrom}.txt.gz"), d[f"meth_{g}"])
    out = tmp_path / "sg"
    argv = ["estimate_parameters_and_regimes", "--mu", MU, "--sigma", SIGMA, "--u", "3",
            "--n_methylated_reads_csv_file", str(data / f"n_methylated_reads_control_{chrom}.txt.gz"),
            "--genomic_positions_csv_file", str(data / f"positions_{chrom}.txt.gz"),
            "--n_total_reads_csv_file", str(data / f"n_total_reads_control_{chrom}.txt.gz"),
            "--regime_probabilities_csv_file", str(out / f"regimes_{chrom}.csv.gz"),
            "--theta_trace_csv_file", str(out / f"theta_trace_{chrom}.csv.gz"),
            "--p_csv_file", str(out / f"p_{chrom}.csv.gz"), "--kappa_csv_file", str(out / f"kappa_{chrom}.csv.gz"),
            "--omega_csv_file", str(out / f"omega_{chrom}.csv.gz"), "--theta_file", str(out / f"theta_{chrom}.csv.gz"),
            "--estimate_regime_probabilities", "--estimate_parameters", "--randomise_rng_seed", "FALSE",
            "--rng_seed", str(seed), "--n_steps_without_parameter_update", str(every), "--is_kappa_fixed", "FALSE"]
    assert cli.main(argv) == 0

    meth, tot = d["meth_control"][1:], d["tot_control"][1:]
    theta0 = np.random.default_rng(seed).standard_normal(42)
    p = sg.make_params(K=6, mu=[float(x) for x in MU.split(",")], sigma=[float(x) for x in SIGMA.split(",")], u=3,
                       kappa=np.exp(theta0[36:]), kappa_fixed=False)
    for i, v in enumerate(theta0):
        p.theta[i] = v
    ref = sg.chain_pe(p, sg.make_pe(every=every), sg.emission(p, meth, tot), seed, 0)
    assert ref["status"] == 0 and ref["theta"].shape[1] == 42
    n = T - 1
    _, rows = _read_csv(str(out / f"regimes_{chrom}.csv.gz"))
    cols = list(zip(*rows))
    for r in range(6):
        assert list(cols[1 + r]) == list(sgc.r_format_column(ref["regime_probs"][:, r])), r
    head, rows = _read_csv(str(out / f"theta_trace_{chrom}.csv.gz"))
    assert head == [f"theta_{j + 1}" for j in range(42)] and len(rows) == n
    np.testing.assert_array_equal(np.array(rows, dtype=np.float64), ref["theta"][np.arange(n) // every])
    last = ref["theta"][(n - 1) // every]
    np.testing.assert_array_equal(last[36:], theta0[36:])  # log kappa never moves
    _, rows = _read_csv(str(out / f"kappa_{chrom}.csv.gz"))
    np.testing.assert_array_equal(np.array([float(v[0]) for v in rows]), np.exp(last[36:]))
    _, rows = _read_csv(str(out / f"theta_{chrom}.csv.gz"))
    assert len(rows) == 42
    th_inf = cli.read_theta(str(out), chrom)
    np.testing.assert_array_equal(cli.control_theta(th_inf, 6), np.concatenate([th_inf[:30], th_inf[36:]]))
    res = tmp_path / "res"
    assert cli.main(["infer", "--chrom", chrom, "--data_dir", str(data), "--single_group_dir", str(out),
                     "--results_dir", str(res), "--seed", "0", "--batch", "0", "--mu", MU, "--sigma", SIGMA]) == 0
    assert os.path.exists(str(res / f"chrom_{chrom}_0" / "optimal_regime_probs_2400_0.npz"))
