"""`hygeia estimate_parameters_and_regimes` host logic on CPU (hygeia_amd/single_group.py):
the R script's flags (bin/estimate_parameters_and_regimes:12-204), its input
quirks (first line read as a header), the theta <-> (p, omega) conversions of
model_functions.R:62-111 with their transpose, R's format(scientific = FALSE)
for the regimes CSV, the theta trace, and that the command fails loudly without
a GPU. The engine's parity is tests/test_gpu_single_group_cli.py.
"""
import gzip

import numpy as np
import pytest

from hygeia_amd import single_group as sgc


def test_flag_defaults_are_the_r_scripts():
    f = sgc.parse_flags([])
    assert f["mu"] == "0.99,0.01,0.80,0.20,0.50,0.50" and f["u"] == 2 and f["n_particles"] == 250
    assert f["is_kappa_fixed"] is True and f["use_adam"] is True and f["normalise_gradients"] is False
    assert f["randomise_rng_seed"] is True and f["rng_seed"] == -73
    assert f["n_steps_without_parameter_update"] == 200 and f["epsilon"] == 0.01
    assert f["learning_rate_exponent"] == 0.1 and f["learning_rate_factor"] == 0.01
    assert f["theta_file"] == "p.csv" and f["omega_csv_file"] == "omega.csv"
    assert f["estimate_parameters"] is False and f["estimate_regime_probabilities"] is False


def test_flag_parsing():
    f = sgc.parse_flags(["--u", "3", "--estimate_parameters", "--use_adam", "FALSE", "--randomise_rng_seed=F",
                         "--rng_seed", "11", "--epsilon", "1e-3", "--estimate_regime_probabilities"])
    assert f["u"] == 3 and f["estimate_parameters"] and f["estimate_regime_probabilities"]
    assert f["use_adam"] is False and f["randomise_rng_seed"] is False and f["rng_seed"] == 11
    assert f["epsilon"] == 1e-3
    for bad in (["--nope", "1"], ["--u"], ["--use_adam", "maybe"], ["--estimate_parameters=TRUE"], ["--u", "2.5"]):
        with pytest.raises(sgc.FlagError):
            sgc.parse_flags(bad)


def test_default_p_is_one_fifth_off_the_diagonal():
    for K in (3, 6, 8):
        p = sgc.default_p(K)
        assert np.all(np.diag(p) == 0.0)
        assert np.all(p[~np.eye(K, dtype=bool)] == 1 / 5)


def test_theta_round_trip_transposes_p():
    """convert_model_parameters_to_theta reads p column-major, the engine and
    convert_theta_to_model_parameters row-major: p comes back transposed (row
    normalised), omega unchanged."""
    rng = np.random.default_rng(3)
    K = 5
    p = rng.uniform(0.1, 1.0, size=(K, K))
    np.fill_diagonal(p, 0.0)
    p /= p.sum(1, keepdims=True)
    omega = rng.uniform(0.8, 0.99, size=K)
    theta = sgc.theta_from_model(p, omega)
    assert theta.shape == (K * K,)
    # block r = log of column r without its diagonal entry
    for r in range(K):
        np.testing.assert_allclose(theta[r * (K - 1):(r + 1) * (K - 1)], np.log(np.delete(p[:, r], r)))
    q, om, _ = sgc.model_from_theta(theta, K)
    pt = p.T / p.T.sum(1, keepdims=True)
    np.testing.assert_allclose(q, pt, rtol=1e-12)
    np.testing.assert_allclose(om, omega, rtol=1e-12)


@pytest.mark.parametrize("x,want", [
    ([1.0, 0.5], ["1.0", "0.5"]),
    ([0.123456789, 1.0], ["0.1234568", "1.0000000"]),
    ([1e-10, 1.0], ["0.0000000001", "1.0000000000"]),
    ([10468.0, 1000000.0], ["  10468", "1000000"]),
    ([0.25, 0.125], ["0.250", "0.125"]),
    ([-1.5, 2.0], ["-1.5", " 2.0"]),
    ([0.0, 0.0], ["0", "0"]),
    ([248946058.0, 12.0], ["248946058", "       12"]),
    ([0.99999999, 0.5], ["1.0", "0.5"]),
])
def test_r_format_known_answers(x, want):
    """R: format(x, scientific = FALSE) with the default 7 digits."""
    assert list(sgc.r_format_column(np.array(x))) == want


def test_read_csv_matrix_consumes_the_first_line(tmp_path):
    path = str(tmp_path / "n.txt.gz")
    with gzip.open(path, "wt") as fh:
        fh.write("12.0,3.0\n4.0,5.0\n6.0,7.0\n")
    a = sgc.read_csv_matrix(path)
    np.testing.assert_array_equal(a, [[4.0, 5.0], [6.0, 7.0]])


def test_theta_trace_repeats_rows_between_updates(tmp_path):
    rows = np.array([[0.5, -1.25], [0.75, 2.0], [1.0, 3.0]])
    path = str(tmp_path / "t.csv")
    sgc.write_theta_trace(path, rows, 7, 3)  # updates at t = 3, 6 -> rows 0,0,0,1,1,1,2
    lines = open(path).read().splitlines()
    assert lines[0] == "theta_1,theta_2"
    assert lines[1:] == ["0.5,-1.25"] * 3 + ["0.75,2"] * 3 + ["1,3"]


def test_vector_files(tmp_path):
    sgc.write_vector(str(tmp_path / "theta.csv.gz"), "data", [0.1, -2.0, 1 / 3])
    with gzip.open(str(tmp_path / "theta.csv.gz"), "rt") as fh:
        lines = fh.read().splitlines()
    assert lines[0] == "data" and [float(v) for v in lines[1:]] == [0.1, -2.0, 1 / 3]


def test_command_fails_loudly_without_a_gpu(tmp_path):
    from hygeia_amd import _lib, cli

    if _lib.load(import_torch=False).hyg_device_count() > 0:
        pytest.skip("a GPU is visible")
    for name, a in (("pos", np.arange(1, 12)[:, None]), ("tot", np.full((11, 2), 10)), ("meth", np.full((11, 2), 4))):
        np.savetxt(str(tmp_path / f"{name}.txt.gz"), a, fmt="%s", delimiter=",")
    argv = ["estimate_parameters_and_regimes", "--genomic_positions_csv_file", str(tmp_path / "pos.txt.gz"),
            "--n_total_reads_csv_file", str(tmp_path / "tot.txt.gz"),
            "--n_methylated_reads_csv_file", str(tmp_path / "meth.txt.gz"),
            "--regime_probabilities_csv_file", str(tmp_path / "out" / "regimes.csv.gz"),
            "--estimate_regime_probabilities"]
    with pytest.raises(_lib.HygError) as e:
        cli.main(argv)
    assert e.value.code == _lib.HYG_EDEVICE
    assert (tmp_path / "out").is_dir()  # create_dirs_for_file ran first, as in the R script
    assert not (tmp_path / "out" / "regimes.csv.gz").exists()


def test_theta_file_reads_back_through_pandas_within_3_ulp(tmp_path):
    """The theta file is read by `hygeia infer` with pandas' default parser (as
    run_inference_two_groups.py:76-79): its 17-digit exponent form comes back
    within 3 ulp, where the shortest text of small values loses thousands."""
    import pandas as pd

    from hygeia_amd import cli

    rng = np.random.default_rng(5)
    x = np.concatenate([rng.standard_normal(3000), rng.standard_normal(3000) * 1e-3])
    sgc.write_vector(str(tmp_path / "theta_1.csv.gz"), "data", x, exp17=True)
    y = cli.read_theta(str(tmp_path), "1")
    assert np.all(np.abs(y - x) <= 3 * np.spacing(np.abs(x)))
    sgc.write_vector(str(tmp_path / "theta_2.csv.gz"), "data", x)
    z = pd.read_table(str(tmp_path / "theta_2.csv.gz"), sep=",")["data"].to_numpy()
    assert np.max(np.abs(z - x) / np.spacing(np.abs(x))) > 100  # why the theta file is not written shortest
