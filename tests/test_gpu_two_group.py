"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar: bit-exact trajectories (merged / control / case int16 arrays), bit-exact
split and regime probabilities (f32), bit-exact log normalising constant and
final weights (f64) -- the arithmetic contract of include/hyg_arith.h makes the
kernels and the oracle compute the same numbers.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _have_gpu():
    from hygeia_amd import _lib

    return _lib.load().hyg_device_count() > 0


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not _have_gpu():
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X (gpurun)")


def _setup(oracle, K, M, B, T, S, cov, dseed, split_frac=0.1):
    from hygeia_amd import synthetic as syn

    mu, sg = syn.regime_params(K)
    d = syn.simulate(T, S, S, K=K, seed=dseed, coverage=cov, split_frac=split_frac)
    p = oracle.make_params(K=K, M=M, B=B, mu=mu, sigma=sg)
    theta = np.array(p.theta[: p.theta_len])
    return mu, sg, theta, d, p


def _model(mu, sg, theta, M, B, max_reads, max_dur):
    from hygeia_amd import two_group

    return two_group.CaseControlModel(mu, sg, theta, num_resampled_ancestors=M, num_samples_backward=B,
                                      max_total_reads=max_reads, max_duration=max_dur)


CASES = [
    # K, M, B, T, S, coverage, data seed, inference seed
    (6, 50, 25, 1500, 4, 100.0, 11, 0),   # the pipeline configuration, short chain
    (6, 50, 25, 800, 4, 1000.0, 12, 1),   # high coverage: unbiased-fallback steps occur
    (6, 10, 5, 600, 2, 30.0, 13, 2),      # small M / B
    (4, 20, 8, 700, 3, 60.0, 14, 3),
    (3, 7, 4, 500, 1, 10.0, 15, 4),       # K = 3, one sample per group
    (2, 5, 3, 300, 2, 20.0, 16, 5),       # K = 2 (empty uniform case-regime sets)
    (6, 50, 25, 1, 4, 100.0, 17, 6),      # a single site: no filter step
    (6, 50, 25, 2, 4, 100.0, 18, 7),
    (6, 50, 25, 5, 4, 100.0, 19, 8),
    (12, 50, 25, 300, 6, 100.0, 20, 9),   # K = 12 (config C5 regimes): N_max = 8400
    (6, 100, 30, 400, 4, 100.0, 21, 10),  # M > 64: general weight / backward paths
    (4, 30, 70, 300, 2, 50.0, 22, 11),    # B > 64: general backward path
]


@pytest.mark.parametrize("K,M,B,T,S,cov,dseed,seed", CASES)
def test_chain_bit_exact(oracle, K, M, B, T, S, cov, dseed, seed):
    from hygeia_amd import two_group

    mu, sg, theta, d, p = _setup(oracle, K, M, B, T, S, cov, dseed)
    E = oracle.emission(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
    ref = oracle.chain(p, E, seed, 1000 + seed)
    assert ref["status"] == 0
    maxr = int(max(d["tot_control"].max(), d["tot_case"].max()))
    model = _model(mu, sg, theta, M, B, maxr, T + 5)
    res, fw, ex = two_group.run({"control": d["meth_control"], "case": d["meth_case"]},
                                {"control": d["tot_control"], "case": d["tot_case"]}, model, seed, 1000 + seed)
    pr = res.particle
    np.testing.assert_array_equal(pr["merged_state"], ref["merged"])
    np.testing.assert_array_equal(pr["control_state"], ref["control"])
    np.testing.assert_array_equal(pr["case_state"], ref["case"])
    np.testing.assert_array_equal(ex["split_probs"], ref["split_probs"])
    np.testing.assert_array_equal(ex["regime_probs"], ref["regime_probs"])
    assert ex["log_z"] == ref["log_z"]
    np.testing.assert_array_equal(fw, ref["final_log_weights"])


WIDTHS = [256, 512, 768]


@pytest.fixture
def force_width():
    """Pins the chain workgroup size (hyg_tg_force_threads) for one test and
    restores the automatic choice afterwards."""
    from hygeia_amd import _lib

    L = _lib.load()

    def set_width(fwd, bwd=None):
        _lib.check(L.hyg_tg_force_threads(fwd, fwd if bwd is None else bwd))

    yield set_width
    L.hyg_tg_force_threads(0, 0)


@pytest.mark.parametrize("width", WIDTHS)
@pytest.mark.parametrize("case", [0, 1, 2, 4, 9, 10])
def test_chain_bit_exact_every_width(oracle, force_width, width, case):
    """Every chain-kernel width computes the same bits: 256 threads (up to three
    chains per CU, C3 on one GPU), 512 (one per CU: an 8-GPU rank; the C5
    width) and 768, forward and backward (the backward at the same width, and
    the 256-thread backward behind a wide forward)."""
    from hygeia_amd import two_group

    K, M, B, T, S, cov, dseed, seed = CASES[case]
    mu, sg, theta, d, p = _setup(oracle, K, M, B, T, S, cov, dseed)
    E = oracle.emission(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
    ref = oracle.chain(p, E, seed, 1000 + seed)
    maxr = int(max(d["tot_control"].max(), d["tot_case"].max()))
    model = _model(mu, sg, theta, M, B, maxr, T + 5)
    for bwd in (width, 256):
        force_width(width, bwd)
        res, fw, ex = two_group.run({"control": d["meth_control"], "case": d["meth_case"]},
                                    {"control": d["tot_control"], "case": d["tot_case"]}, model, seed, 1000 + seed)
        pr = res.particle
        np.testing.assert_array_equal(pr["merged_state"], ref["merged"])
        np.testing.assert_array_equal(pr["control_state"], ref["control"])
        np.testing.assert_array_equal(pr["case_state"], ref["case"])
        np.testing.assert_array_equal(ex["split_probs"], ref["split_probs"])
        np.testing.assert_array_equal(ex["regime_probs"], ref["regime_probs"])
        assert ex["log_z"] == ref["log_z"]
        np.testing.assert_array_equal(fw, ref["final_log_weights"])


def test_width_selection_by_chains_per_cu():
    """The automatic width: 512 threads up to one chain per CU, 256 beyond (C3
    on one GPU, an 8-GPU rank of C4), 512 for the C5 shape whose LDS allows
    one chain per CU anyway."""
    from hygeia_amd import _lib, synthetic as syn, two_group

    L = _lib.load()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    mu, sg = syn.regime_params(6)
    m6 = two_group.CaseControlModel(mu, sg, two_group.uniform_theta(6), max_total_reads=200, max_duration=100)
    assert [L.hyg_tg_threads_per_chain(m6.handle, n) for n in (1, cus, cus + 1, 582)] == [512, 512, 256, 256]
    # the C3 shape keeps three chains per CU at 256 threads (LDS <= 160 KiB / 3)
    assert L.hyg_tg_chains_per_cu(m6.handle, 582) == 3
    assert L.hyg_tg_chains_per_cu(m6.handle, 73) >= 1
    mu, sg = syn.regime_params(12)
    m12 = two_group.CaseControlModel(mu, sg, two_group.uniform_theta(12), max_total_reads=200, max_duration=100)
    assert L.hyg_tg_threads_per_chain(m12.handle, 10) == 512
    assert L.hyg_tg_threads_per_chain(m12.handle, 1164) == 512
    # the choice follows the current device's own CU count (cached per device):
    # on a faked 64-CU device 100 chains are more than one per CU
    assert L.hyg_tg_device_cus(0) == cus
    try:
        assert L.hyg_tg_set_device_cus(0, 64) == 0
        assert [L.hyg_tg_threads_per_chain(m6.handle, n) for n in (64, 100)] == [512, 256]
    finally:
        L.hyg_tg_set_device_cus(0, 0)
    assert L.hyg_tg_device_cus(0) == cus
    assert [L.hyg_tg_threads_per_chain(m6.handle, n) for n in (64, 100)] == [512, 512]


def test_zero_coverage_stretch(oracle):
    """Missing data (n = 0 for every sample) contributes exactly 0 (TFP BB at n=0)."""
    from hygeia_amd import two_group

    mu, sg, theta, d, p = _setup(oracle, 6, 50, 25, 900, 4, 80.0, 21)
    for k in ("meth_control", "tot_control", "meth_case", "tot_case"):
        d[k][200:400] = 0
        d[k][600:610, :2] = 0
    E = oracle.emission(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
    assert np.all(E[200:400] == 0.0)
    ref = oracle.chain(p, E, 3, 77)
    model = _model(mu, sg, theta, 50, 25, int(d["tot_case"].max()), 1000)
    res, fw, ex = two_group.run({"control": d["meth_control"], "case": d["meth_case"]},
                                {"control": d["tot_control"], "case": d["tot_case"]}, model, 3, 77)
    np.testing.assert_array_equal(res.particle["control_state"], ref["control"])
    np.testing.assert_array_equal(res.particle["case_state"], ref["case"])
    np.testing.assert_array_equal(ex["regime_probs"], ref["regime_probs"])


def test_batched_chains_and_emission(oracle):
    """Many chains of different lengths in one launch (the sharded driver's
    path), device-resident inputs; each chain equals its own oracle run."""
    from hygeia_amd import two_group

    K, M, B, S = 6, 50, 25, 4
    mu, sg, theta, d, p = _setup(oracle, K, M, B, 5300, S, 100.0, 31)
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(np.ascontiguousarray(d[k]).view(np.int16)).to(dev) for k in
         ("meth_control", "tot_control", "meth_case", "tot_case")}
    lengths = [1000, 37, 1, 2200, 963, 1000]
    chains, site, out = [], 0, 0
    for i, n in enumerate(lengths):
        chains.append((site, n, 5 + i % 2, 900 + i, out))
        site += n
        out += n
    model = _model(mu, sg, theta, M, B, int(max(d["tot_control"].max(), d["tot_case"].max())), 3000)
    dc = two_group.DeviceChains(model, chains, out, device=dev, final_weights=True)
    E = dc.emission(t["meth_control"], t["tot_control"], t["meth_case"], t["tot_case"])
    dc.run(E)
    torch.cuda.synchronize()
    E_ref = oracle.emission(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
    np.testing.assert_array_equal(E.cpu().numpy(), E_ref)
    assert (dc.status.cpu().numpy() == 0).all()
    for i, (s0, n, seed, cid, o0) in enumerate(chains):
        ref = oracle.chain(p, E_ref[s0:s0 + n], seed, cid)
        np.testing.assert_array_equal(dc.merged[o0:o0 + n].cpu().numpy(), ref["merged"])
        np.testing.assert_array_equal(dc.control[o0:o0 + n].cpu().numpy(), ref["control"])
        np.testing.assert_array_equal(dc.case[o0:o0 + n].cpu().numpy(), ref["case"])
        np.testing.assert_array_equal(dc.split_probs[o0:o0 + n].cpu().numpy(), ref["split_probs"])
        np.testing.assert_array_equal(dc.regime_probs[o0:o0 + n].cpu().numpy(), ref["regime_probs"])
        assert dc.log_z[i].item() == ref["log_z"]
        np.testing.assert_array_equal(dc.final_w[i].cpu().numpy(), ref["final_log_weights"])


def test_batched_host_entry(oracle):
    """hyg_tg_run_chains_host (infer_many's torch-free launch): overlapping
    chains over one count range (segments with buffers, two seeds), outputs
    in any row order; each chain equals its own oracle run. Bad chain ranges
    and counts are refused before anything runs."""
    from hygeia_amd import _lib, two_group

    K, M, B, S = 6, 50, 25, 4
    mu, sg, theta, d, p = _setup(oracle, K, M, B, 3000, S, 100.0, 33)
    obs = {"control": d["meth_control"], "case": d["meth_case"]}
    tot = {"control": d["tot_control"], "case": d["tot_case"]}
    spans = [(0, 1200), (800, 1400), (1800, 1200), (2999, 1)]  # (site_begin, n_sites)
    chains, out = [], 0
    for j, (s0, n) in enumerate(reversed(spans)):  # output rows in reverse site order
        for seed in (0, 1):
            chains.append((s0, n, seed, 4000 + j, out))
            out += n
    model = _model(mu, sg, theta, M, B, int(max(d["tot_control"].max(), d["tot_case"].max())), 1500)
    r = two_group.run_chains_host(obs, tot, model, chains, out + 7, final_weights=True)
    assert (r["status"] == 0).all()
    E_ref = oracle.emission(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
    for i, (s0, n, seed, cid, o0) in enumerate(chains):
        ref = oracle.chain(p, E_ref[s0:s0 + n], seed, cid)
        for k, rk in (("merged", "merged"), ("control", "control"), ("case", "case"),
                      ("split_probs", "split_probs"), ("regime_probs", "regime_probs")):
            np.testing.assert_array_equal(r[k][o0:o0 + n], ref[rk])
        assert r["log_z"][i] == ref["log_z"]
        np.testing.assert_array_equal(r["final_w"][i], ref["final_log_weights"])
    # past the sites (the C entry refuses it) / past the output rows (refused by
    # run_chains_host's own range check, before the C entry, as overlapping rows are)
    for bad, err in (([(2500, 600, 0, 1, 0)], _lib.HygError), ([(0, 100, 0, 1, out)], ValueError),
                     ([(0, 100, 0, 1, 0), (0, 100, 1, 1, 50)], ValueError)):
        with pytest.raises(err):
            two_group.run_chains_host(obs, tot, model, bad, out)
    m2 = {k: v.copy() for k, v in obs.items()}
    m2["case"][5, 0] = tot["case"][5, 0] + 1
    with pytest.raises(_lib.HygError):
        two_group.run_chains_host(m2, tot, model, chains[:1], out)


def test_long_chain_properties_and_determinism():
    """A full-length segment chain (110k sites, the reference's segment +
    buffers): size-independent properties, and bit-identical reruns."""
    from hygeia_amd import synthetic as syn
    from hygeia_amd import two_group

    T = 110000
    d = syn.simulate(T, 4, 4, K=6, seed=41, coverage=100.0)
    mu, sg = syn.regime_params(6)
    theta = two_group.uniform_theta(6)
    model = _model(mu, sg, theta, 50, 25, int(max(d["tot_control"].max(), d["tot_case"].max())), T)
    obs = {"control": d["meth_control"], "case": d["meth_case"]}
    tot = {"control": d["tot_control"], "case": d["tot_case"]}
    res, fw, ex = two_group.run(obs, tot, model, 0, 1)
    res2, fw2, ex2 = two_group.run(obs, tot, model, 0, 1)
    ctl = res.particle["control_state"].astype(np.int64)
    case = res.particle["case_state"].astype(np.int64)
    m = res.particle["merged_state"]
    np.testing.assert_array_equal(ctl, res2.particle["control_state"])
    np.testing.assert_array_equal(ex["regime_probs"], ex2["regime_probs"])
    # durations advance by one or restart at a change point (int16 wrap aside)
    dd = (ctl[1:, :, 0] - ctl[:-1, :, 0]) % 65536
    assert np.all((dd == 1) | (ctl[1:, :, 0] == 1))
    # regimes only change at change points
    assert np.all((ctl[1:, :, 1] == ctl[:-1, :, 1]) | (ctl[1:, :, 0] == 1))
    # merged sites carry identical control and case states
    mm = m == 1
    assert np.all(ctl[mm] == case[mm])
    # probabilities are means over B: regime probs of each group sum to 1
    rp = ex["regime_probs"]
    np.testing.assert_allclose(rp[:, :6].sum(1), 1.0, atol=1e-6)
    np.testing.assert_allclose(rp[:, 6:].sum(1), 1.0, atol=1e-6)
    np.testing.assert_array_equal(ex["split_probs"], (m == 0).mean(1).astype(np.float32))
    # recovery of the simulated control regimes
    acc = (rp[:, :6].argmax(1) == d["regime_control"]).mean()
    assert acc > 0.95, acc
    assert np.isfinite(ex["log_z"])


@pytest.mark.parametrize("name", ["tg_chain_k6", "tg_chain_k4"])
def test_golden_fixture(name):
    """The committed golden fixtures (tests/golden/make_golden.py), through the C ABI."""
    import os

    from hygeia_amd import two_group

    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name + ".npz"))
    K, M, B = int(g["K"]), int(g["M"]), int(g["B"])
    theta = two_group.uniform_theta(K, 0.8)
    T = g["tot_control"].shape[0]
    maxr = int(max(g["tot_control"].max(), g["tot_case"].max()))
    model = _model(g["mu"], g["sigma"], theta, M, B, maxr, T + 5)
    res, fw, ex = two_group.run({"control": g["meth_control"], "case": g["meth_case"]},
                                {"control": g["tot_control"], "case": g["tot_case"]}, model, int(g["seed"]),
                                int(g["chain_id"]))
    pr = res.particle
    np.testing.assert_array_equal(pr["merged_state"], g["merged"])
    np.testing.assert_array_equal(pr["control_state"], g["control"])
    np.testing.assert_array_equal(pr["case_state"], g["case"])
    np.testing.assert_array_equal(ex["split_probs"], g["split_probs"])
    np.testing.assert_array_equal(ex["regime_probs"], g["regime_probs"])
    assert ex["log_z"] == float(g["log_z"])
    np.testing.assert_array_equal(fw, g["final_log_weights"])


def test_cli_infer_end_to_end(tmp_path, oracle):
    """`hygeia infer` (hygeia_amd/cli.py) on a 3-batch chromosome: the saved,
    trimmed trajectories and the untrimmed probabilities equal the oracle's run
    of the same segment with the same (seed, chain id)."""
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_cli import _write_inputs

    from hygeia_amd import cli, two_group

    data = _write_inputs(str(tmp_path), "7", 2300)
    for batch in (0, 1, 2):
        rc = cli.main(["infer", "--chrom", "7", "--batch", str(batch), "--segment_size", "1000",
                       "--buffer_size", "50", "--num_resampled_particles", "20", "--num_samples_backward", "8",
                       "--seed", "3", "--data_dir", str(tmp_path / "data"),
                       "--single_group_dir", str(tmp_path / "sg"), "--results_dir", str(tmp_path / "res")])
        assert rc == 0
        (lo, hi), (r0, r1) = cli.segment_index(2300, batch, 1000, 50)
        mu = np.array([0.95, 0.05, 0.80, 0.20, 0.50, 0.50], np.float32)
        sg = np.array([0.05, 0.05, 0.1, 0.1, 0.1, 0.2886751], np.float32)
        p = oracle.make_params(K=6, M=20, B=8, mu=mu, sigma=sg, theta=two_group.uniform_theta(6, 0.8))
        E = oracle.emission(p, data["meth_control"][lo:hi], data["tot_control"][lo:hi], data["meth_case"][lo:hi],
                            data["tot_case"][lo:hi])
        ref = oracle.chain(p, E, 3, cli.chain_id("7", batch))
        out = tmp_path / "res" / f"chrom_7_{batch}"
        N = 20 * 48
        ld = lambda n: np.load(out / f"{n}_{N}_3.npz")["arr_0"]  # noqa: E731
        np.testing.assert_array_equal(ld("optimal_backward_particles_merged_state"), ref["merged"][r0:r1])
        np.testing.assert_array_equal(ld("optimal_backward_particles_control_state"), ref["control"][r0:r1])
        np.testing.assert_array_equal(ld("optimal_backward_particles_case_state"), ref["case"][r0:r1])
        np.testing.assert_array_equal(ld("optimal_split_probs"), ref["split_probs"])
        np.testing.assert_array_equal(ld("optimal_regime_probs"), ref["regime_probs"])
        txt = (out / "log_normalizing_constants_optimal_3.txt").read_text()
        assert txt.startswith("{960: ")
        assert float(txt.split(":")[1].strip(" }\n")) == pytest.approx(ref["log_z"], rel=1e-15)


def test_infer_many_equals_single_task_runs(tmp_path):
    """`hygeia infer_many` (every (batch, seed) task of a chromosome in one
    launch) writes the same per-(chrom, batch) directories as the single-task
    `hygeia infer` runs modules/two_group/4_infer.nf fans out: identical flags
    files, trimmed trajectories, untrimmed probabilities, log Z and inputs
    (gzip headers aside: compared decompressed)."""
    import gzip
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_cli import _write_inputs

    from hygeia_amd import cli

    _write_inputs(str(tmp_path), "5", 2600)
    common = ["--chrom", "5", "--segment_size", "1000", "--buffer_size", "60", "--num_resampled_particles", "12",
              "--num_resampled_particles", "20", "--num_samples_backward", "7", "--data_dir", str(tmp_path / "data"),
              "--single_group_dir", str(tmp_path / "sg")]
    for b in (0, 1, 2):  # get_chrom_segments: 1 + 2600 // 1000 segments
        for sd in (0, 4):
            assert cli.main(["infer", "--batch", str(b), "--seed", str(sd), "--results_dir", str(tmp_path / "one")]
                            + common) == 0
    assert cli.main(["infer_many", "--batches", "all", "--seeds", "0,4", "--results_dir", str(tmp_path / "many")]
                    + common) == 0
    one, many = tmp_path / "one", tmp_path / "many"
    assert sorted(p.name for p in one.iterdir()) == sorted(p.name for p in many.iterdir()) == [
        "chrom_5_0", "chrom_5_1", "chrom_5_2"]
    for d in one.iterdir():
        names = sorted(p.name for p in d.iterdir())
        assert names == sorted(p.name for p in (many / d.name).iterdir())
        for nm in names:
            a, b = d / nm, many / d.name / nm
            if nm.startswith("optimal_time_"):
                continue  # wall times
            if nm.endswith(".npz"):
                np.testing.assert_array_equal(np.load(a)["arr_0"], np.load(b)["arr_0"])
            elif nm.endswith(".gz"):
                assert gzip.open(a).read() == gzip.open(b).read(), nm
            else:  # the flags files name their own --results_dir
                assert a.read_text().replace(str(one), "R") == b.read_text().replace(str(many), "R"), nm


def test_tail_overlap_equals_one_launch(oracle):
    """The tail overlap of hyg_tg_run_chains (the C5 shape, one forward chain
    per CU: more chains than CUs with a partial last round run as the full
    rounds' forward, then the rest's forward beside the full rounds' backward on
    a second stream) gives the outputs of the unsplit launch, and chains on
    either side of the split equal their own oracle runs."""
    from hygeia_amd import _lib, two_group

    L = _lib.load()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    K, M, B, S = 12, 50, 25, 3
    mu, sg, theta, d, p = _setup(oracle, K, M, B, 1600, S, 100.0, 35)
    obs = {"control": d["meth_control"], "case": d["meth_case"]}
    tot = {"control": d["tot_control"], "case": d["tot_case"]}
    n_chains = cus + 37
    rng = np.random.default_rng(5)
    chains, out = [], 0
    for i in range(n_chains):
        n = int(rng.integers(20, 90)) if i < cus else int(rng.integers(1, 120))
        s0 = int(rng.integers(0, 1600 - n))
        chains.append((s0, n, i % 3, 7000 + i, out))
        out += n
    model = _model(mu, sg, theta, M, B, int(max(d["tot_control"].max(), d["tot_case"].max())), 200)
    assert L.hyg_tg_chains_per_cu(model.handle, n_chains) == 1  # the split applies
    runs = []
    for on in (1, 0):
        _lib.check(L.hyg_tg_set_tail_overlap(on))
        try:
            runs.append(two_group.run_chains_host(obs, tot, model, chains, out, final_weights=True))
        finally:
            L.hyg_tg_set_tail_overlap(1)
    a, b = runs
    assert (a["status"] == 0).all()
    for k in ("merged", "control", "case", "split_probs", "regime_probs", "log_z", "final_w", "status"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    E_ref = oracle.emission(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
    for i in (0, cus - 1, cus, n_chains - 1):
        s0, n, seed, cid, o0 = chains[i]
        ref = oracle.chain(p, E_ref[s0:s0 + n], seed, cid)
        for k in ("merged", "control", "case", "split_probs", "regime_probs"):
            np.testing.assert_array_equal(a[k][o0:o0 + n], ref[k], err_msg=f"chain {i} {k}")
        assert a["log_z"][i] == ref["log_z"]
        np.testing.assert_array_equal(a["final_w"][i], ref["final_log_weights"])



@pytest.mark.parametrize("K,S", [(6, 4), (12, 50), (4, 3)])
def test_emission_table_equals_per_term_path(oracle, K, S):
    """The emission from the per-(n, y) term table (built at model creation
    when it stays L2-sized) has the bits of the per-term emission (a model
    whose read range makes the table too large) and of the oracle, at the
    pipeline shape, the stress shape (K = 12, 50 samples) and a generic K; zero
    coverage and invalid rows included."""
    from hygeia_amd import two_group

    T = 6000
    mu, sg, theta, d, p = _setup(oracle, K, 50, 25, T, S, 100.0, 40 + K)
    for k in ("meth_control", "tot_control", "meth_case", "tot_case"):
        d[k][100:130] = 0
    d["meth_case"][200, 0] = d["tot_case"][200, 0] + 1  # methylated > total: a NaN row on every path
    maxr = int(max(d["tot_control"].max(), d["tot_case"].max()))
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(np.ascontiguousarray(d[k]).view(np.int16)).to(dev) for k in
         ("meth_control", "tot_control", "meth_case", "tot_case")}
    out = []
    for reads in (maxr, 3000):  # (3000: a table of 144-864 MB, over the 16 MB bound: the per-term kernel)
        m = _model(mu, sg, theta, 50, 25, reads, 10)
        dc = two_group.DeviceChains(m, [(0, 5, 0, 0, 0)], 5, device=dev)
        out.append(dc.emission(t["meth_control"], t["tot_control"], t["meth_case"], t["tot_case"]).cpu().numpy())
    np.testing.assert_array_equal(out[0], out[1])  # (NaN rows compare equal)
    assert np.isnan(out[0][200, K:]).all() and not np.isnan(out[0][200, :K]).any()
    ok = np.ones(T, bool)
    ok[200] = False  # (the oracle refuses invalid counts)
    E_ref = oracle.emission(p, d["meth_control"][ok], d["tot_control"][ok], d["meth_case"][ok], d["tot_case"][ok])
    np.testing.assert_array_equal(out[0][ok], E_ref)
    assert np.all(out[0][100:130] == 0.0)
