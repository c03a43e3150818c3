"""GPU parity of the aggregation / DMP-calling stage (hyg_dmp_* through the C
ABI) against oracle/dmp_oracle.py and the reference's golden vectors.

Bar: exact. FDR outputs (k, Q_k, threshold) bit-identical to numpy's
FDR_procedure; weighted-FDR selections identical to the stable-argsort
restatement (and, on the golden cases, to the reference's own selections);
per-site counts identical to numpy."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
from oracle import dmp_oracle as od  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "dmp_fdr.npz")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    from hygeia_amd import _lib

    if _lib.load().hyg_device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X (gpurun)")


def _dev(a, dtype):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dtype).to("cuda:0")


@pytest.mark.parametrize("i", range(8))
def test_fdr_and_weighted_vs_reference_golden(i):
    from hygeia_amd import dmp

    z = np.load(GOLD)
    c, P, thr = z[f"case_{i}_counts"], int(z[f"case_{i}_P"]), float(z[f"case_{i}_thr"])
    counts = _dev(c.reshape(-1, 1), torch.int32)
    k, q, th = dmp.fdr(counts, 0, P, thr)
    g = z[f"case_{i}_fdr"]
    assert (k, q, th) == (int(g[0]), g[1], g[2])
    wfn = _dev(z[f"case_{i}_wfn"], torch.float64)
    idx, ns = dmp.weighted_fdr(counts, 0, P, thr, torch.ones_like(wfn), wfn)
    np.testing.assert_array_equal(np.sort(idx), z[f"case_{i}_widx"])
    assert ns == z[f"case_{i}_wsum"]
    t = od.statistics_from_counts(c, P)
    oidx, _ = od.weighted_fdr_procedure(t, thr, np.ones(len(t)), z[f"case_{i}_wfn"])
    np.testing.assert_array_equal(idx, oidx)  # same order too (both stable)


@pytest.mark.parametrize("n,P,thr,seed", [(1, 50, 0.05, 0), (7, 3, 0.4, 1), (100000, 50, 0.05, 2),
                                          (300000, 2400, 0.02, 3), (50000, 65535, 0.1, 4), (20000, 50, 1e-9, 5)])
def test_fdr_random_vs_oracle(n, P, thr, seed):
    """Counting-sort FDR + host cumsum replay vs numpy on random counts, incl.
    a single site, P = 3, large P (global-atomic histogram) and thr < min t."""
    from hygeia_amd import dmp

    rng = np.random.default_rng(seed)
    c = np.where(rng.random(n) < 0.2, rng.integers(0, P + 1, n), rng.binomial(P, 0.02, n)).astype(np.int32)
    counts = _dev(np.stack([rng.integers(0, 5, n), c], 1), torch.int32)  # column 1, stride 2
    assert dmp.fdr(counts, 1, P, thr) == od.fdr_procedure(od.statistics_from_counts(c, P), thr)


def test_fdr_rejects_out_of_range_counts():
    from hygeia_amd import _lib, dmp

    counts = _dev(np.array([[0], [51]]), torch.int32)
    with pytest.raises(_lib.HygError):
        dmp.fdr(counts, 0, 50, 0.05)


@pytest.mark.parametrize("n,P,seed", [(1000, 50, 0), (200001, 50, 1), (70000, 7, 2)])
def test_weighted_fdr_heavy_ties_vs_oracle(n, P, seed):
    """Radix-sort stability: coarse weights give large tie groups; the ranked
    selection (order included) equals numpy's stable argsort."""
    from hygeia_amd import dmp

    rng = np.random.default_rng(seed)
    c = rng.binomial(P, rng.choice([0.02, 0.9], n, p=[0.85, 0.15])).astype(np.int32)
    wfn = 1.0 / rng.choice([1.0, 2.0, 3.0, 1e5], n)
    wfp = rng.choice([1.0, 0.5], n)
    counts = _dev(c.reshape(-1, 1), torch.int32)
    idx, ns = dmp.weighted_fdr(counts, 0, P, 0.05, _dev(wfp, torch.float64), _dev(wfn, torch.float64))
    oidx, ons = od.weighted_fdr_procedure(od.statistics_from_counts(c, P), 0.05, wfp, wfn)
    np.testing.assert_array_equal(idx, oidx)
    assert ns == ons


def test_site_counts_segments_and_seeds_vs_oracle():
    """Several segments, 3 seed blocks each, scattered in one trajectory buffer."""
    from hygeia_amd import dmp

    rng = np.random.default_rng(7)
    B, K, S = 9, 6, 3
    seg = [(0, 40), (40, 25), (65, 1), (66, 30)]  # (site_begin, rows)
    rows = sum(r for _, r in seg) * S + 17  # unused rows too
    merged = rng.integers(0, 2, (rows, B)).astype(np.int16)
    control = np.stack([rng.integers(1, 9, (rows, B)), rng.integers(0, K, (rows, B))], -1).astype(np.int16)
    case = np.stack([rng.integers(1, 9, (rows, B)), rng.integers(0, K, (rows, B))], -1).astype(np.int16)
    perm = rng.permutation(len(seg) * S)
    starts, o = {}, 5
    for q in perm:  # blocks placed in a shuffled order
        g, s = divmod(int(q), S)
        starts[(g, s)] = o
        o += seg[g][1]
    block_rows = [[starts[(g, s)] for s in range(S)] for g in range(len(seg))]
    n_sites = 100
    counts, pairs = dmp.site_counts(_dev(merged, torch.int16), _dev(control, torch.int16), _dev(case, torch.int16),
                                    B, K, seg, block_rows, n_sites, pairs=True)
    exp = np.zeros((n_sites, 2 + 2 * K), np.int32)
    expp = np.zeros((n_sites, K, K), np.int32)
    for g, (s0, nr) in enumerate(seg):
        sl = lambda a, s: a[block_rows[g][s]:block_rows[g][s] + nr]  # noqa: E731
        m = np.concatenate([sl(merged, s) for s in range(S)], 1)
        c = np.concatenate([sl(control, s)[..., 1] for s in range(S)], 1)
        k = np.concatenate([sl(case, s)[..., 1] for s in range(S)], 1)
        o_, p_ = od.site_counts(m, c, k, K)
        exp[s0:s0 + nr], expp[s0:s0 + nr] = o_, p_
    np.testing.assert_array_equal(counts.cpu().numpy(), exp)
    np.testing.assert_array_equal(pairs.cpu().numpy(), expp)


def test_get_dmps_cli_end_to_end(tmp_path):
    """`hygeia get_dmps` on an aggregated directory: every output CSV equals the
    one get_dmps.py's code path writes with the oracle's FDR functions."""
    import pandas as pd

    from hygeia_amd import cli

    rng = np.random.default_rng(11)
    T, P, K, chrom = 3000, 50, 6, "5"
    pos = np.cumsum(1 + rng.geometric(0.02, T)).astype(np.int64)
    base = rng.integers(0, K, T)
    ctrl = np.repeat(base[:, None], P, 1)
    case = ctrl.copy()
    diff = rng.random(T) < 0.1
    flip = rng.random((T, P)) < np.where(diff, 0.95, 0.01)[:, None]
    case[flip] = (case[flip] + 1 + rng.integers(0, K - 1, int(flip.sum()))) % K
    agg = tmp_path / "agg"
    agg.mkdir()
    for name, a in (("control_regimes", ctrl), ("case_regimes", case)):
        pd.DataFrame(a.astype(np.int8)).set_index(pd.Series(pos.astype(np.int32), name="pos")).to_csv(
            agg / f"{name}_chrom_{chrom}.csv.gz", sep="\t", compression="gzip")
    sp = pd.Series((case == 99).mean(1), index=pd.Index(pos.astype(np.int32), name="pos"))
    sp.to_csv(agg / f"split_probs_{chrom}.csv.gz", sep="\t", compression="gzip")
    out = tmp_path / "dmp"
    assert cli.main(["get_dmps", "--results_dir", str(agg), "--output_dir", str(out), "--chrom", chrom,
                     "--fdr_thresholds", "0.01", "--fdr_thresholds", "0.05", "--test_regime_combinations"]) == 0
    # expected, from the oracle with get_dmps.py's frame construction
    t = 1. - np.sum(ctrl != case, axis=1) / P
    fnw = od.false_negative_weights(pos)
    for thr in (0.01, 0.05):
        k, q, th = od.fdr_procedure(t, thr)
        ind = t < th
        got = pd.read_csv(out / f"dmp_{thr}.csv")
        np.testing.assert_array_equal(got["position"].to_numpy(), pos[ind])
        np.testing.assert_allclose(got["null_stats"].to_numpy(), np.round(t[ind], 4), atol=1e-12)
        freq = np.stack([np.bincount(r, minlength=K) / P for r in ctrl[ind]]) if ind.any() else np.zeros((0, K))
        np.testing.assert_allclose(got[[f"Control_METEOR_{i + 1}" for i in range(K)]].to_numpy(),
                                   np.round(freq, 4), atol=1e-12)
        widx, _ = od.weighted_fdr_procedure(t, thr, np.ones(T), fnw)
        gw = pd.read_csv(out / f"weighted_dmp_{thr}.csv")
        np.testing.assert_array_equal(gw["position"].to_numpy(), pos[np.sort(widx)])
        for i in range(K):
            for j in range(K):
                if i != j:
                    tij = 1 - np.sum((ctrl == i) * (case == j), axis=1) / P
                    _, _, thij = od.fdr_procedure(tij, thr)
                    g = pd.read_csv(out / f"dmp_{i}_{j}_{thr}.csv")
                    np.testing.assert_array_equal(g["position"].to_numpy(), pos[tij < thij])


def test_aggregate_cli_end_to_end(tmp_path):
    """`hygeia infer` for 2 batches x 2 seeds, then `hygeia aggregate`: the
    per-chromosome files equal aggregate_results.py's construction from the
    saved trajectories (split probabilities = mean over particles of merged == 0)."""
    import sys

    import pandas as pd

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_cli import _write_inputs

    from hygeia_amd import cli

    _write_inputs(str(tmp_path), "9", 1700)
    for batch in (0, 1):
        for seed in (0, 1):
            assert cli.main(["infer", "--chrom", "9", "--batch", str(batch), "--segment_size", "1000",
                             "--buffer_size", "50", "--num_resampled_particles", "10", "--num_samples_backward", "6",
                             "--seed", str(seed), "--data_dir", str(tmp_path / "data"),
                             "--single_group_dir", str(tmp_path / "sg"), "--results_dir", str(tmp_path / "res")]) == 0
    N = 10 * 48
    out = tmp_path / "agg"
    assert cli.main(["aggregate", "--results_dir", str(tmp_path / "res"), "--chrom", "9", "--seeds", "2",
                     "--num_particles", str(N), "--output_dir", str(out), "--num_batches", "5",
                     "--compute_freqs"]) == 0
    merged, ctrl = [], []
    for batch in (0, 1):
        d = tmp_path / "res" / f"chrom_9_{batch}"
        merged.append(np.concatenate([np.load(d / f"optimal_backward_particles_merged_state_{N}_{s}.npz")["arr_0"]
                                      for s in (0, 1)], -1))
        ctrl.append(np.concatenate([np.load(d / f"optimal_backward_particles_control_state_{N}_{s}.npz")["arr_0"]
                                    for s in (0, 1)], 1))
    merged, ctrl = np.concatenate(merged), np.concatenate(ctrl)
    sp = pd.read_csv(out / "split_probs_9.csv.gz", sep="\t", float_precision="round_trip")
    np.testing.assert_array_equal(sp["0"].to_numpy(), np.mean(merged == 0, axis=1))
    cr = pd.read_csv(out / "control_regimes_chrom_9.csv.gz", sep="\t").set_index("pos").to_numpy()
    np.testing.assert_array_equal(cr, ctrl[:, :, 1])
    ms = pd.read_csv(out / "merge_states_chrom_9.csv.gz", sep="\t").set_index("pos").to_numpy()
    np.testing.assert_array_equal(ms, merged)
    # --compute_freqs (aggregate_results.py:208-215): the reference's own pandas
    # expression on the written regime frames gives the same files
    for g in ("case", "control"):
        reg = pd.read_csv(out / f"{g}_regimes_chrom_9.csv.gz", sep="\t").set_index("pos").astype(np.int8)
        want = reg.apply(lambda x: x.value_counts(normalize=True), 1)
        assert (out / f"{g}_regimes_freq_9.csv").read_text() == want.to_csv(sep="\t")


def test_weighted_fdr_tie_at_cutoff_vs_reference_golden():
    """The reference's selection at a cutoff inside a tie group depends on
    np.argsort's unstable order; the device ranking is stable (lowest site
    indices of the group). Same s, same Nsums[s-1], same sites outside the
    group, same number from inside it (tests/test_dmp_oracle.py)."""
    import sys

    from hygeia_amd import dmp

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_dmp_oracle import tie_boundary_check

    z = np.load(GOLD)
    c, P = z["tie_counts"], int(z["tie_P"])
    wfn = _dev(z["tie_wfn"], torch.float64)
    idx, ns = dmp.weighted_fdr(_dev(c.reshape(-1, 1), torch.int32), 0, P, float(z["tie_thr"]),
                               torch.ones_like(wfn), wfn)
    tie_boundary_check(np.asarray(idx), ns, z)
    t = od.statistics_from_counts(c, P)
    oidx, _ = od.weighted_fdr_procedure(t, float(z["tie_thr"]), np.ones(len(t)), z["tie_wfn"])
    np.testing.assert_array_equal(idx, oidx)
