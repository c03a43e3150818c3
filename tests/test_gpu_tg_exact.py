"""GPU: the tiny chains of tests/test_tg_exact.py through the HIP path.

Each configuration runs many seeds as chains of ONE batched launch
(hyg_tg_run_chains through two_group.DeviceChains) and is compared
(1) bit for bit with the CPU oracle, chain by chain, and
(2) with the exact enumeration of the model (tests/tg_exact_model.py): in the
    keep-all regime the GPU's log Z equals the exact log marginal likelihood
    given the phantom regime to 1e-12 and the GPU's backward draws pass the
    chi-square tests against the exact smoother; with M = 2-3 (optimal
    finite-state resampling active) the seed average of Z_hat / Z stays 1
    within its standard error. Cases at u = 2, the pipeline's u = 3, and u = 4,
    and (round 4) at the pipeline's K = 6 and K = 4 with 2 + 2 samples, where
    the case transition's uniform normalisers are 1/5 and 1/4, and (round 5) at
    the stress shape's K = 12 (1/11 and 1/10).
"""
import math
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_tg_exact import (BACKWARD_CASES, KEEP_ALL_CASES, KEEP_ALL_M, RESAMPLING_CASES, _problem,  # noqa: E402
                           check_draws_follow_exact_smoother)
from tg_exact_model import phantom_regime  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    from hygeia_amd import _lib

    if _lib.load().hyg_device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X (gpurun)")


def _run_seeds(p, E, K, M, B, seeds, cid):
    """All seeds as chains of one launch over the same sites."""
    from hygeia_amd import two_group

    T = E.shape[0]
    dev = torch.device("cuda", 0)
    mu = [p.mu[i] for i in range(K)]
    sg = [p.sigma[i] for i in range(K)]
    theta = [p.theta[i] for i in range(p.theta_len)]
    model = two_group.CaseControlModel(mu, sg, theta, minimum_duration=p.minimum_duration,
                                       num_resampled_ancestors=M, num_samples_backward=B, max_total_reads=64,
                                       max_duration=T + 5)
    chains = [(0, T, s, cid, i * T) for i, s in enumerate(seeds)]
    dc = two_group.DeviceChains(model, chains, T * len(seeds), device=dev, final_weights=True)
    Ed = torch.from_numpy(np.ascontiguousarray(E)).to(dev)
    dc.run(Ed)
    torch.cuda.synchronize()
    assert (dc.status.cpu().numpy() == 0).all()
    return dc


def _check_chain_bits(oracle, p, E, dc, i, seed, cid, T):
    ref = oracle.chain(p, E, seed, cid)
    o = i * T
    np.testing.assert_array_equal(dc.merged[o:o + T].cpu().numpy(), ref["merged"])
    np.testing.assert_array_equal(dc.control[o:o + T].cpu().numpy(), ref["control"])
    np.testing.assert_array_equal(dc.case[o:o + T].cpu().numpy(), ref["case"])
    np.testing.assert_array_equal(dc.split_probs[o:o + T].cpu().numpy(), ref["split_probs"])
    np.testing.assert_array_equal(dc.regime_probs[o:o + T].cpu().numpy(), ref["regime_probs"])
    assert dc.log_z[i].item() == ref["log_z"]
    np.testing.assert_array_equal(dc.final_w[i].cpu().numpy(), ref["final_log_weights"])


@pytest.mark.parametrize("K,T,dseed,u", KEEP_ALL_CASES)
def test_keep_all_gpu_vs_oracle_and_exact(oracle, K, T, dseed, u):
    B = 8
    p, ex, E, E_ex = _problem(oracle, K, T, dseed, M=KEEP_ALL_M, B=B, u=u)
    seeds = list(range(24))
    cid = 40
    dc = _run_seeds(p, E, K, KEEP_ALL_M, B, seeds, cid)
    lz = dc.log_z.cpu().numpy()
    exact = {}
    for i, s in enumerate(seeds):
        _check_chain_bits(oracle, p, E, dc, i, s, cid, T)
        r_ph = phantom_regime(oracle, s, cid, K)
        if r_ph not in exact:
            exact[r_ph] = ex.forward_backward(E_ex, r_ph)[0]
        assert abs(lz[i] - exact[r_ph]) < 1e-12 * max(1.0, abs(exact[r_ph]))
    assert len(exact) >= 2


@pytest.mark.parametrize("K,T,M,dseed,u", RESAMPLING_CASES)
def test_resampling_gpu_vs_oracle_and_unbiased_z(oracle, K, T, M, dseed, u):
    p, ex, E, E_ex = _problem(oracle, K, T, dseed, M=M, B=2, u=u)
    seeds = list(range(8192))
    cid = 3
    dc = _run_seeds(p, E, K, M, 2, seeds, cid)
    for i in range(0, len(seeds), 511):  # bit-exact spot checks across the batch
        _check_chain_bits(oracle, p, E, dc, i, seeds[i], cid, T)
    lz = dc.log_z.cpu().numpy()
    zex = {}
    ratios = []
    for i, s in enumerate(seeds):
        r_ph = phantom_regime(oracle, s, cid, K)
        if r_ph not in zex:
            zex[r_ph] = ex.log_z(E_ex, r_ph)
        ratios.append(math.exp(lz[i] - zex[r_ph]))
    r = np.array(ratios)
    se = r.std() / math.sqrt(len(r))
    assert abs(r.mean() - 1.0) < 4 * se + 1e-3, (r.mean(), se)


@pytest.mark.parametrize("K,T,dseed,u", BACKWARD_CASES)
def test_backward_gpu_draws_follow_exact_smoother(oracle, K, T, dseed, u):
    M, B, nseeds, cid = KEEP_ALL_M, 60, 300, 7
    p, ex, E, E_ex = _problem(oracle, K, T, dseed, M=M, B=B, cov=2, u=u)
    seeds = list(range(nseeds))
    dc = _run_seeds(p, E, K, M, B, seeds, cid)
    for i in range(0, nseeds, 37):
        _check_chain_bits(oracle, p, E, dc, i, seeds[i], cid, T)
    mg, ct, cs = dc.merged.cpu().numpy(), dc.control.cpu().numpy(), dc.case.cpu().numpy()

    def paths_of(i, seed):
        return mg[i * T:(i + 1) * T], ct[i * T:(i + 1) * T], cs[i * T:(i + 1) * T]

    check_draws_follow_exact_smoother(oracle, ex, E_ex, K, T, u, B, seeds, cid, paths_of)


# ----------------------------------------------------- the pipeline's K (4, 6)
from test_tg_exact import (PIPELINE_BACKWARD, PIPELINE_KEEP_ALL, PIPELINE_RESAMPLING,  # noqa: E402
                           backward_seeds, draws_branch_counts)


@pytest.mark.parametrize("K,T,dseed,u,S,M", [c[:6] for c in PIPELINE_KEEP_ALL if c[6]])
def test_pipeline_k_keep_all_gpu_vs_oracle_and_exact(oracle, K, T, dseed, u, S, M):
    """K = 6 / K = 4 / K = 12, u = 3, 2 + 2 samples, every finite particle kept:
    the GPU's log Z is the exact log marginal likelihood (1e-12), bit for bit
    the oracle."""
    B = 8
    p, ex, E, E_ex = _problem(oracle, K, T, dseed, M=M, B=B, u=u, S=S)
    seeds = list(range(24))
    cid = 40
    dc = _run_seeds(p, E, K, M, B, seeds, cid)
    lz = dc.log_z.cpu().numpy()
    exact = {}
    for i, s in enumerate(seeds):
        _check_chain_bits(oracle, p, E, dc, i, s, cid, T)
        r_ph = phantom_regime(oracle, s, cid, K)
        if r_ph not in exact:
            exact[r_ph] = ex.forward_backward(E_ex, r_ph)[0]
        assert abs(lz[i] - exact[r_ph]) < 1e-12 * max(1.0, abs(exact[r_ph]))
    assert len(exact) >= 2


@pytest.mark.parametrize("K,T,M,dseed,u,S", PIPELINE_RESAMPLING)
def test_pipeline_k_resampling_gpu_unbiased_z(oracle, K, T, M, dseed, u, S):
    p, ex, E, E_ex = _problem(oracle, K, T, dseed, M=M, B=2, u=u, S=S)
    seeds = list(range(8192))
    cid = 3
    dc = _run_seeds(p, E, K, M, 2, seeds, cid)
    for i in range(0, len(seeds), 511):
        _check_chain_bits(oracle, p, E, dc, i, seeds[i], cid, T)
    lz = dc.log_z.cpu().numpy()
    zex = {}
    ratios = []
    for i, s in enumerate(seeds):
        r_ph = phantom_regime(oracle, s, cid, K)
        if r_ph not in zex:
            zex[r_ph] = ex.log_z(E_ex, r_ph)
        ratios.append(math.exp(lz[i] - zex[r_ph]))
    r = np.array(ratios)
    se = r.std() / math.sqrt(len(r))
    assert abs(r.mean() - 1.0) < 4 * se + 1e-3, (r.mean(), se)
    assert r.std() > 1e-3


@pytest.mark.parametrize("K,T,dseed,u,S,M", [c[:6] for c in PIPELINE_BACKWARD if c[6]])
def test_pipeline_k_backward_gpu_draws_follow_exact_smoother(oracle, K, T, dseed, u, S, M):
    B, nseeds, cid = 60, backward_seeds(K), 7
    p, ex, E, E_ex = _problem(oracle, K, T, dseed, M=M, B=B, cov=2, u=u, S=S)
    seeds = list(range(nseeds))
    dc = _run_seeds(p, E, K, M, B, seeds, cid)
    for i in range(0, nseeds, 37):
        _check_chain_bits(oracle, p, E, dc, i, seeds[i], cid, T)
    mg, ct, cs = dc.merged.cpu().numpy(), dc.control.cpu().numpy(), dc.case.cpu().numpy()

    def paths_of(i, seed):
        return mg[i * T:(i + 1) * T], ct[i * T:(i + 1) * T], cs[i * T:(i + 1) * T]

    check_draws_follow_exact_smoother(oracle, ex, E_ex, K, T, u, B, seeds, cid, paths_of)
    paths = []
    for i in range(nseeds):
        m, c, k = (a.astype(int) for a in paths_of(i, seeds[i]))
        paths += [[(m[t, b], c[t, b, 0], c[t, b, 1], k[t, b, 0], k[t, b, 1]) for t in range(T)] for b in range(B)]
    n = draws_branch_counts(ex, paths)
    assert n[(2, True)] > 0 and n[(4, True)] > 0, dict(n)


from test_tg_exact import PIPELINE_M50  # noqa: E402


@pytest.mark.parametrize("K,T,M,dseed,u,S,cov", PIPELINE_M50)
def test_pipeline_m50_resampling_gpu_unbiased_z(oracle, K, T, M, dseed, u, S, cov):
    """The pipeline's M = 50 through the GPU's top-set resampling path (8 192
    seeds in one launch): bit for bit the oracle (spot checks) and Z_hat / Z
    unbiased against the exact enumeration."""
    p, ex, E, E_ex = _problem(oracle, K, T, dseed, M=M, B=2, u=u, S=S, cov=cov)
    seeds = list(range(8192))
    cid = 3
    dc = _run_seeds(p, E, K, M, 2, seeds, cid)
    for i in range(0, len(seeds), 511):
        _check_chain_bits(oracle, p, E, dc, i, seeds[i], cid, T)
    lz = dc.log_z.cpu().numpy()
    zex = {r: ex.log_z(E_ex, r) for r in range(K)}
    r = np.array([math.exp(lz[i] - zex[phantom_regime(oracle, s, cid, K)]) for i, s in enumerate(seeds)])
    se = r.std() / math.sqrt(len(r))
    assert abs(r.mean() - 1.0) < 4 * se + 1e-6, (r.mean(), se)
    assert r.std() > 5e-4
