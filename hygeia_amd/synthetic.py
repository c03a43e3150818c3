"""Synthetic two-group methylation data, vectorised numpy.

Follows the generative model of src/two_group/simulate_two_groups.py
(regimes_config 8 = the pipeline defaults): semi-Markov regime segments whose
lengths are the minimum duration u plus NegBin(kappa, omega) draws
(case_control_regime_model.py:111-168 hazard), uniform off-diagonal regime
transitions, a case group that copies the control segmentation except inside
"split" stretches where it draws its own segments, Beta(alpha_r, beta_r)
methylation levels and Poisson(lambda) coverage, i.e. Beta-Binomial counts
(case_control_regime_model.py:197-231).
"""
from __future__ import annotations

import math

import numpy as np

# hg38 autosome lengths chr1..chr22
HG38 = np.array([
    248956422, 242193529, 198295559, 190214555, 181538259, 170805979, 159345973, 145138636,
    138394717, 133797422, 135086622, 133275309, 114364328, 107043718, 101991189, 90338345,
    83257441, 80373285, 58617616, 64444167, 46709983, 50818468], dtype=np.int64)

DEFAULT_MU = np.array([0.95, 0.05, 0.80, 0.20, 0.50, 0.50])
DEFAULT_SIGMA = np.array([0.05, 0.05, 0.1, 0.1, 0.1, 0.2886751])
DATA_SEED = 20251024


def regime_params(K: int):
    """mu/sigma for K regimes: the pipeline's 6, duplicated with sigma*0.8 for K=12 (8d)."""
    if K == 6:
        return DEFAULT_MU.copy(), DEFAULT_SIGMA.copy()
    if K == 12:
        return np.concatenate([DEFAULT_MU, DEFAULT_MU]), np.concatenate([DEFAULT_SIGMA, DEFAULT_SIGMA * 0.8])
    mu = (np.arange(K) + 0.5) / K
    return mu, 0.05 + 0.2 * np.minimum(mu, 1 - mu)


def chromosome_sizes(total_sites: int, n_chrom: int = 22) -> np.ndarray:
    w = HG38[:n_chrom].astype(np.float64)
    sizes = np.floor(total_sites * w / w.sum()).astype(np.int64)
    sizes[-1] += total_sites - sizes.sum()
    return sizes


# single-group model of bin/simulate_data: per-regime omega
SG_OMEGA = np.array([0.995, 0.975, 0.95, 0.925, 0.9, 0.9])


def _segments_per_regime(rng, n: int, K: int, u: int, kappa: float, omega, start_regime=None):
    """As _segments with a NegBin success probability per regime (the
    single-group model's omega vector): the regime sequence first, then each
    segment's length from its own regime's omega."""
    omega = np.asarray(omega, np.float64)
    mean_len = u + kappa * float(omega.min()) / (1 - float(omega.min()))
    n_seg = int(n / max(mean_len, 1.0) * 1.3) + 16
    first = rng.integers(0, K) if start_regime is None else start_regime
    regs, lens, tot = [], [], 0
    while tot < n:
        steps = rng.integers(1, K, size=n_seg)  # uniform off-diagonal move
        if regs:  # continue from the last regime
            reg = (first + np.cumsum(steps)) % K
        else:
            reg = (first + np.concatenate([[0], np.cumsum(steps[1:])])) % K
        ln = np.maximum(u + rng.negative_binomial(kappa, 1.0 - omega[reg]), 1)
        regs.append(reg)
        lens.append(ln)
        tot += int(ln.sum())
        first = int(reg[-1])
    return np.repeat(np.concatenate(regs), np.concatenate(lens))[:n]


def _segments(rng, n: int, K: int, u: int, kappa: float, omega, start_regime=None):
    """regime per site for n sites of a semi-Markov chain."""
    if np.ndim(omega) > 0:
        return _segments_per_regime(rng, n, K, u, kappa, omega, start_regime)
    mean_len = u + kappa * omega / (1 - omega)
    n_seg = int(n / max(mean_len, 1.0) * 1.3) + 16
    lens = u + rng.negative_binomial(kappa, 1.0 - omega, size=n_seg)
    lens = np.maximum(lens, 1)
    while lens.sum() < n:
        lens = np.concatenate([lens, u + rng.negative_binomial(kappa, 1.0 - omega, size=n_seg)])
        lens = np.maximum(lens, 1)
    steps = rng.integers(1, K, size=lens.shape[0])  # uniform off-diagonal move
    first = rng.integers(0, K) if start_regime is None else start_regime
    reg = (first + np.concatenate([[0], np.cumsum(steps[1:])])) % K
    out = np.repeat(reg, lens)[:n]
    return out


def simulate(n_sites: int, n_ctrl: int, n_case: int, K: int = 6, u: int = 3, omega=0.8,
             kappa: float = 2.0, coverage: float = 100.0, split_frac: float = 0.1, seed: int = DATA_SEED,
             mu=None, sigma=None):
    """Returns dict with uint16 meth/total arrays [T][S] per group and the true
    regimes. omega: the NegBin success probability of every regime, or one per
    regime (SG_OMEGA, the single-group model)."""
    rng = np.random.default_rng(seed)
    if mu is None or sigma is None:
        mu, sigma = regime_params(K)
    nu = mu * (1 - mu) / sigma ** 2 - 1
    alpha, beta = mu * nu, (1 - mu) * nu
    r_ctrl = _segments(rng, n_sites, K, u, kappa, omega)
    # split stretches: geometric lengths, about split_frac of the sites
    mean_split = 200.0
    n_str = max(1, int(n_sites * split_frac / mean_split))
    starts = rng.integers(0, n_sites, size=n_str)
    lens = rng.geometric(1.0 / mean_split, size=n_str)
    split = np.zeros(n_sites, dtype=bool)
    delta = np.zeros(n_sites + 1, dtype=np.int64)
    np.add.at(delta, starts, 1)
    np.add.at(delta, np.minimum(starts + lens, n_sites), -1)
    split = np.cumsum(delta[:-1]) > 0
    r_case_own = _segments(rng, n_sites, K, u, kappa, omega)
    r_case = np.where(split, r_case_own, r_ctrl)
    out = {"regime_control": r_ctrl.astype(np.int8), "regime_case": r_case.astype(np.int8), "split": split}
    for name, reg, S in (("control", r_ctrl, n_ctrl), ("case", r_case, n_case)):
        tot = rng.poisson(coverage, size=(n_sites, S))
        tot = np.minimum(tot, 65535)
        lvl = rng.beta(alpha[reg][:, None], beta[reg][:, None], size=(n_sites, S))
        meth = rng.binomial(tot, lvl)
        out[f"tot_{name}"] = tot.astype(np.uint16)
        out[f"meth_{name}"] = meth.astype(np.uint16)
    return out


def positions(n_sites: int, seed: int = DATA_SEED) -> np.ndarray:
    rng = np.random.default_rng(seed + 1)
    return np.cumsum(1 + rng.geometric(0.01, size=n_sites)).astype(np.int64)


def segment_chains(chrom_sizes, segment_size: int = 100000, buffer_size: int = 5000):
    """(chrom, batch, site_begin, n_sites, return_begin, return_len) per chain, as
    get_chrom_segments.py:246 and run_inference_two_groups.py:194-218 cut them."""
    chains = []
    base = 0
    for ci, n in enumerate(chrom_sizes):
        n = int(n)
        for b in range(1 + n // segment_size):
            if b * segment_size > n:
                break
            lo = max(0, b * segment_size - buffer_size)
            hi = min((b + 1) * segment_size + buffer_size, n)
            if hi <= lo:
                continue
            if b == 0:
                r0, r1 = 0, min(hi - lo, segment_size)
            else:
                r0, r1 = buffer_size, min(hi - lo, buffer_size + segment_size)
            chains.append((ci, b, base + lo, hi - lo, r0, max(0, r1 - r0)))
        base += n
    return chains


def simulate_device(n_sites: int, n_ctrl: int, n_case: int, K: int = 6, u: int = 3, omega=0.8,
                    kappa: float = 2.0, coverage: float = 100.0, split_frac: float = 0.1, seed: int = DATA_SEED,
                    device=None):
    """simulate() with the per-sample draws (Beta levels, Poisson coverage,
    Binomial counts) done on the GPU with torch: 28M sites in seconds. Returns
    int16 device tensors holding the uint16 count bit patterns [T][S]."""
    import torch

    rng = np.random.default_rng(seed)
    mu, sigma = regime_params(K)
    nu = mu * (1 - mu) / sigma ** 2 - 1
    alpha, beta = torch.tensor(mu * nu, device=device), torch.tensor((1 - mu) * nu, device=device)
    r_ctrl = _segments(rng, n_sites, K, u, kappa, omega).astype(np.int8)
    mean_split = 200.0
    n_str = max(1, int(n_sites * split_frac / mean_split))
    starts = rng.integers(0, n_sites, size=n_str)
    lens = rng.geometric(1.0 / mean_split, size=n_str)
    delta = np.zeros(n_sites + 1, dtype=np.int32)
    np.add.at(delta, starts, 1)
    np.add.at(delta, np.minimum(starts + lens, n_sites), -1)
    split = np.cumsum(delta[:-1]) > 0
    r_case = np.where(split, _segments(rng, n_sites, K, u, kappa, omega).astype(np.int8), r_ctrl)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    torch.manual_seed(seed)
    out = {}
    for name, reg, S in (("control", r_ctrl, n_ctrl), ("case", r_case, n_case)):
        rg = torch.from_numpy(reg.astype(np.int64)).to(device)
        a = alpha[rg][:, None].expand(n_sites, S).float()
        b = beta[rg][:, None].expand(n_sites, S).float()
        lvl = torch.distributions.Beta(a, b).sample()
        tot = torch.poisson(torch.full((n_sites, S), float(coverage), device=device), generator=gen)
        tot = tot.clamp(max=65535.0)
        meth = torch.binomial(tot, lvl.clamp(0.0, 1.0), generator=gen)
        out[f"tot_{name}"] = tot.to(torch.int32).to(torch.int16).contiguous()
        out[f"meth_{name}"] = meth.to(torch.int32).to(torch.int16).contiguous()
        del a, b, lvl, tot, meth
    out["regime_control"] = r_ctrl
    out["regime_case"] = r_case
    return out
