"""Generates the committed golden fixtures under tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).

The reference's two-group engine needs TensorFlow 2.3 / TFP 0.11, which are absent
here, and the reference ships no golden vectors. The fixtures are
therefore produced by the CPU oracle (oracle/tg_oracle.c), which tests/test_oracle.py
cross-checks bit for bit against the independent pure-Python restatement
(oracle/tg_oracle_np.py) and tests/test_model_tables.py pins against scipy and
SURVEY.md Appendix C. Inputs come from hygeia_amd/synthetic.simulate (numpy, seeded).

Fixtures (npz, inputs + expected outputs):
  tg_chain_k6.npz    T=2000, 2+2 samples, K=6, M=10, B=5, coverage 30 (SURVEY.md 8c iv)
  tg_chain_k4.npz    T=700, 3+2 samples, K=4, M=50, B=25, coverage 100, a zero-coverage stretch
  tg_tables.npz      BB emission grid + hazard rows (log rho, log 1-rho) for the pipeline defaults
  sg_chain_k6.npz    single group (oracle/sg_oracle.c): T=3000, S=2, K=6, pipeline defaults
                     (N_max=250, epsilon=0.01, u=3), coverage 12
  sg_chain_k3.npz    single group: T=800, S=3, K=3, N_max=20, epsilon=1e-4, u=2, a zero-coverage stretch

The single-group oracle is pinned by tests/test_sg_oracle.py (exact semi-Markov
smoother without resampling, scipy tables).
``python tests/golden/make_golden.py sg`` regenerates only the sg_* fixtures, ``... tg`` only
the two-group chains.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from hygeia_amd import synthetic as syn  # noqa: E402
from oracle import binding as ob  # noqa: E402
from oracle import sg_binding as sb  # noqa: E402

CHAINS = {
    "tg_chain_k6": dict(K=6, M=10, B=5, T=2000, S=(2, 2), coverage=30.0, data_seed=11, seed=0, chain_id=3),
    "tg_chain_k4": dict(K=4, M=50, B=25, T=700, S=(3, 2), coverage=100.0, data_seed=12, seed=5, chain_id=(7 << 32) | 2,
                        zero=(300, 340)),
}


def chain_fixture(name: str, K, M, B, T, S, coverage, data_seed, seed, chain_id, zero=None):
    mu, sg = syn.regime_params(K)
    d = syn.simulate(T, S[0], S[1], K=K, coverage=coverage, seed=data_seed)
    if zero is not None:
        for k in ("meth_control", "tot_control", "meth_case", "tot_case"):
            d[k][zero[0]:zero[1]] = 0
    p = ob.make_params(K=K, M=M, B=B, mu=mu, sigma=sg)
    E = ob.emission(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
    out = ob.chain(p, E, seed, chain_id)
    assert out["status"] == 0
    np.savez_compressed(
        os.path.join(HERE, name + ".npz"),
        K=K, M=M, B=B, seed=np.uint64(seed), chain_id=np.uint64(chain_id), mu=mu, sigma=sg,
        meth_control=d["meth_control"], tot_control=d["tot_control"], meth_case=d["meth_case"],
        tot_case=d["tot_case"], regime_control=d["regime_control"], regime_case=d["regime_case"],
        split=d["split"], E=E, merged=out["merged"], control=out["control"], case=out["case"],
        split_probs=out["split_probs"], regime_probs=out["regime_probs"], log_z=out["log_z"],
        final_log_weights=out["final_log_weights"])


def tables_fixture():
    p = ob.make_params(K=6)
    rng = np.random.default_rng(13)
    tot = rng.integers(0, 400, size=(256, 2)).astype(np.uint16)
    meth = np.minimum((tot * rng.uniform(size=tot.shape)).astype(np.uint16), tot)
    z = np.zeros((256, 1), np.uint16)
    E = ob.emission(p, meth, tot, z, z)
    hz = np.stack([np.stack([ob.hazard(p, g, r, 200) for r in range(6)]) for g in range(2)])
    np.savez_compressed(os.path.join(HERE, "tg_tables.npz"), meth=meth, tot=tot, E=E, hazard=hz)


SG_CHAINS = {
    "sg_chain_k6": dict(K=6, T=3000, S=2, coverage=12.0, data_seed=31, seed=4, chain_id=(21 << 32) | 1,
                        u=3, Nmax=250, epsilon=0.01, omega=None),
    "sg_chain_k3": dict(K=3, T=800, S=3, coverage=8.0, data_seed=32, seed=9, chain_id=5, u=2, Nmax=20,
                        epsilon=1e-4, omega=(0.9, 0.85, 0.95), zero=(200, 260)),
}


def sg_chain_fixture(name, K, T, S, coverage, data_seed, seed, chain_id, u, Nmax, epsilon, omega, zero=None):
    mu, sg = syn.regime_params(K)
    d = syn.simulate(T, S, 1, K=K, coverage=coverage, seed=data_seed, u=u, omega=0.9)
    meth, tot = d["meth_control"], d["tot_control"]
    if zero is not None:
        meth[zero[0]:zero[1]] = 0
        tot[zero[0]:zero[1]] = 0
    P = np.full((K, K), 1.0 / (K - 1))
    np.fill_diagonal(P, 0.0)
    if omega is None:
        omega = sb.DEFAULT_OMEGA if K == 6 else [0.95] * K
    omega = np.asarray(omega, np.float64)
    p = sb.make_params(K=K, mu=mu, sigma=sg, P=P, omega=omega, u=u, Nmax=Nmax, epsilon=epsilon)
    E = sb.emission(p, meth, tot)
    out = sb.chain(p, E, seed, chain_id)
    assert out["status"] == 0
    np.savez_compressed(os.path.join(HERE, name + ".npz"), K=K, u=u, Nmax=Nmax, epsilon=epsilon,
                        seed=np.uint64(seed), chain_id=np.uint64(chain_id), mu=mu, sigma=sg, P=P, omega=omega,
                        meth=meth, tot=tot, regime=d["regime_control"], E=E, regime_probs=out["regime_probs"])


def sg_pe_fixture():
    """single-group chain with online parameter estimation (8f-1): pipeline
    model (make_params defaults), ADAM, an update every 100 steps"""
    T, every, seed, chain_id = 2500, 100, 4, (9 << 32) | 1
    d = syn.simulate(T, 2, 1, K=6, coverage=15.0, seed=41, u=3, omega=0.9)
    meth, tot = d["meth_control"], d["tot_control"]
    p = sb.make_params(K=6)
    out = sb.chain_pe(p, sb.make_pe(every=every), sb.emission(p, meth, tot), seed, chain_id)
    assert out["status"] == 0
    np.savez_compressed(os.path.join(HERE, "sg_pe_chain.npz"), every=every, seed=np.uint64(seed),
                        chain_id=np.uint64(chain_id), meth=meth, tot=tot, regime_probs=out["regime_probs"],
                        theta=out["theta"])


def main():
    only_sg = "sg" in sys.argv[1:]
    if "sg_pe" in sys.argv[1:]:
        sg_pe_fixture()
        return
    if not only_sg:
        for name, kw in CHAINS.items():
            chain_fixture(name, **kw)
        if "tg" in sys.argv[1:]:  # the two-group chains only
            return
        tables_fixture()
    for name, kw in SG_CHAINS.items():
        sg_chain_fixture(name, **kw)
    sg_pe_fixture()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
