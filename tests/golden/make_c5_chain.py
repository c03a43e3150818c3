"""Generates tests/golden/c5_chain_digest.json: the CPU oracle's outputs on two
full-length chains of the stress shape (BASELINE.json configs[4]: 50 + 50
samples, K = 12, M = 50, B = 25) as SHA-256 digests (run from the repo root:
``python tests/golden/make_c5_chain.py``; about 6 minutes per chain on one core,
the two chains in threads).

Each chain is 110 000 sites, the reference's longest task (a 100 000-site
segment + 2 x 5 000 buffers, run_inference_two_groups.py:67-72,194-218):

- ``synthetic``: the generative model of simulate_two_groups.py at K = 12
  (hygeia_amd/synthetic.simulate, coverage 100);
- ``one_regime``: every site drawn from one methylation level, so the sojourns
  run past the float32 hazard saturation (case_control_regime_model.py:111-168)
  and the int16 duration outputs wrap (run_inference_two_groups.py:292-314).

The outputs (5.5 MB of merged states, 11 MB each of control / case states, 10.5
MB of regime probabilities per chain) are too large to commit, so the fixture
holds the digest of every output array, of every 10 000-row block of it (to
locate a mismatch), of the inputs and of the emission table (to detect a
change of the input generator), and the oracle's step-mode counts (keep-all /
optimal finite-state / unbiased fallback). tests/test_gpu_configs.py::
test_c5_full_length_chain recomputes the inputs, runs them through the HIP
path and compares digests: bit-exact or failed.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from hygeia_amd import synthetic as syn  # noqa: E402

OUT = os.path.join(HERE, "c5_chain_digest.json")
T, S, K, M, B = 110_000, 50, 12, 50, 25
BLOCK = 10_000
CHAINS = {"synthetic": dict(seed=4, chain_id=(11 << 32) | 7),
          "one_regime": dict(seed=1, chain_id=(11 << 32) | 8)}
MODES = {0: "keep_all", 1: "optimal", 2: "unbiased"}


def inputs(name: str) -> dict:
    """The chain's read counts (numpy-seeded, identical on every host with this
    numpy)."""
    if name == "synthetic":
        return syn.simulate(T, S, S, K=K, seed=53, coverage=100.0)
    rng = np.random.default_rng(54)
    tot = rng.poisson(30, size=(T, 2 * S)).astype(np.uint16)
    meth = rng.binomial(tot.astype(np.int64), 0.95).astype(np.uint16)
    return {"meth_control": meth[:, :S].copy(), "tot_control": tot[:, :S].copy(),
            "meth_case": meth[:, S:].copy(), "tot_case": tot[:, S:].copy()}


def digest(a: np.ndarray) -> str:
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.dtype.str.encode() + str(a.shape).encode() + a.tobytes()).hexdigest()


def block_digests(a: np.ndarray) -> list:
    return [digest(a[i:i + BLOCK]) for i in range(0, a.shape[0], BLOCK)]


def input_digest(d: dict) -> str:
    return hashlib.sha256(b"".join(np.ascontiguousarray(d[k]).tobytes() for k in
                                   ("meth_control", "tot_control", "meth_case", "tot_case"))).hexdigest()


OUTPUTS = ("merged", "control", "case", "split_probs", "regime_probs", "final_log_weights")


def output_record(out: dict) -> dict:
    rec = {"log_z": float(out["log_z"]).hex()}
    for k in OUTPUTS:
        rec[k] = digest(out[k])
        if out[k].shape[0] == T:
            rec[k + "_blocks"] = block_digests(out[k])
    return rec


def run_chain(name: str) -> dict:
    from oracle import binding as ob

    mu, sg = syn.regime_params(K)
    d = inputs(name)
    p = ob.make_params(K=K, M=M, B=B, mu=mu, sigma=sg)
    E = ob.emission(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
    cfg = CHAINS[name]
    out = ob.chain(p, E, cfg["seed"], cfg["chain_id"], want_modes=True)
    assert out["status"] == 0
    modes = out["modes"][1:] // 65536
    rec = {"seed": cfg["seed"], "chain_id": cfg["chain_id"], "inputs": input_digest(d), "emission": digest(E),
           "modes": {MODES[k]: int((modes == k).sum()) for k in MODES},
           "min_duration_output": int(min(out["control"][:, :, 0].min(), out["case"][:, :, 0].min()))}
    rec.update(output_record(out))
    return rec


def main() -> None:
    with cf.ThreadPoolExecutor(max_workers=len(CHAINS)) as ex:
        futs = {n: ex.submit(run_chain, n) for n in CHAINS}
        recs = {n: f.result() for n, f in futs.items()}
    doc = {"T": T, "S": S, "K": K, "M": M, "B": B, "block": BLOCK, "numpy": np.__version__, "chains": recs}
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    for n, r in recs.items():
        print(n, r["modes"], "min duration output", r["min_duration_output"])


if __name__ == "__main__":
    main()
