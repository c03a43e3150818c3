"""Golden vectors of the DMP-calling stage (run in the build container only).

Inputs are seeded synthetic count arrays of the shape get_dmps.py builds
(t = 1 - c / P for per-site counts c over P trajectories); the expected outputs
are those of the REFERENCE's own multiple_testing.py (FDR_procedure,
weighted_FDR_procedure), imported from /root/reference/src/two_group (numpy
only). Saved as data in tests/golden/dmp_fdr.npz:

    case_<i>_counts [n] int32, case_<i>_P, case_<i>_thr, case_<i>_wfn [n] f64
    case_<i>_fdr    [k, Q_k, threshold]            (FDR_procedure)
    case_<i>_widx   ranking_indices[:s] (int64)    (weighted_FDR_procedure, w_fp = 1)
    case_<i>_wsum   Nsums[s - 1]
    tie_*           one more weighted case whose cutoff falls inside a ranking tie group

Usage: python -B tests/golden/make_dmp_golden.py
"""
import os
import sys

import numpy as np

REF = "/root/reference/src/two_group"
HERE = os.path.dirname(os.path.abspath(__file__))


def cases():
    rng = np.random.default_rng(20251024)
    out = []
    for i, (n, P, thr) in enumerate([(2000, 50, 0.05), (2000, 50, 0.01), (5000, 100, 0.2), (3000, 2400, 0.05),
                                     (500, 25, 0.5), (4, 1000, 0.05), (300, 50, 0.001), (200, 50, 0.99)]):
        # mostly "no change" sites (c small -> t near 1) plus a differential block
        c = rng.binomial(P, 0.03, size=n)
        hot = rng.random(n) < 0.15
        c[hot] = rng.binomial(P, rng.uniform(0.6, 1.0, size=int(hot.sum())))
        if i == 5:
            c = np.array([999, 800, 990, 500])  # t = .001, .2, .01, .5
        if i == 7:
            c = rng.binomial(P, 0.9, size=n)  # every running mean below the threshold
        pos = np.cumsum(1 + rng.geometric(0.01, size=n)).astype(np.int64)
        out.append((c.astype(np.int32), P, thr, pos))
    return out


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import multiple_testing as mt  # the reference, numpy only
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import dmp_oracle as od

    blob = {}
    for i, (c, P, thr, pos) in enumerate(cases()):
        t = 1.0 - c.astype(np.int64) / P
        k, q, th = mt.FDR_procedure(t, thr)
        k = int(k[0]) if isinstance(k, tuple) else int(k)
        wfn = od.false_negative_weights(pos)
        widx, wsum = mt.weighted_FDR_procedure(t, fdr_threshold=thr, weights_false_negatives=wfn,
                                               weights_false_positives=np.ones(t.shape[0]))
        blob[f"case_{i}_counts"] = c
        blob[f"case_{i}_P"] = np.int64(P)
        blob[f"case_{i}_thr"] = np.float64(thr)
        blob[f"case_{i}_pos"] = pos
        blob[f"case_{i}_wfn"] = wfn
        blob[f"case_{i}_fdr"] = np.array([k, q, th], dtype=np.float64)
        blob[f"case_{i}_widx"] = np.sort(np.asarray(widx, dtype=np.int64))
        blob[f"case_{i}_wsum"] = np.float64(wsum)
    blob["n_cases"] = np.int64(len(cases()))
    # a weighted-FDR cutoff inside a ranking tie group: equally spaced sites
    # (equal false-negative weights) and P = 10 (few distinct statistics); the
    # reference ranks with np.argsort's default (unstable) sort, so WHICH tied
    # sites it selects at the boundary is an accident of numpy's introsort
    rng = np.random.default_rng(5)
    n, P, thr = 3000, 10, 0.3
    c = rng.binomial(P, 0.5, size=n).astype(np.int32)
    pos = (np.arange(n) * 100 + 1000).astype(np.int64)
    t = 1.0 - c.astype(np.int64) / P
    wfn = od.false_negative_weights(pos)
    widx, wsum = mt.weighted_FDR_procedure(t, fdr_threshold=thr, weights_false_negatives=wfn,
                                           weights_false_positives=np.ones(n))
    blob.update(tie_counts=c, tie_P=np.int64(P), tie_thr=np.float64(thr), tie_wfn=wfn,
                tie_widx=np.sort(np.asarray(widx, dtype=np.int64)), tie_wsum=np.float64(wsum))
    np.savez_compressed(os.path.join(HERE, "dmp_fdr.npz"), **blob)
    print("wrote", os.path.join(HERE, "dmp_fdr.npz"), blob["n_cases"], "cases")


if __name__ == "__main__":
    main()
