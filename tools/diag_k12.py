"""Diagnostic: the K=12 chain of tests/test_gpu_two_group.py, GPU vs oracle, mismatch statistics."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import binding as ob
from hygeia_amd import synthetic as syn, two_group

K, M, B, T, S, cov, dseed, seed = (12, 50, 25, 300, 6, 100.0, 20, 9)
mu, sg = syn.regime_params(K)
d = syn.simulate(T, S, S, K=K, seed=dseed, coverage=cov, split_frac=0.1)
p = ob.make_params(K=K, M=M, B=B, mu=mu, sigma=sg)
theta = np.array(p.theta[: p.theta_len])
E = ob.emission(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
ref = ob.chain(p, E, seed, 1000 + seed)
maxr = int(max(d["tot_control"].max(), d["tot_case"].max()))
model = two_group.CaseControlModel(mu, sg, theta, num_resampled_ancestors=M, num_samples_backward=B,
                                   max_total_reads=maxr, max_duration=T + 5)
res, fw, ex = two_group.run({"control": d["meth_control"], "case": d["meth_case"]},
                            {"control": d["tot_control"], "case": d["tot_case"]}, model, seed, 1000 + seed)
pr = res.particle
print("finalw equal", np.array_equal(np.asarray(fw), np.asarray(ref["final_w"])) if "final_w" in ref else list(ref.keys()))
for k, r in (("merged_state", "merged"), ("control_state", "control"), ("case_state", "case")):
    a, b = np.asarray(pr[k]), np.asarray(ref[r])
    bad = np.argwhere(a != b)
    print(k, a.shape, "mismatches", len(bad), "first", bad[:5].tolist())
    if len(bad):
        t0 = bad[0][0]
        print("  site", t0, "gpu", a[t0].tolist()[:10], "ref", b[t0].tolist()[:10])
print("logz gpu/ref", ex.get("log_z"), ref.get("log_z"))
