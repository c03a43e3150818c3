"""GPU parity at the BASELINE.json configurations' own sizes (bit-exact against
the CPU oracle, every output array compared):

- C5 (configs[4]): 50 + 50 samples, K = 12, M = 50, B = 25 -- the emission on
  50-sample rows (hyg_tg_emission on the device) and a whole chain; round 5:
  two full-length 110 000-site chains of that shape through the production
  (512 / 768-thread, shape-specialised) kernels, against the oracle's digests
  (tests/golden/c5_chain_digest.json, made by tests/golden/make_c5_chain.py:
  the oracle needs about 6 minutes per chain at this shape);
- C3 (configs[2]): full-length segment chains of 110 000 sites (the reference's
  100 000-site segment + 2 x 5 000 buffers, run_inference_two_groups.py:67-72,
  194-218), 4 + 4 samples, K = 6, M = 50, B = 25: one on the synthetic
  generative model, and one on a single-regime stretch whose sojourns outgrow
  the float32 hazard saturation (case_control_regime_model.py:111-168) and wrap
  the int16 duration outputs (run_inference_two_groups.py:292-314);
- C2 (configs[1]): one single-group chain of 200 000 sites at the pipeline
  settings (4 samples, K = 6, N_max = 250, epsilon = 0.01), long enough for the
  log-weights to reach the large-magnitude regime noted in DESIGN.md 1;
- C2 at full length (round 6): the chromosome-1 chain of the C2 genome
  (2 424 617 sites, the C2 bench's critical chain), with and without the
  pipeline's online parameter estimation, against the oracle's digests
  (tests/golden/sg_long_digest.json, made by tests/golden/make_sg_long.py);
- C1 (configs[0]): the whole chr21-sized single-group chain (454 914 sites of
  the 28M-site genome), 2 samples, K = 6, N_max = 250,
  epsilon = 0.01, 1 seed, data from the single-group model (per-regime omega),
  as estimate_parameters_and_regimes:303-322 runs it per chromosome.

The oracle chains take about a minute each on one core; they run in threads
(ctypes releases the GIL) started when the module is first used, overlapping
the GPU work.
"""
import concurrent.futures as cf
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

T_LONG = 110_000


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    from hygeia_amd import _lib

    if _lib.load().hyg_device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X (gpurun)")


def _long_inputs():
    from hygeia_amd import synthetic as syn

    d = syn.simulate(T_LONG, 4, 4, K=6, seed=41, coverage=100.0)
    rng = np.random.default_rng(5)
    tot = rng.poisson(30, size=(T_LONG, 8)).astype(np.uint16)
    meth = rng.binomial(tot.astype(np.int64), 0.95).astype(np.uint16)
    c = {"meth_control": meth[:, :4].copy(), "tot_control": tot[:, :4].copy(),
         "meth_case": meth[:, 4:].copy(), "tot_case": tot[:, 4:].copy()}
    return {"synthetic": d, "one_regime": c}


@pytest.fixture(scope="module")
def long_refs(oracle):
    """Oracle runs of the two 110k chains and the 200k single-group chain, in
    background threads."""
    from hygeia_amd import synthetic as syn
    from oracle import sg_binding as sgb

    data = _long_inputs()
    mu, sg = syn.regime_params(6)
    p = oracle.make_params(K=6, M=50, B=25, mu=mu, sigma=sg)

    def tg(name):
        d = data[name]
        E = oracle.emission(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
        return E, oracle.chain(p, E, 2, (7 << 32) | 3)

    sgd = syn.simulate(200_000, 4, 1, K=6, seed=77, coverage=100.0, omega=0.95)
    psg = sgb.make_params(K=6)

    def sgchain():
        E = sgb.emission(psg, sgd["meth_control"], sgd["tot_control"])
        return sgb.chain(psg, E, seed=3, chain_id=5)

    c1d = syn.simulate(int(syn.chromosome_sizes(28_000_000)[20]), 2, 1, K=6, seed=2121, coverage=100.0,
                       omega=syn.SG_OMEGA)

    def c1chain():
        E = sgb.emission(psg, c1d["meth_control"], c1d["tot_control"])
        return sgb.chain(psg, E, seed=1, chain_id=20)

    ex = cf.ThreadPoolExecutor(max_workers=4)
    futs = {"c1": ex.submit(c1chain), "synthetic": ex.submit(tg, "synthetic"),
            "one_regime": ex.submit(tg, "one_regime"), "sg": ex.submit(sgchain)}
    yield data, futs, (sgd, psg, c1d)
    ex.shutdown(wait=True)


def _compare(res, fw, ex, ref):
    pr = res.particle
    np.testing.assert_array_equal(pr["merged_state"], ref["merged"])
    np.testing.assert_array_equal(pr["control_state"], ref["control"])
    np.testing.assert_array_equal(pr["case_state"], ref["case"])
    np.testing.assert_array_equal(ex["split_probs"], ref["split_probs"])
    np.testing.assert_array_equal(ex["regime_probs"], ref["regime_probs"])
    assert ex["log_z"] == ref["log_z"]
    np.testing.assert_array_equal(fw, ref["final_log_weights"])


def _model(mu, sg, theta, M, B, max_reads, max_dur):
    from hygeia_amd import two_group

    return two_group.CaseControlModel(mu, sg, theta, num_resampled_ancestors=M, num_samples_backward=B,
                                      max_total_reads=max_reads, max_duration=max_dur)


@pytest.mark.timeout(300)
def test_c5_emission_and_chain(oracle):
    """C5: 50 + 50 samples, K = 12 (N_max = 8400)."""
    from hygeia_amd import synthetic as syn
    from hygeia_amd import two_group

    K, M, B, T = 12, 50, 25, 400
    mu, sg = syn.regime_params(K)
    d = syn.simulate(T, 50, 50, K=K, seed=3, coverage=100.0)
    p = oracle.make_params(K=K, M=M, B=B, mu=mu, sigma=sg)
    theta = np.array(p.theta[: p.theta_len])
    E_ref = oracle.emission(p, d["meth_control"], d["tot_control"], d["meth_case"], d["tot_case"])
    maxr = int(max(d["tot_control"].max(), d["tot_case"].max()))
    model = _model(mu, sg, theta, M, B, maxr, T + 5)
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(np.ascontiguousarray(d[k]).view(np.int16)).to(dev) for k in
         ("meth_control", "tot_control", "meth_case", "tot_case")}
    dc = two_group.DeviceChains(model, [(0, T, 4, 99, 0)], T, device=dev, final_weights=True)
    E = dc.emission(t["meth_control"], t["tot_control"], t["meth_case"], t["tot_case"])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(E.cpu().numpy(), E_ref)
    ref = oracle.chain(p, E_ref, 4, 99)
    assert ref["status"] == 0
    res, fw, ex = two_group.run({"control": d["meth_control"], "case": d["meth_case"]},
                                {"control": d["tot_control"], "case": d["tot_case"]}, model, 4, 99)
    _compare(res, fw, ex, ref)
    # the batched device path gives the same chain
    dc.run(E)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dc.control.cpu().numpy(), ref["control"])
    np.testing.assert_array_equal(dc.regime_probs.cpu().numpy(), ref["regime_probs"])
    assert dc.log_z[0].item() == ref["log_z"]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", ["synthetic", "one_regime"])
def test_c3_full_length_chain(oracle, long_refs, name):
    from hygeia_amd import synthetic as syn
    from hygeia_amd import two_group

    data, futs, _ = long_refs
    d = data[name]
    mu, sg = syn.regime_params(6)
    model = _model(mu, sg, two_group.uniform_theta(6, 0.8), 50, 25,
                   int(max(d["tot_control"].max(), d["tot_case"].max())), T_LONG)
    res, fw, ex = two_group.run({"control": d["meth_control"], "case": d["meth_case"]},
                                {"control": d["tot_control"], "case": d["tot_case"]}, model, 2, (7 << 32) | 3)
    _, ref = futs[name].result()
    assert ref["status"] == 0
    _compare(res, fw, ex, ref)
    if name == "one_regime":
        dur = ref["control"][:, :, 0].astype(np.int64)
        assert dur.min() < 0  # the int16 duration output wrapped (sojourn > 32767 sites)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("bwd", [0, 256])
@pytest.mark.parametrize("name", ["synthetic", "one_regime"])
def test_c5_full_length_chain(name, bwd):
    """C5 at full segment length: 110 000 sites, 50 + 50 samples, K = 12, M = 50,
    B = 25, every output array bit-exact against the oracle (as digests, with
    per-10 000-row block digests to locate a difference); one chain on the
    synthetic model, one on a single-level stretch past the float32 hazard
    saturation whose int16 duration outputs wrap. bwd = 256: the backward width
    of a C5 launch with more chains than CUs, whose full-N weights live in
    global memory (GW); 0: the automatic width of one chain (768, LDS)."""
    import importlib.util
    import json
    import os

    from hygeia_amd import _lib
    from hygeia_amd import synthetic as syn
    from hygeia_amd import two_group

    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    spec = importlib.util.spec_from_file_location("make_c5_chain", os.path.join(here, "make_c5_chain.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    with open(g.OUT) as f:
        doc = json.load(f)
    ref = doc["chains"][name]
    d = g.inputs(name)
    assert g.input_digest(d) == ref["inputs"], "the input generator changed: regenerate the fixture"
    K, M, B, T = doc["K"], doc["M"], doc["B"], doc["T"]
    mu, sg = syn.regime_params(K)
    model = _model(mu, sg, two_group.uniform_theta(K, 0.8), M, B,
                   int(max(d["tot_control"].max(), d["tot_case"].max())), T)
    L = _lib.load()
    # the production shape: one chain per CU at most, so the wide (512-thread
    # forward / 768-thread backward) shape-specialised kernels run
    assert L.hyg_tg_threads_per_chain(model.handle, 1) == 512
    assert L.hyg_tg_force_threads(0, bwd) == 0
    try:
        res, fw, ex = two_group.run({"control": d["meth_control"], "case": d["meth_case"]},
                                    {"control": d["tot_control"], "case": d["tot_case"]}, model, ref["seed"],
                                    ref["chain_id"])
    finally:
        L.hyg_tg_force_threads(0, 0)
    out = {"merged": res.particle["merged_state"], "control": res.particle["control_state"],
           "case": res.particle["case_state"], "split_probs": ex["split_probs"],
           "regime_probs": ex["regime_probs"], "final_log_weights": fw, "log_z": ex["log_z"]}
    got = g.output_record(out)
    print(f"C5 {name}: oracle step modes {ref['modes']}, min duration output {ref['min_duration_output']}")
    for k in g.OUTPUTS:
        if got[k] != ref[k]:
            blocks = [i for i, (a, b) in enumerate(zip(got.get(k + "_blocks", []), ref.get(k + "_blocks", [])))
                      if a != b]
            pytest.fail(f"{name}: {k} differs from the oracle (first differing {g.BLOCK}-row blocks: {blocks[:5]})")
    assert got["log_z"] == ref["log_z"]
    if name == "one_regime":
        assert ref["min_duration_output"] < 0  # the int16 duration output wrapped (sojourn > 32767 sites)


def _sg_host_chain(psg, meth, tot, seed, chain_id):
    from hygeia_amd import _lib

    L = _lib.load()
    p = _lib.SgParams.from_buffer_copy(bytes(psg))
    h = C.c_void_p()
    meth = np.ascontiguousarray(meth, np.uint16)
    tot = np.ascontiguousarray(tot, np.uint16)
    T, S = tot.shape
    _lib.check(L.hyg_sg_model_create(C.byref(p), int(tot.max()), T + 10, C.byref(h)))
    try:
        out = np.full((T, 6), np.nan)
        rc = L.hyg_sg_run_chain_host(h, meth.ctypes.data_as(C.c_void_p), tot.ctypes.data_as(C.c_void_p), S, T, seed,
                                     chain_id, out.ctypes.data_as(C.c_void_p))
        assert rc == 0, L.hyg_last_error()
    finally:
        L.hyg_sg_model_destroy(h)
    return out


@pytest.mark.timeout(600)
def test_c2_single_group_200k_chain(long_refs):
    _, futs, (sgd, psg, _) = long_refs
    out = _sg_host_chain(psg, sgd["meth_control"], sgd["tot_control"], 3, 5)
    ref = futs["sg"].result()
    assert ref["status"] == 0
    bad = np.argwhere(out != ref["regime_probs"])
    assert bad.size == 0, (len(bad), bad[:5])
    np.testing.assert_allclose(out.sum(1), 1.0, atol=1e-8)


def _sg_long_fixture():
    import importlib.util
    import json
    import os

    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    spec = importlib.util.spec_from_file_location("make_sg_long", os.path.join(here, "make_sg_long.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    with open(g.OUT) as f:
        doc = json.load(f)
    d = g.inputs()
    assert g.input_digest(d) == doc["inputs"], "the input generator changed: regenerate the fixture"
    return g, doc, d


def _first_bad_blocks(got, ref):
    return [i for i, (a, b) in enumerate(zip(got, ref)) if a != b][:5]


@pytest.mark.timeout(900)
def test_c2_chr1_chain():
    """C2's critical chain at the length the pipeline runs it: chromosome 1 of
    the 28 M genome (2 424 617 sites), 4 samples, K = 6, N_max = 250,
    epsilon = 0.01, every regime probability bit-exact against the oracle's
    digests (tests/golden/make_sg_long.py)."""
    from hygeia_amd import _lib

    g, doc, d = _sg_long_fixture()
    ref = doc["chains"]["plain"]
    p = _lib.SgParams.from_buffer_copy(bytes(g.params(False)))
    out = _sg_host_chain(p, d["meth_control"], d["tot_control"], ref["seed"], ref["chain_id"])
    got = g.output_record(out)
    assert got["regime_probs"] == ref["regime_probs"], (
        "chr1 chain differs from the oracle; first differing 100k-row blocks: "
        f"{_first_bad_blocks(got['regime_probs_blocks'], ref['regime_probs_blocks'])}")


@pytest.mark.timeout(1200)
def test_c2_chr1_pe_chain():
    """The pipeline's step 2 on the same chromosome-1 chain: online parameter
    estimation (ADAM, an update every 200 steps, theta_0 from the prior), the
    regime probabilities and all 12 124 theta rows bit-exact against the
    oracle's digests."""
    from hygeia_amd import _lib

    g, doc, d = _sg_long_fixture()
    ref = doc["chains"]["pe"]
    L = _lib.load()
    p = _lib.SgParams.from_buffer_copy(bytes(g.params(True)))
    pe = _lib.SgPeParams()
    L.hyg_sg_pe_params_default(C.byref(pe))
    assert pe.n_steps_without_update == ref["every"]
    meth = np.ascontiguousarray(d["meth_control"], np.uint16)
    tot = np.ascontiguousarray(d["tot_control"], np.uint16)
    T, S = tot.shape
    h = C.c_void_p()
    _lib.check(L.hyg_sg_model_create(C.byref(p), int(tot.max()), T + 10, C.byref(h)))
    try:
        out = np.full((T, 6), np.nan)
        th = np.full((1 + (T - 1) // ref["every"], 36), np.nan)
        rc = L.hyg_sg_run_chain_host_pe(h, C.byref(pe), meth.ctypes.data_as(C.c_void_p),
                                        tot.ctypes.data_as(C.c_void_p), S, T, ref["seed"], ref["chain_id"],
                                        out.ctypes.data_as(C.c_void_p), th.ctypes.data_as(C.c_void_p))
        assert rc == 0, L.hyg_last_error()
    finally:
        L.hyg_sg_model_destroy(h)
    got = g.output_record(out, th)
    assert got["theta"] == ref["theta"], (
        "theta rows differ from the oracle; first differing 1000-row blocks: "
        f"{_first_bad_blocks(got['theta_blocks'], ref['theta_blocks'])}")
    assert got["regime_probs"] == ref["regime_probs"], (
        "regime probabilities differ from the oracle; first differing 100k-row blocks: "
        f"{_first_bad_blocks(got['regime_probs_blocks'], ref['regime_probs_blocks'])}")


@pytest.mark.timeout(600)
def test_c1_single_group_chr21_chain(long_refs):
    """C1 in full: the chr21-sized chain (454 914 sites), S = 2, bit-exact."""
    _, futs, (_, psg, c1d) = long_refs
    assert c1d["tot_control"].shape == (454914, 2)
    out = _sg_host_chain(psg, c1d["meth_control"], c1d["tot_control"], 1, 20)
    ref = futs["c1"].result()
    assert ref["status"] == 0
    bad = np.argwhere(out != ref["regime_probs"])
    assert bad.size == 0, (len(bad), bad[:5])
    np.testing.assert_allclose(out.sum(1), 1.0, atol=1e-8)
