"""The job's gather of posterior counts on the device (hyg_tg_posterior_counts,
bench.py's step) against the torch reference parallel.posterior_counts: the
same integers, with segments of two seeds sharing sites, rows at every offset
and probabilities exactly on the k / B grid (round half to even at .5 B)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.mark.parametrize("K,B", [(6, 25), (12, 25), (2, 4)])
def test_device_counts_equal_torch_reference(K, B):
    from hygeia_amd import _lib, parallel

    L = _lib.load()
    if L.hyg_device_count() < 1:
        pytest.fail("no HIP device visible")
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(K * 100 + B)
    n_sites, rows = 5000, 0
    pieces = [(0, 1700, 0), (1700, 2000, 100), (3700, 1300, 60)]  # (first site, sites, leading buffer)
    chains, seg_of = [], {}
    for seed in (0, 1):  # two seeds over the same sites
        for b, (a, n, r0) in enumerate(pieces):
            cid = (7 << 32) | b
            seg_of[cid] = (a - r0, r0, n)  # (site_begin, trim offset, trimmed rows)
            chains.append((a - r0, r0 + n + 40, seed, cid, rows))
            rows += r0 + n + 40
    split = torch.from_numpy((rng.integers(0, B + 1, rows) / B).astype(np.float32)).to(dev)
    regime = torch.from_numpy((rng.integers(0, B + 1, (rows, 2 * K)) / B).astype(np.float32)).to(dev)
    tab = parallel.segment_table(chains, seg_of)
    src = np.concatenate([np.arange(a, a + n) for a, _, n in tab])
    dst = np.concatenate([np.arange(s, s + n) for _, s, n in tab])
    ref = parallel.posterior_counts(split, regime, B, torch.from_numpy(src).to(dev), torch.from_numpy(dst).to(dev),
                                    n_sites)
    # both seeds in one call (atomics), and one exclusive call per seed
    got = torch.zeros_like(ref)
    parallel.posterior_counts_device(L, split, regime, B, torch.from_numpy(tab).to(dev), int(tab[:, 2].max()), got)
    got_x = torch.zeros_like(ref)
    for t in parallel.seed_tables(chains, seg_of):
        parallel.posterior_counts_device(L, split, regime, B, torch.from_numpy(t).to(dev), int(t[:, 2].max()), got_x,
                                         exclusive=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), ref.cpu().numpy())
    np.testing.assert_array_equal(got_x.cpu().numpy(), ref.cpu().numpy())
    assert int(got[:, 0].max()) <= 2 * B


@pytest.mark.parametrize("exclusive", [False, True])
def test_device_counts_more_segments_than_one_grid(exclusive):
    """More than 65 535 segments: the launcher splits the grid's y dimension
    over several launches (dmp_kernels.hip), each with its own segment offset;
    70 000 one- to three-row segments against the torch reference."""
    from hygeia_amd import _lib, parallel

    L = _lib.load()
    if L.hyg_device_count() < 1:
        pytest.fail("no HIP device visible")
    dev = torch.device("cuda", 0)
    K, B, n_seg = 6, 25, 70_000
    rng = np.random.default_rng(70)
    lens = rng.integers(1, 4, n_seg)
    sites = np.concatenate([[0], np.cumsum(lens)[:-1]])  # disjoint, adjacent site ranges
    if not exclusive:  # a second copy of every segment over the same sites: atomics needed
        lens, sites = np.concatenate([lens, lens]), np.concatenate([sites, sites])
    rows_out = np.concatenate([[0], np.cumsum(lens)[:-1]])
    tab = np.stack([rows_out, sites, lens], axis=1).astype(np.int64)
    rows, n_sites = int(lens.sum()), int(sites.max() + lens[np.argmax(sites)] + 1)
    assert parallel.disjoint_sites(tab) == exclusive
    split = torch.from_numpy((rng.integers(0, B + 1, rows) / B).astype(np.float32)).to(dev)
    regime = torch.from_numpy((rng.integers(0, B + 1, (rows, 2 * K)) / B).astype(np.float32)).to(dev)
    src = np.concatenate([np.arange(a, a + n) for a, _, n in tab])
    dst = np.concatenate([np.arange(s, s + n) for _, s, n in tab])
    ref = parallel.posterior_counts(split, regime, B, torch.from_numpy(src).to(dev), torch.from_numpy(dst).to(dev),
                                    n_sites)
    got = torch.zeros_like(ref)
    parallel.posterior_counts_device(L, split, regime, B, torch.from_numpy(tab).to(dev), int(lens.max()), got,
                                     exclusive=exclusive)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), ref.cpu().numpy())
