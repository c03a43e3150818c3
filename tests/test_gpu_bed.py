"""SURVEY.md 8f-4 on the GPU: hyg_bed_labels (per-site max, first argmax,
"equiprobable" ties) bit-exact against the restatement of make_bed_file:27-39,
and `hygeia make_bed_file` end to end on a regimes CSV written the way
estimate_parameters_and_regimes:325-338 writes it (R format(): padded fixed
notation)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from tests.test_bed import r_labels, r_make_bed, regimes_probs  # noqa: E402


@pytest.fixture(scope="module")
def lib():
    from hygeia_amd import _lib

    L = _lib.load()
    if L.hyg_device_count() <= 0:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X (gpurun)")
    return L


@pytest.mark.parametrize("K,n", [(6, 1_000_003), (2, 1000), (12, 4097), (16, 50), (6, 1)])
def test_labels_bit_exact(lib, K, n):
    from hygeia_amd import bed

    probs = regimes_probs(n, K, K * 7 + n)
    lab, sc = bed.labels(probs)
    rl, rs = r_labels(probs)
    np.testing.assert_array_equal(lab, rl)
    np.testing.assert_array_equal(sc, rs)


def test_make_bed_file_end_to_end(lib, tmp_path):
    from hygeia_amd import bed, cli

    K, n = 6, 20000
    probs = regimes_probs(n, K, 5)
    pos = np.cumsum(np.random.default_rng(6).integers(1, 200, n)) + 1000
    cols = [f"regime_{r + 1}" for r in range(K)]
    # R: mutate(across(where(is.numeric), ~ format(., scientific = FALSE))) pads to a common width
    w = len(str(pos.max()))
    with open(tmp_path / "regimes_21.csv", "w") as fh:
        fh.write("genomic_position," + ",".join(cols) + "\n")
        for i in range(n):
            fh.write(f"{pos[i]:>{w}d}," + ",".join(f"{v:.7f}" for v in probs[i]) + "\n")
    out = tmp_path / "nextflow_output" / "s1_regimes_21.bed"
    rc = cli.main(["make_bed_file", "--chr", "21", "--regimes_file", str(tmp_path / "regimes_21.csv"),
                   "--output_file", str(out)])
    assert rc == 0
    assert out.read_bytes() == r_make_bed("21", pos, np.round(probs, 7), cols)


@pytest.mark.parametrize("K", [6, 4])
def test_labels_on_an_8_byte_aligned_view(lib, K):
    """hyg_bed_labels takes any device pointer: a view at an odd element offset
    (8- but not 16-byte aligned) must take the scalar-load path."""
    from hygeia_amd import _lib

    n = 5001
    probs = regimes_probs(n, K, 99)
    buf = torch.zeros(n * K + 1, dtype=torch.float64, device="cuda")
    view = buf[1:].view(n, K)
    view.copy_(torch.from_numpy(probs).cuda())
    assert view.data_ptr() % 16 == 8
    lab = torch.empty(n, dtype=torch.int8, device="cuda")
    sc = torch.empty(n, dtype=torch.float64, device="cuda")
    _lib.check(lib.hyg_bed_labels(view.data_ptr(), K, n, lab.data_ptr(), sc.data_ptr(),
                                  C.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    rl, rs = r_labels(probs)
    np.testing.assert_array_equal(lab.cpu().numpy(), rl)
    np.testing.assert_array_equal(sc.cpu().numpy(), rs)
