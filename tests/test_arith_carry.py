"""The hipcc forms of the multiword fixed-point primitives in include/hyg_arith.h
(32-bit __builtin_addc / __builtin_subc carry chains, the forms the GPU kernels
compile) against exact Python integers. The gcc-built oracle uses the C forms,
which tests/test_arith.py and every oracle test exercise; together they pin
both sides of the bit-exact contract to the same integers.

The program is compiled for the host by hipcc (the same builtins and the same
header the device code uses); no GPU is needed.
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

PROG = r"""
#include <hip/hip_runtime.h>
#include <cstdio>
#include "hyg_arith.h"
static uint64_t st = 0x9E3779B97F4A7C15ull;
static uint64_t nx() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
static uint64_t word() {  // edge-heavy: 0, all ones, small, random
  const uint64_t x = nx();
  switch (nx() & 3) { case 0: return 0; case 1: return ~0ull; case 2: return x & 0xff; default: return x; }
}
int main() {
  for (int i = 0; i < 4000; ++i) {
    hyg_u128 a{word(), word()}, b{word(), word()};
    if ((nx() & 7) == 0) b = a;
    const hyg_u128 s = hyg_u128_add(a, b);
    printf("A %016llx %016llx %016llx %016llx %016llx %016llx %d\n", (unsigned long long)a.lo,
           (unsigned long long)a.hi, (unsigned long long)b.lo, (unsigned long long)b.hi, (unsigned long long)s.lo,
           (unsigned long long)s.hi, hyg_u128_lt(a, b));
    hyg_u192 x{word(), word(), word()}, y{word(), word(), word()};
    if ((nx() & 7) == 0) y = x;
    if ((nx() & 7) == 0) { y.w2 = x.w2; y.w1 = x.w1; }
    const hyg_u192 z = hyg_u192_add(x, y);
    const int ge = hyg_u192_ge(x, y);
    const hyg_u192 d = ge ? hyg_u192_sub(x, y) : hyg_u192_sub(y, x);
    printf("B %016llx %016llx %016llx %016llx %016llx %016llx %016llx %016llx %016llx %d %016llx %016llx %016llx\n",
           (unsigned long long)x.w0, (unsigned long long)x.w1, (unsigned long long)x.w2, (unsigned long long)y.w0,
           (unsigned long long)y.w1, (unsigned long long)y.w2, (unsigned long long)z.w0, (unsigned long long)z.w1,
           (unsigned long long)z.w2, ge, (unsigned long long)d.w0, (unsigned long long)d.w1,
           (unsigned long long)d.w2);
  }
  return 0;
}
"""


def _join(words):
    return sum(int(w, 16) << (64 * i) for i, w in enumerate(words))


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_carry_chain_forms_match_exact_integers(tmp_path):
    src = tmp_path / "carry.hip"
    exe = tmp_path / "carry"
    src.write_text(PROG)
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-I", os.path.join(REPO, "include"), "-o", str(exe), str(src)],
                   check=True, capture_output=True, timeout=300)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True, timeout=60).stdout.split("\n")
    n128 = n192 = 0
    for line in out:
        f = line.split()
        if not f:
            continue
        if f[0] == "A":
            a, b, s = _join(f[1:3]), _join(f[3:5]), _join(f[5:7])
            assert s == (a + b) % (1 << 128)
            assert int(f[7]) == int(a < b)
            n128 += 1
        else:
            x, y, z = _join(f[1:4]), _join(f[4:7]), _join(f[7:10])
            assert z == (x + y) % (1 << 192)
            assert int(f[10]) == int(x >= y)
            assert _join(f[11:14]) == abs(x - y)
            n192 += 1
    assert n128 == 4000 and n192 == 4000


PROG_LOW128 = r"""
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "hyg_arith.h"
static uint64_t st = 0x2545F4914F6CDD1Dull;
static uint64_t nx() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
static void show(uint32_t b) {
  float m;
  std::memcpy(&m, &b, 4);
  const hyg_u192 w = hyg_fix149f(m);
  const hyg_u128 n = hyg_fix149f_low128(m);
  printf("%08x %016llx %016llx %016llx %016llx %016llx\n", b, (unsigned long long)w.w0, (unsigned long long)w.w1,
         (unsigned long long)w.w2, (unsigned long long)n.lo, (unsigned long long)n.hi);
}
int main() {
  // every exponent below 2^-21 (E = 0 subnormals .. 105), incl. the word
  // boundary sh = E - 1 = 63 / 64, with edge significands
  for (uint32_t E = 0; E <= 105; ++E) {
    const uint32_t mans[4] = {0u, 1u, 0x7fffffu, (uint32_t)(nx() & 0x7fffffu)};
    for (int i = 0; i < 4; ++i) show((E << 23) | mans[i]);
  }
  for (int i = 0; i < 3000; ++i) show((uint32_t)(nx() % (106u << 23)));
  show(0x80000000u);  // -0 and negative masses image to 0
  show(0x80000001u);
  return 0;
}
"""


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_fix149f_low128_equals_fix149f_below_2_pow_minus_21(tmp_path):
    """the narrow u128 image of the top-set outside masses equals the
    low two words of hyg_fix149f (whose top word is 0) for every f32 m < 2^-21,
    subnormals and the sh = 63 / 64 word boundary included."""
    src = tmp_path / "low128.hip"
    exe = tmp_path / "low128"
    src.write_text(PROG_LOW128)
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-I", os.path.join(REPO, "include"), "-o", str(exe), str(src)],
                   check=True, capture_output=True, timeout=300)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True, timeout=60).stdout.split("\n")
    import struct
    n = 0
    for line in out:
        f = line.split()
        if not f:
            continue
        b = int(f[0], 16)
        w0, w1, w2, lo, hi = (int(x, 16) for x in f[1:])
        m = struct.unpack("<f", struct.pack("<I", b))[0]
        assert m < 2.0 ** -21
        exact = 0 if (b >> 31) else int(round(m * 2.0 ** 149)) if m > 0 else 0
        assert (w0 | (w1 << 64) | (w2 << 128)) == exact
        assert w2 == 0
        assert (lo, hi) == (w0, w1)
        n += 1
    assert n == 106 * 4 + 3000 + 2


PROG_EXPFIX = r"""
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "hyg_arith.h"
static uint64_t st = 0x9E3779B97F4A7C15ull;
static uint64_t nx() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
static int check(double x) {
  const hyg_u128 a = hyg_fix100(hyg_exp(x)), b = hyg_exp_fix100(x);
  if (a.lo != b.lo || a.hi != b.hi) {
    printf("MISMATCH %.17g %016llx %016llx %016llx %016llx\n", x, (unsigned long long)a.hi,
           (unsigned long long)a.lo, (unsigned long long)b.hi, (unsigned long long)b.lo);
    return 1;
  }
  return 0;
}
int main() {
  int bad = 0, n = 0;
  // uniform over the used range and beyond, dense near the cut points
  for (int i = 0; i < 400000; ++i, ++n) bad += check(-80.0 + 80.0 * (double)(nx() >> 11) * 0x1p-53);
  for (int i = 0; i < 100000; ++i, ++n) bad += check(-70.5 + 1.5 * (double)(nx() >> 11) * 0x1p-53);
  for (int i = 0; i < 100000; ++i, ++n) bad += check(-1e-3 * (double)(nx() >> 11) * 0x1p-53);
  // every reduction boundary k ln2 +- a few ulps
  for (int k = -102; k <= 1; ++k)
    for (int d = -4; d <= 4; ++d, ++n) {
      double x = (k + 0.5) * 0.69314718055994530942;
      uint64_t b; std::memcpy(&b, &x, 8); b += d; std::memcpy(&x, &b, 8);
      bad += check(x);
    }
  const double sp[] = {0.0, -0.0, -70.0, -69.3147, -1e-300, -HUGE_VAL, NAN, 5.0, 10.9};
  for (double x : sp) { bad += check(x); ++n; }
  printf("N %d BAD %d\n", n, bad);
  return bad != 0;
}
"""


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_exp_fix100_shift_form_equals_float_form(tmp_path):
    """hyg_exp_fix100 (the kernels' shift-based image) is hyg_fix100(hyg_exp(x))
    (the oracle's form) integer for integer on and around [-70, 0]."""
    src = tmp_path / "expfix.hip"
    exe = tmp_path / "expfix"
    src.write_text(PROG_EXPFIX)
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(REPO, "include"), "-o",
                    str(exe), str(src)], check=True, capture_output=True, timeout=300)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout[-2000:]
    assert "BAD 0" in out.stdout


PROG_CEILMUL = r"""
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "hyg_arith.h"
static uint64_t st = 0x2545F4914F6CDD1Dull;
static uint64_t nx() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
int main() {
  int bad = 0, n = 0;
  for (int i = 0; i < 300000; ++i, ++n) {
    float T;
    const int kind = (int)(nx() & 3);
    if (kind == 0) {  // the systematic targets ((j + U) / L in f32)
      const int L = 1 + (int)(nx() % 64), j = (int)(nx() % (uint64_t)L);
      const float U = (float)(nx() >> 40) * 0x1p-24f;
      T = ((float)j + U) / (float)L;
    } else if (kind == 1) {  // any float in [0, 1]
      uint32_t b = (uint32_t)(nx() % 0x3f800001u);
      std::memcpy(&T, &b, 4);
    } else if (kind == 2) {  // subnormals and tiny values
      uint32_t b = (uint32_t)(nx() % 0x01000000u);
      std::memcpy(&T, &b, 4);
    } else {
      T = (nx() & 1) ? 1.0f : 0.0f;
    }
    hyg_u192 R{nx(), nx(), nx() & ((1ull << (nx() % 24)) - 1)};  // R < 2^151
    if (nx() & 1) R.w2 = 0;
    if ((nx() & 7) == 0) R.w1 = 0;
    const hyg_u192 a = hyg_ceil_mul_f32(T, R), b = hyg_ceil_mul_f32_bf(T, R);
    if (a.w0 != b.w0 || a.w1 != b.w1 || a.w2 != b.w2) {
      if (bad < 5) printf("MISMATCH T=%a\\n", (double)T);
      ++bad;
    }
  }
  printf("N %d BAD %d\\n", n, bad);
  return bad != 0;
}
"""


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_ceil_mul_branch_free_equals_branch_form(tmp_path):
    """The kernels' branch-free exact systematic threshold (hyg_ceil_mul_f32_bf)
    is the oracle's hyg_ceil_mul_f32, integer for integer."""
    src = tmp_path / "ceilmul.hip"
    exe = tmp_path / "ceilmul"
    src.write_text(PROG_CEILMUL)
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(REPO, "include"), "-o",
                    str(exe), str(src)], check=True, capture_output=True, timeout=300)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout[-2000:]
    assert "BAD 0" in out.stdout
