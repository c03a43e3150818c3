"""Builds hygeia_amd/lib/libhygeia_amd.so for gfx950 with hipcc (in-tree).

Flags that are part of the arithmetic contract (include/hyg_arith.h):
  -ffp-contract=off                        no FMA contraction (host and device)
  -fno-gpu-flush-denormals-to-zero         IEEE f32 subnormals on the device
  -fhip-fp32-correctly-rounded-divide-sqrt correctly rounded f32 division
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libhygeia_amd.so")
SOURCES = [os.path.join(HERE, "csrc", f) for f in ("capi.cpp", "tg_kernels.hip", "sg_kernels.hip", "dmp_kernels.hip")]
DEPS = SOURCES + [os.path.join(HERE, "csrc", f) for f in ("tg_common.h", "sg_common.h", "dmp_common.h", "hyg_dev.h")] + [
    os.path.join(ROOT, "include", f) for f in ("hygeia_amd.h", "hyg_arith.h", "hyg_model.h", "hyg_sg_model.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-ffp-contract=off",
         "-fno-gpu-flush-denormals-to-zero", "-fhip-fp32-correctly-rounded-divide-sqrt",
         "-Wall", "-Wno-unused-function"]


def stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not stale():
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = [HIPCC] + FLAGS + ["-o", tmp] + SOURCES
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
