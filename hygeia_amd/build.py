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
SOURCES = [os.path.join(HERE, "csrc", f) for f in ("capi.cpp", "tg_kernels.hip", "sg_kernels.hip", "dmp_kernels.hip", "bed_kernels.hip", "pre_kernels.hip")]
DEPS = SOURCES + [os.path.join(HERE, "csrc", f) for f in ("tg_common.h", "sg_common.h", "dmp_common.h", "hyg_dev.h")] + [
    os.path.join(ROOT, "include", f) for f in ("hygeia_amd.h", "hyg_arith.h", "hyg_model.h", "hyg_sg_model.h", "hyg_sg_pe.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-ffp-contract=off",
         "-fno-gpu-flush-denormals-to-zero", "-fhip-fp32-correctly-rounded-divide-sqrt",
         "-Wall", "-Wno-unused-function"]


def source_hash() -> str:
    """Digest of every file compiled into the library plus the flags: tags
    measurements (profiles/pmc_*.json) with the kernel build they were taken on."""
    import hashlib

    h = hashlib.sha256(" ".join(FLAGS).encode())
    for d in sorted(DEPS):
        h.update(os.path.relpath(d, ROOT).encode())
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force: bool = False, verbose: bool = False) -> str:
    """Compiles the translation units in parallel (one hipcc each, objects
    under lib/obj) and links the shared library."""
    if not force and not stale():
        return LIB
    from concurrent.futures import ThreadPoolExecutor

    obj_dir = os.path.join(LIB_DIR, "obj")
    os.makedirs(obj_dir, exist_ok=True)
    cflags = [f for f in FLAGS if f != "-shared"]
    objs, cmds = [], []
    headers = [d for d in DEPS if d not in SOURCES]
    newest_header = max(os.path.getmtime(h) for h in headers)
    for src in SOURCES:
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        objs.append(obj)
        fresh = (not force and os.path.exists(obj) and
                 os.path.getmtime(obj) > max(os.path.getmtime(src), newest_header))
        if not fresh:
            cmds.append([HIPCC] + cflags + ["-c", src, "-o", obj])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    with ThreadPoolExecutor(max_workers=max(1, min(len(cmds), 8))) as ex:
        for f in [ex.submit(run, c) for c in cmds]:
            f.result()
    tmp = LIB + ".tmp"
    link = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp] + objs
    run(link)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
