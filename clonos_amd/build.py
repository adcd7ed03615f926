"""Build libclonos_engine.so (gfx950) in-tree with hipcc.

The shared library is the product: the C-ABI in include/clonos_engine.h plus the HIP
kernels.  It is built in-tree so that it travels with the repository snapshot to the GPU
box (git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libclonos_engine.so")
SOURCES = [os.path.join(CSRC, "engine.cpp"), os.path.join(CSRC, "kernels.hip"), os.path.join(CSRC, "decode_fast.hip"),
           os.path.join(CSRC, "decode_fused.hip"), os.path.join(CSRC, "replay.hip"), os.path.join(CSRC, "encode.hip"),
           os.path.join(CSRC, "response.cpp")]
HEADERS = [
    os.path.join(CSRC, "kernels.h"),
    os.path.join(CSRC, "jser_device.h"),
    os.path.join(CSRC, "dev_common.h"),
    os.path.join(CSRC, "dev_slow.h"),
    os.path.join(ROOT, "include", "clonos_engine.h"),
]
ARCH = os.environ.get("CLONOS_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    return "hipcc"


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return LIB
    objs = []
    for src in SOURCES:
        obj = os.path.join(CSRC, os.path.basename(src) + ".o")
        cmd = [
            hipcc(),
            "-x", "hip" if src.endswith(".hip") else "hip",
            f"--offload-arch={ARCH}",
            "-O3",
            "-std=c++17",
            "-fPIC",
            "-Wall",
            "-Wno-unused-function",
            "-Wno-unused-value",
            "-I", os.path.join(ROOT, "include"),
            "-c", src,
            "-o", obj,
        ]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    link = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs
    if verbose:
        print(" ".join(link), flush=True)
    subprocess.run(link, check=True)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
