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
    os.path.join(CSRC, "jser_flat.h"),
    os.path.join(CSRC, "handoff.h"),
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


def _compile_cmd(src: str, obj: str) -> list:
    return [
        hipcc(),
        "-x", "hip",
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


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile every source whose object is older than it or any header (all of them with
    force), in parallel, then link."""
    if not force and not needs_build():
        return LIB
    hdr_t = max(os.path.getmtime(h) for h in HEADERS)
    objs, procs = [], []
    for src in SOURCES:
        obj = os.path.join(CSRC, os.path.basename(src) + ".o")
        objs.append(obj)
        if not force and os.path.exists(obj) and os.path.getmtime(obj) > max(hdr_t, os.path.getmtime(src)):
            continue
        cmd = _compile_cmd(src, obj)
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((src, subprocess.Popen(cmd)))
    bad = [src for src, p in procs if p.wait() != 0]
    if bad:
        raise RuntimeError(f"hipcc failed for {bad}")
    link = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs
    if verbose:
        print(" ".join(link), flush=True)
    subprocess.run(link, check=True)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
