"""Developer probe (run explicitly after other test files): can torch still initialise HIP?"""
import ctypes

import pytest


@pytest.mark.gpu
def test_probe_torch():
    import os
    import resource
    fds = os.listdir("/proc/self/fd")
    kinds = {}
    for f in fds:
        try:
            t = os.readlink(f"/proc/self/fd/{f}")
        except OSError:
            continue
        k = t.split(":")[0] if ":" in t else os.path.dirname(t)
        kinds[k] = kinds.get(k, 0) + 1
    print("open fds", len(fds), "limit", resource.getrlimit(resource.RLIMIT_NOFILE), sorted(kinds.items(), key=lambda x: -x[1])[:8],
          flush=True)
    hip = ctypes.CDLL("libamdhip64.so")
    c = ctypes.c_int()
    r = hip.hipGetDeviceCount(ctypes.byref(c))
    import torch
    print("hipGetDeviceCount", r, c.value, "raw", torch._C._cuda_getDeviceCount(), flush=True)
    torch.empty(4, device="cuda")
