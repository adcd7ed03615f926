"""Developer check: does torch's HIP init still see the GPU after many engines were
created and destroyed in the same process?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes  # noqa: E402

from clonos_amd import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 80
for i in range(n):
    e = Engine(segment_bytes=256, pool_segments=1 << 16, timing=True)
    e.close()
hip = ctypes.CDLL("libamdhip64.so")
c = ctypes.c_int()
print("hipGetDeviceCount", hip.hipGetDeviceCount(ctypes.byref(c)), c.value, flush=True)
import torch  # noqa: E402
print("torch device_count", torch.cuda.device_count(), flush=True)
x = torch.empty(10, device="cuda")
print("ok", x.device, flush=True)
