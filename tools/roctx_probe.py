"""Probe of rocprofv3's roctx handling on the box: a named range around ten kernels
(roctxRangePushA / roctxRangePop), for --marker-trace."""
import ctypes

import torch

lib = ctypes.CDLL("/opt/rocm/lib/librocprofiler-sdk-roctx.so")
lib.roctxRangePushA.argtypes, lib.roctxRangePushA.restype = [ctypes.c_char_p], ctypes.c_int
lib.roctxRangePop.argtypes, lib.roctxRangePop.restype = [], ctypes.c_int
x = torch.randn(1000, device="cuda")
y = x * 2
torch.cuda.synchronize()
print("push", lib.roctxRangePushA(b"timed"), flush=True)
for _ in range(10):
    y = torch.sin(y)
torch.cuda.synchronize()
print("pop", lib.roctxRangePop(), flush=True)
y = torch.cos(y)
torch.cuda.synchronize()
