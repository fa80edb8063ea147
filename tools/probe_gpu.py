"""Round-1 de-risking probe: does a hipcc-built C-ABI .so loaded via ctypes
share torch's HIP runtime (pointers + streams)?"""
import ctypes, os, sys, time
import torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "..", "speech-enhancement_amd", "sehip", "libsehip.so"))
lib.se_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
print("cuda avail", torch.cuda.is_available(), torch.cuda.get_device_name(0))
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    out = torch.zeros(100000, dtype=torch.int32, device="cuda")
    rc = lib.se_probe(out.data_ptr(), out.numel(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
ref = torch.arange(100000, dtype=torch.int32, device="cuda") * 3 + 1
print("rc", rc, "ok", bool((out == ref).all()))
with open("/proc/self/maps") as f:
    libs = sorted({l.split()[-1] for l in f if "amdhip" in l or "sehip" in l})
print("\n".join(libs))
