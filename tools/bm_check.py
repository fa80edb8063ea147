"""Writes the outputs of the f16x3 data-grad / forward passes at dec5 and joined
decoder shapes to a file, so two processes with different SEHIP_GEMM_BM can be
compared for bit-identity (tools/gpu_bm.sh)."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
from sehip import functional as F

out = {}
dev = torch.device("cuda")
torch.manual_seed(0)
# dec5-like transposed conv 256 -> 128 at B = 8 (data-grad has N = 256 outputs)
x = torch.randn(8, 256, 158, 403, device=dev)
w = torch.randn(128, 64, 5, 2, device=dev) * 0.05
wi = torch.randn(128, 64, 5, 2, device=dev) * 0.05
d = F.conv_desc(tuple(x.shape), 128, (5, 2), (2, 1), (0, 0), (1, 1), (0, 0), True, True)
d.math = F._MATH_CODES["f16x3"]
lib = F.N.lib()
ho, wo = F.N.c_int(), F.N.c_int()
lib.se_conv2d_out_shape(F.N.ctypes.byref(d), F.N.ctypes.byref(ho), F.N.ctypes.byref(wo))
dy = torch.randn(8, 128, ho.value, wo.value, device=dev)
dx = torch.empty_like(x)
ws = torch.empty(lib.se_conv2d_workspace_size(F.N.ctypes.byref(d)), dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream().cuda_stream
assert lib.se_conv2d_bwd_data(F.N.ctypes.byref(d), dy.data_ptr(), w.data_ptr(), wi.data_ptr(), dx.data_ptr(),
                              ws.data_ptr(), ws.numel(), st) == 0
torch.cuda.synchronize()
out["dec5_data"] = dx.cpu()
torch.save(out, sys.argv[1])
print("saved", sys.argv[1], {k: float(v.abs().sum()) for k, v in out.items()})
