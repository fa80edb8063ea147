"""Bounds-checked run of the chunked small-N stencil (variant libsehip_stcdbg.so, built
with -DSE_STC_DEBUG=1: every index clamped into its buffer, violations counted per
kind: 0 x loads, 1 LDS writes, 2 LDS reads, 3 weights, 4 partials, 5 outputs).
  SEHIP_LIB=.../libsehip_stcdbg.so python tools/stencil_debug.py"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, ROOT)
import torch
from sehip import functional as F, _native as N
import paramfill
from oracle import complex_nn as O_cnn

lib = ctypes.CDLL(N.LIB_PATH)
counts = (ctypes.c_int * 8)()
for shape, kernel, stride, padding in [((2, 40, 9, 17), (3, 3), (1, 1), (1, 1)),
                                       ((2, 128, 33, 63), (7, 5), (2, 2), (3, 2)),
                                       ((1, 96, 20, 70), (5, 3), (2, 1), (2, 1))]:
    m = paramfill.fill_(O_cnn.ComplexConvTranspose2d(shape[1], 2, kernel, stride=stride, padding=padding), seed=5)
    x = torch.randn(*shape)
    with torch.no_grad():
        ref = m.double()(x.double())
        y = F.conv2d(x.cuda(), m.real_conv.weight.float().cuda(), m.imag_conv.weight.float().cuda(),
                     m.real_conv.bias.float().cuda(), m.imag_conv.bias.float().cuda(), out_channels=2,
                     kernel=kernel, stride=stride, padding=padding, transposed=True)
    torch.cuda.synchronize()
    lib.se_debug_stencil_counts(counts)
    err = ((y.double().cpu() - ref).norm() / ref.norm()).item()
    print(shape, kernel, stride, "violations", list(counts), "rel err", f"{err:.2e}", flush=True)
