"""Operands whose address has a low 32-bit word >= 2^31.

The GEMMs build their buffer-resource bases from readfirstlane'd pointer words
(se::uniform_ptr, csrc/common.hpp). Before d630867 the chunked stencil widened the
signed low word directly, so any operand whose low address word was >= 2^31 got a base
with 0xffffffff in its high word: an illegal-address fault that appeared only when the
allocator happened to return such an address. Here every operand of each pass is
carved out of one 6 GB buffer inside a 2 GB window whose low address words are all
>= 2^31 (such a window always exists in 6 GB), so the case is hit deterministically:
- the chunked LDS stencil (gather_stencil_ch_kernel: DCUNet's final 128 -> 2 convT,
  _1903_03107_dcunet.py:80-83),
- the tap-uniform split-fp16 gather GEMMs (forward and data-grad, gather_x3_kernel) and
- the split-fp16 weight-grad (wgrad_x3_kernel)
of FRCRN encoder / decoder layer shapes. Each result must be bit-identical to the
same pass on allocator-placed operands, and within fp32 rounding of fp64.
tests/test_uniform_ptr_cpu.py checks the word join itself on the host."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

LAYERS = [   # (transposed, cin, cout, (B, h, w), pad, kernel, stride, env)
    (False, 128, 128, (2, 40, 41), (0, 0), (5, 2), (2, 1), {}),          # FRCRN enc: TU gather + wgrad
    (True, 256, 128, (2, 17, 40), (0, 0), (5, 2), (2, 1), {}),           # FRCRN dec: 256-column data-grad
    (True, 128, 2, (2, 33, 63), (3, 2), (7, 5), (2, 2), {"SEHIP_STENCIL": "1"}),   # DCUNet final: stencil
]


class _HighWindow:
    """A 6 GB device buffer and a bump allocator over its 2 GB window of addresses
    whose low 32-bit word is >= 2^31."""

    def __init__(self, dev):
        self.buf = torch.empty(6 << 30, dtype=torch.uint8, device=dev)
        b = self.buf.data_ptr()
        w = (b + (1 << 32) - 1) >> 32 << 32          # next 4 GB boundary
        start = w - (1 << 31) if w - b >= (1 << 31) else w + (1 << 31)
        self.cur, self.end = start - b, start - b + (1 << 31)

    def take(self, shape):
        n = 1
        for s in shape:
            n *= s
        off = self.cur
        self.cur = (off + 4 * n + 255) // 256 * 256
        assert self.cur <= self.end
        t = self.buf[off:off + 4 * n].view(torch.float32).view(shape)
        assert (t.data_ptr() & 0xFFFFFFFF) >= (1 << 31)
        return t


@pytest.mark.parametrize("layer", LAYERS, ids=["enc", "dec", "stencil"])
def test_passes_on_high_low_word_addresses(layer, gpu_device, monkeypatch):
    from sehip import functional as F, _native as N
    tr, cin, cout, (B, h, w), pad, k, s, env = layer
    for key, v in env.items():
        monkeypatch.setenv(key, v)
    lib = N.lib()
    d = F.conv_desc((B, cin, h, w), cout, k, s, pad, (1, 1), (0, 0), tr, True)
    d.math = F._MATH_CODES["f16x3"]
    ho, wo = ctypes.c_int(), ctypes.c_int()
    assert lib.se_conv2d_out_shape(ctypes.byref(d), ctypes.byref(ho), ctypes.byref(wo)) == 0
    xs, ys = (B, cin, h, w), (B, cout, ho.value, wo.value)
    wsh = (cin // 2, cout // 2, *k) if tr else (cout // 2, cin // 2, *k)
    g = torch.Generator(device=gpu_device).manual_seed(3)
    src = {"x": torch.randn(xs, device=gpu_device, generator=g),
           "dy": torch.randn(ys, device=gpu_device, generator=g),
           "wr": torch.randn(wsh, device=gpu_device, generator=g) * .05,
           "wi": torch.randn(wsh, device=gpu_device, generator=g) * .05}
    shapes = {"y": ys, "dx": xs, "dwr": wsh, "dwi": wsh}
    nws = lib.se_conv2d_workspace_size(ctypes.byref(d))

    def run(alloc, ws):
        t = {n: alloc(v.shape) for n, v in src.items()}
        for n, v in src.items():
            t[n].copy_(v)
        o = {n: alloc(sh) for n, sh in shapes.items()}
        b, st = ctypes.byref(d), N.stream_of(t["x"])
        rc = [lib.se_conv2d_fwd(b, t["x"].data_ptr(), t["wr"].data_ptr(), t["wi"].data_ptr(), None, None,
                                o["y"].data_ptr(), ws.data_ptr(), nws, st),
              lib.se_conv2d_bwd_data(b, t["dy"].data_ptr(), t["wr"].data_ptr(), t["wi"].data_ptr(),
                                     o["dx"].data_ptr(), ws.data_ptr(), nws, st),
              lib.se_conv2d_bwd_weight(b, t["x"].data_ptr(), t["dy"].data_ptr(), o["dwr"].data_ptr(),
                                       o["dwi"].data_ptr(), None, None, ws.data_ptr(), nws, st)]
        torch.cuda.synchronize()
        assert rc == [0, 0, 0], rc
        return {n: v.clone() for n, v in o.items()}

    low = run(lambda sh: torch.empty(sh, device=gpu_device),
              torch.empty(nws, dtype=torch.uint8, device=gpu_device))
    hw = _HighWindow(gpu_device)
    ws_hi = hw.take(((nws + 3) // 4,))
    assert (ws_hi.data_ptr() & 0xFFFFFFFF) >= (1 << 31)
    high = run(hw.take, ws_hi)
    del hw
    for n in shapes:
        assert torch.equal(low[n], high[n]), f"{n}: result depends on the operand address"
    # and against fp64 (torch's CPU convs on the block weight, as the oracle composes them)
    from oracle import complex_nn as O
    cls = O.ComplexConvTranspose2d if tr else O.ComplexConv2d
    m = cls(cin, cout, k, stride=s, padding=pad, bias=False).double()
    with torch.no_grad():
        m.real_conv.weight.copy_(src["wr"].double().cpu())
        m.imag_conv.weight.copy_(src["wi"].double().cpu())
    x64 = src["x"].double().cpu().requires_grad_(True)
    y64 = m(x64)
    y64.backward(src["dy"].double().cpu())
    ref = {"y": y64.detach(), "dx": x64.grad, "dwr": m.real_conv.weight.grad, "dwi": m.imag_conv.weight.grad}
    for n, r in ref.items():
        e = ((high[n].double().cpu() - r).norm() / r.norm()).item()
        assert e < 2e-6, (n, e)
