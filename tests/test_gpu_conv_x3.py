"""GPU parity of the split conv GEMMs against the fp64 oracle
(complex_nn.py:52-91 in the reference's four-real-conv form) at FRCRN layer
geometries and the golden conv cases, every pass (y, dx, dwr, dwi):

* "f32" (math 0, v_mfma_f32_32x32x2_f32): the exact-fp32 path, pinned
  absolutely at rel-L2 < 1e-5.
* "f16x3" (math 4, scaled split-fp16, three terms): fp32-class — at or below
  1.25x the exact-fp32 path's own error (and < 1e-5), and scale-invariant
  (inputs scaled by 2^-40 .. 2^30 keep that error).
* "bf16x6" (math 2, three-way split bf16, six terms; gather passes): within 3x
  of the exact-fp32 path.
* "bf16x3" (math 1): drops lo*lo and rounds lo to bf16, <= ~2^-15 relative per
  product, ~6e-6 rms: rel-L2 < 3e-5 and within 30x of the exact-fp32 path."""
import pytest
import torch

from conftest import golden, rel_l2
import paramfill
from oracle import complex_nn as O_cnn

pytestmark = pytest.mark.gpu

TOL = 3e-5

LAYERS = [
    ("enc1", False, 128, 128, (2, 128, 158, 41), (2, 1)),
    ("enc5", False, 128, 128, (2, 128, 7, 41), (2, 1)),
    ("dec0", True, 256, 128, (2, 256, 2, 40), (2, 1)),
    ("dec5", True, 256, 128, (2, 256, 158, 40), (2, 1)),
    ("dec_odd", True, 256, 192, (3, 256, 9, 37), (2, 1)),   # N = 192: partial n-tile
    ("s22", False, 128, 256, (2, 128, 33, 29), (2, 2)),     # two n-tiles, stride 2 in time
]


def _hip(F, m, x, gy, transposed, stride, math):
    prev = F.get_conv_math()
    F.set_conv_math(math)
    try:
        wr = m.real_conv.weight.detach().float().cuda().requires_grad_(True)
        wi = m.imag_conv.weight.detach().float().cuda().requires_grad_(True)
        xg = x.float().cuda().requires_grad_(True)
        y = F.conv2d(xg, wr, wi, out_channels=2 * m.real_conv.out_channels,
                     kernel=m.real_conv.kernel_size, stride=stride, transposed=transposed)
        y.backward(gy.float().cuda())
        torch.cuda.synchronize()
        return dict(y=y.detach().cpu(), dx=xg.grad.cpu(), dwr=wr.grad.cpu(), dwi=wi.grad.cpu())
    finally:
        F.set_conv_math(prev)


def _fp64_ref(name, tr, cin, cout, shape, stride, x_scale=1.0, gy_scale=1.0):
    cls = O_cnn.ComplexConvTranspose2d if tr else O_cnn.ComplexConv2d
    m = paramfill.fill_(cls(cin, cout, (5, 2), stride=stride, bias=False), seed=7).double()
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(*shape, generator=gen, dtype=torch.float64) * x_scale
    xo = x.clone().requires_grad_(True)
    yo = m(xo)
    gy = torch.randn(yo.shape, generator=gen, dtype=torch.float64) * gy_scale
    yo.backward(gy)
    ref = dict(y=yo.detach(), dx=xo.grad, dwr=m.real_conv.weight.grad, dwi=m.imag_conv.weight.grad)
    return m, x, gy, ref


F16_VS_F32 = 1.25   # f16x3 error may exceed the exact-fp32 path's by at most 25 %


@pytest.mark.parametrize("name,tr,cin,cout,shape,stride", LAYERS)
def test_split_layer_vs_fp64_oracle(name, tr, cin, cout, shape, stride, gpu_device):
    from sehip import functional as F
    m, x, gy, ref = _fp64_ref(name, tr, cin, cout, shape, stride)
    exact = _hip(F, m, x, gy, tr, stride, "f32")
    split = _hip(F, m, x, gy, tr, stride, "bf16x3")
    split6 = _hip(F, m, x, gy, tr, stride, "fwd=bf16x6,data=bf16x6,weight=f32")
    f16 = _hip(F, m, x, gy, tr, stride, "f16x3")
    for k, r in ref.items():
        e32 = rel_l2(exact[k].numpy(), r.numpy())
        ex3 = rel_l2(split[k].numpy(), r.numpy())
        ex6 = rel_l2(split6[k].numpy(), r.numpy())
        e16 = rel_l2(f16[k].numpy(), r.numpy())
        print(f"{name} {k}: f32 {e32:.2e}  f16x3 {e16:.2e}  bf16x6 {ex6:.2e}  bf16x3 {ex3:.2e}")
        assert e32 < 1e-5, (name, k, e32)                       # the exact-fp32 path, absolutely
        assert e16 < 1e-5 and e16 <= max(F16_VS_F32 * e32, 1e-7), (name, k, e16, e32)
        assert ex3 < TOL, (name, k, ex3)
        assert ex3 < max(30 * e32, 1e-6), (name, k, ex3, e32)
        # three-way split: fp32-class (within 3x of the exact-fp32 MFMA path)
        assert ex6 < max(3 * e32, 1e-6), (name, k, ex6, e32)


@pytest.mark.parametrize("x_scale,gy_scale", [(2.0 ** -40, 2.0 ** -30), (2.0 ** 30, 2.0 ** 20),
                                              (1.0, 2.0 ** -60)])
@pytest.mark.parametrize("name,tr,cin,cout,shape,stride", [LAYERS[1], LAYERS[3]])
def test_f16x3_is_scale_invariant(name, tr, cin, cout, shape, stride, x_scale, gy_scale, gpu_device):
    """The per-tensor power-of-two scales keep fp16's exponent range out of the
    result: activations and gradients of any magnitude (SI-SNR gradients reach
    1e-9 and below) keep the fp32-class error."""
    from sehip import functional as F
    m, x, gy, ref = _fp64_ref(name, tr, cin, cout, shape, stride, x_scale, gy_scale)
    exact = _hip(F, m, x, gy, tr, stride, "f32")
    f16 = _hip(F, m, x, gy, tr, stride, "f16x3")
    for k, r in ref.items():
        e32 = rel_l2(exact[k].numpy(), r.numpy())
        e16 = rel_l2(f16[k].numpy(), r.numpy())
        print(f"{name} x*{x_scale:.1e} gy*{gy_scale:.1e} {k}: f32 {e32:.2e}  f16x3 {e16:.2e}")
        assert e16 < 1e-5 and e16 <= max(F16_VS_F32 * e32, 1e-7), (name, k, e16, e32)


BF16_TOL = 1e-2   # one bf16 rounding per operand: ~2^-9 relative, rms ~3e-3 on random data


@pytest.mark.parametrize("name,tr,cin,cout,shape,stride", LAYERS[:4])
def test_bf16_layer_vs_fp64_oracle(name, tr, cin, cout, shape, stride, gpu_device):
    """SE_MATH_BF16 (one MFMA term, operands rounded to bf16, fp32 accumulate):
    every pass within bf16 rounding of fp64, and measurably coarser than
    bf16x3 (so the one-term kernels really ran)."""
    from sehip import functional as F
    cls = O_cnn.ComplexConvTranspose2d if tr else O_cnn.ComplexConv2d
    m = paramfill.fill_(cls(cin, cout, (5, 2), stride=stride, bias=False), seed=7).double()
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(*shape, generator=gen, dtype=torch.float64)
    xo = x.clone().requires_grad_(True)
    yo = m(xo)
    gy = torch.randn(yo.shape, generator=gen, dtype=torch.float64)
    yo.backward(gy)
    ref = dict(y=yo.detach(), dx=xo.grad, dwr=m.real_conv.weight.grad, dwi=m.imag_conv.weight.grad)
    b1 = _hip(F, m, x, gy, tr, stride, "bf16")
    for k, r in ref.items():
        e = rel_l2(b1[k].numpy(), r.numpy())
        print(f"{name} {k}: bf16 {e:.2e}")
        assert 1e-4 < e < BF16_TOL, (name, k, e)


CONV_CASES = [
    ("enc", False, 16, 12, (5, 2), dict(stride=(2, 1), bias=False)),
    ("dec", True, 16, 12, (5, 2), dict(stride=(2, 1), bias=False)),
]


@pytest.mark.parametrize("i,case", [(0, CONV_CASES[0]), (3, CONV_CASES[1])])
def test_bf16x3_small_channels_match_golden(i, case, gpu_device):
    """Shapes outside the split kernels' tiles (N <= 64) run the fp32 GEMM in
    bf16x3 mode too: same goldens, same 1e-5 bar as test_gpu_cconv."""
    from sehip import functional as F
    g = golden("cconv")
    name, tr, cin, cout, k, kw = case
    cls = O_cnn.ComplexConvTranspose2d if tr else O_cnn.ComplexConv2d
    m = paramfill.fill_(cls(cin, cout, k, **kw), seed=i)
    r = _hip(F, m, torch.from_numpy(g[f"{name}_x"]), torch.from_numpy(g[f"{name}_gy"]), tr,
             kw["stride"], "bf16x3")
    for key in ("y", "dx", "dwr", "dwi"):
        assert rel_l2(r[key].numpy(), g[f"{name}_{key}"]) < 1e-5, (name, key)


@pytest.mark.parametrize("n,off,complex_w", [(81920, 0, True), (81920, 0, False), (40963, 0, True),
                                             (40960, 1, True), (7, 0, True), (1 << 20, 0, True)])
def test_amax_weights_exact(n, off, complex_w):
    """se_amax_weights (the f16x3 weight scale source): max |wr|, |wi| exactly,
    on the 16-B vector path, ragged tails and unaligned pointers."""
    from sehip import _native as N
    g = torch.Generator().manual_seed(n + off)
    wr = (torch.randn(n + off, generator=g) * 3).cuda()[off:]
    wi = (torch.randn(n + off, generator=g) * 5).cuda()[off:] if complex_w else None
    wr[n // 2] = -17.5   # the maximum magnitude, negative
    out = torch.full((1,), -1.0, device="cuda")
    N.check(N.lib().se_amax_weights(wr.data_ptr(), n, N.ptr(wi), out.data_ptr(), N.stream_of(wr)),
            "se_amax_weights")
    ref = wr.abs().max() if wi is None else torch.maximum(wr.abs().max(), wi.abs().max())
    assert out.item() == ref.item()

CONV16_CASES = LAYERS[:4] + [
    ("n32", False, 32, 64, (2, 32, 65, 37), (2, 1)),     # DCCRN enc1-like: 32 -> 64 channels (128-col tiles)
    ("t64", True, 128, 64, (2, 128, 17, 30), (2, 1)),    # convT 128 -> 64 (DCCRN decoder-like)
    ("n16", False, 64, 16, (2, 64, 33, 21), (1, 1)),     # N = 16: the small-N gather, 16-wide weight-grad tile
]


@pytest.mark.parametrize("dtype,tol", [(torch.bfloat16, 6e-3), (torch.float16, 1e-3)])
@pytest.mark.parametrize("name,tr,cin,cout,shape,stride", CONV16_CASES)
def test_conv_16bit_storage(name, tr, cin, cout, shape, stride, dtype, tol, gpu_device, monkeypatch):
    """bf16 / fp16 storage (model.to(bfloat16) / .half(); BASELINE configs 2 / 3 / 5): every
    pass reads and writes the 16-bit tensors directly (se_conv2d_desc.dtype) with the
    one-term MFMA of that format, whose products of the 16-bit operands are exact. So each
    result equals, bit for bit, the same one-term arithmetic on fp32 copies rounded once
    at the end (SEHIP_NATIVE16=0), and is within the 16-bit output rounding of fp64."""
    from sehip import functional as F
    cls = O_cnn.ComplexConvTranspose2d if tr else O_cnn.ComplexConv2d
    m = paramfill.fill_(cls(cin, cout, (5, 2), stride=stride, bias=False), seed=7)
    gen = torch.Generator().manual_seed(13)
    x = torch.randn(*shape, generator=gen).to(dtype)
    wr16, wi16 = m.real_conv.weight.detach().to(dtype), m.imag_conv.weight.detach().to(dtype)
    md = m.double()
    with torch.no_grad():
        md.real_conv.weight.copy_(wr16.double()); md.imag_conv.weight.copy_(wi16.double())
    xo = x.double().requires_grad_(True)
    yo = md(xo)
    gy = torch.randn(yo.shape, generator=gen).to(dtype)
    yo.backward(gy.double())
    ref = dict(y=yo.detach(), dx=xo.grad, dwr=md.real_conv.weight.grad, dwi=md.imag_conv.weight.grad)

    def run(native):
        monkeypatch.setenv("SEHIP_NATIVE16", "1" if native else "0")
        wr = wr16.cuda().requires_grad_(True)
        wi = wi16.cuda().requires_grad_(True)
        xg = x.cuda().requires_grad_(True)
        before = F.NATIVE16_CALLS[0]
        y = F.conv2d(xg, wr, wi, out_channels=2 * m.real_conv.out_channels, kernel=(5, 2), stride=stride,
                     transposed=tr)
        assert (F.NATIVE16_CALLS[0] - before) == (1 if native else 0)
        y.backward(gy.cuda())
        torch.cuda.synchronize()
        assert y.dtype == dtype and xg.grad.dtype == dtype and wr.grad.dtype == dtype
        return dict(y=y.detach().cpu(), dx=xg.grad.cpu(), dwr=wr.grad.cpu(), dwi=wi.grad.cpu())

    nat, cast = run(True), run(False)
    for k, r in ref.items():
        e = rel_l2(nat[k].float().numpy(), r.numpy())
        print(f"{name} {dtype} {k}: native vs fp64 {e:.2e}, bit-identical to the cast path: "
              f"{torch.equal(nat[k], cast[k])}")
        assert torch.equal(nat[k], cast[k]), (name, k)
        assert e < tol, (name, k, e)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,kernel,stride,padding",
                         [((2, 128, 33, 63), (7, 5), (2, 2), (3, 2)),    # DCUNet-16's final convT
                          ((1, 96, 20, 70), (5, 3), (2, 1), (2, 1)),     # 3 row taps, ragged tiles
                          ((2, 40, 9, 17), (3, 3), (1, 1), (1, 1))])     # stride 1, 5 channel chunks
def test_many_channel_small_n_stencil(shape, kernel, stride, padding, dtype, gpu_device, monkeypatch):
    """Small-N transposed convs over many channels (DCUNet's final 128 -> 2 layer,
    _1903_03107_dcunet.py:80-83) run the chunked LDS stencil (gather_stencil_ch_kernel):
    within fp32 summation-order rounding of the per-output gather (SEHIP_STENCIL=0), and
    of fp64; 16-bit storage read and written natively."""
    from sehip import functional as F
    m = paramfill.fill_(O_cnn.ComplexConvTranspose2d(shape[1], 2, kernel, stride=stride, padding=padding),
                        seed=5)
    gen = torch.Generator().manual_seed(17)
    x = torch.randn(*shape, generator=gen).to(dtype)
    md = m.double()
    wr16, wi16 = m.real_conv.weight.detach().to(dtype), m.imag_conv.weight.detach().to(dtype)
    br, bi = m.real_conv.bias.detach().to(dtype), m.imag_conv.bias.detach().to(dtype)
    with torch.no_grad():
        md.real_conv.weight.copy_(wr16.double()); md.imag_conv.weight.copy_(wi16.double())
        md.real_conv.bias.copy_(br.double()); md.imag_conv.bias.copy_(bi.double())
        ref = md(x.double())

    def run(stencil):
        monkeypatch.setenv("SEHIP_STENCIL", "1" if stencil else "0")
        with torch.no_grad():
            y = F.conv2d(x.cuda(), wr16.cuda(), wi16.cuda(), br.cuda(), bi.cuda(), out_channels=2,
                         kernel=kernel, stride=stride, padding=padding, transposed=True)
        torch.cuda.synchronize()
        assert y.dtype == dtype and y.shape == ref.shape
        return y.float().cpu()

    st, gath = run(True), run(False)
    e_st = rel_l2(st.numpy(), ref.numpy())
    e_ga = rel_l2(gath.numpy(), ref.numpy())
    d = rel_l2(st.numpy(), gath.numpy())
    print(f"{shape} {dtype}: stencil vs fp64 {e_st:.2e}, gather vs fp64 {e_ga:.2e}, stencil vs gather {d:.2e}")
    tol = 1e-6 if dtype == torch.float32 else 6e-3
    assert e_st < tol and d < (1e-6 if dtype == torch.float32 else 8e-3)



@pytest.mark.parametrize("name,tr,cin,cout,shape,stride", [LAYERS[0], LAYERS[1]])
def test_encoder_wgrad_256x128_bit_identical(name, tr, cin, cout, shape, stride, gpu_device, monkeypatch):
    """The encoder weight-grad's opt-in 256 x 128 tiles (SEHIP_WGRAD_K256=1: two taps per
    workgroup share each staged dy row, round 6) sum every output over the same m-split in the
    same order as the default 128 x 128 tiles: bit-identical weight gradients."""
    from sehip import functional as F
    m, x, gy, _ = _fp64_ref(name, tr, cin, cout, shape, stride)
    old = _hip(F, m, x, gy, tr, stride, "f16x3")
    monkeypatch.setenv("SEHIP_WGRAD_K256", "1")
    new = _hip(F, m, x, gy, tr, stride, "f16x3")
    for k in ("dwr", "dwi"):
        assert torch.equal(new[k], old[k]), k
