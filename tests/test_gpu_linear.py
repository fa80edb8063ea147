"""The Linear layers on the hand-written GEMM (sehip.linear -> se_gemm, ABI 10):
ComplexLinear (complex_nn.py:93-113; DCCRN's LSTMBlock, dccrn.py:71-86) and
CARN's Linear(512 -> 514) head (carn.py:133, 157-159).

Oracle: the same Linear in fp64 on the CPU (torch.nn.functional.linear of the
halves, autograd for the gradients). Bars, per tensor rel-L2:
  fp32 storage: 2e-6 (split-fp16 "f16x3" arithmetic, fp32-class; measured ~5e-7);
  bf16 / fp16 storage: the output / gradient rounded once to the format against
  the fp64 value of the same 16-bit operands: 2^-8 (bf16) / 2^-11 (fp16) x 1.5.
Layouts: rows and feature-major input, rows and feature-major output, and the
feature-major gradient a conv consumer hands back."""
import pytest
import torch

pytestmark = pytest.mark.gpu

BARS = {torch.float32: 2e-6, torch.bfloat16: 1.5 * 2 ** -8, torch.float16: 1.5 * 2 ** -11}


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def _ref(x, ws, bs, gy):
    """fp64 CPU forward / backward of cat_h(F.linear(x_h, W_h, b_h))."""
    x = x.detach().double().cpu().requires_grad_(True)
    ws = [w.detach().double().cpu().requires_grad_(True) for w in ws]
    bs = [None if b is None else b.detach().double().cpu().requires_grad_(True) for b in bs]
    parts = torch.chunk(x, len(ws), dim=-1)
    y = torch.cat([torch.nn.functional.linear(p, w, b) for p, w, b in zip(parts, ws, bs)], dim=-1)
    y.backward(gy.detach().double().cpu())
    return y, x.grad, [w.grad for w in ws], [None if b is None else b.grad for b in bs]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("halves,B,T,cin,cout,x_feat,y_feat,bias", [
    (2, 3, 77, 128, 512, False, True, True),      # DCCRN LSTMBlock ComplexLinear (scaled down in B, T)
    (2, 2, 50, 96, 40, True, False, True),        # tails, feature-major input
    (1, 2, 301, 512, 514, True, True, True),      # CARN head
    (1, 1, 129, 64, 33, False, False, False),     # no bias, rows both ways
])
def test_linear_halves_vs_fp64(gpu_device, dtype, halves, B, T, cin, cout, x_feat, y_feat, bias):
    from sehip.linear import linear_halves
    torch.manual_seed(3)
    K = halves * cin
    if x_feat:
        x = torch.randn(B, K, T, device=gpu_device).to(dtype).transpose(1, 2)
    else:
        x = torch.randn(B, T, K, device=gpu_device).to(dtype)
    x.requires_grad_(True)
    ws = [(torch.randn(cout, cin, device=gpu_device) / cin ** 0.5).to(dtype).requires_grad_(True)
          for _ in range(halves)]
    bs = [(torch.randn(cout, device=gpu_device) * 0.1).to(dtype).requires_grad_(True) if bias else None
          for _ in range(halves)]
    y = linear_halves(x, ws, bs, feature_major_out=y_feat)
    assert y.shape == (B, T, halves * cout)
    if y_feat:
        assert y.transpose(1, 2).is_contiguous()
    # the gradient in the layout a conv consumer returns it (feature-major) or rows
    gy = torch.randn(B, halves * cout, T, device=gpu_device).to(dtype).transpose(1, 2) if y_feat else \
        torch.randn(B, T, halves * cout, device=gpu_device).to(dtype)
    y.backward(gy)
    ry, rdx, rdw, rdb = _ref(x, ws, bs, gy)
    bar = BARS[dtype]
    assert _rel(y, ry) < bar, ("y", _rel(y, ry))
    assert _rel(x.grad, rdx) < bar, ("dx", _rel(x.grad, rdx))
    for h in range(halves):
        assert _rel(ws[h].grad, rdw[h]) < bar, ("dw", h, _rel(ws[h].grad, rdw[h]))
        if bias:
            assert _rel(bs[h].grad, rdb[h]) < bar, ("db", h, _rel(bs[h].grad, rdb[h]))


def test_complex_linear_module_matches_reference_form(gpu_device):
    """sehip ComplexLinear == the reference's two nn.Linear calls (complex_nn.py:106-113) on the
    same parameters; the state_dict keys are the reference's."""
    from sehip.complex_nn import ComplexLinear
    from sehip import linear as LN
    torch.manual_seed(4)
    m = ComplexLinear(256, 1024).to(gpu_device)
    assert sorted(m.state_dict()) == sorted(["real_linear.weight", "real_linear.bias", "imag_linear.weight",
                                             "imag_linear.bias"])
    x = torch.randn(2, 40, 256, device=gpu_device, dtype=torch.float64)
    n0 = LN.LINEAR_CALLS[0]
    with torch.no_grad():
        y = m(x.float())
        re, im = torch.chunk(x, 2, dim=-1)
        ref = torch.cat([torch.nn.functional.linear(re, m.real_linear.weight.double(), m.real_linear.bias.double()),
                         torch.nn.functional.linear(im, m.imag_linear.weight.double(), m.imag_linear.bias.double())],
                        dim=-1)
    assert LN.LINEAR_CALLS[0] == n0 + 1
    assert _rel(y, ref) < 2e-6


def test_bias_grad_strides(gpu_device):
    """se_bias_grad over rows (sg = 1) and over contiguous rows per feature (sr = 1), all dtypes."""
    from sehip import _native as N
    from sehip import functional as F
    for dt in (torch.float32, torch.bfloat16, torch.float16):
        for feat in (False, True):
            torch.manual_seed(5)
            L, R, G = 3, 1000, 77
            g = torch.randn(L, G, R, device=gpu_device).to(dt).transpose(1, 2) if feat else \
                torch.randn(L, R, G, device=gpu_device).to(dt)
            out = torch.empty(G, device=gpu_device, dtype=dt)
            ws = F._workspace(N.lib().se_bias_grad_workspace_size(L, R, G), gpu_device)
            N.check(N.lib().se_bias_grad(g.data_ptr(), L, R, G, *g.stride(), N.dtype_code(g), out.data_ptr(),
                                         ws.data_ptr(), ws.numel(), N.stream_of(g)), "se_bias_grad")
            ref = g.double().sum((0, 1))
            assert _rel(out, ref) < BARS[dt] + 1e-6, (dt, feat, _rel(out, ref))
