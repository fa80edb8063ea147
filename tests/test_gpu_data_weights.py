"""Data-grad weight images built in the forward (se_conv2d_prep_data_weights,
se_conv2d_desc.data_weights, ABI 5): the input gradient must be bit-identical
to the pass that builds its image itself in the backward (SEHIP_DATA_PREP=0),
for every math, plain / transposed / stride-phase / joined convs and 16-bit
storage. The image is the same kernel's output either way; only where it is
built changes."""
import pytest
import torch

pytestmark = pytest.mark.gpu

GEOMS = [   # (x shape, out channels, kernel, stride, padding, transposed)
    ((2, 180, 33, 21), 180, (5, 2), (2, 1), (2, 0), False),   # FRCRN encoder conv
    ((2, 180, 17, 21), 180, (5, 2), (2, 1), (2, 0), True),    # decoder convT: 2 stride phases
    ((2, 96, 12, 10), 64, (3, 3), (1, 1), (1, 1), False),     # 96 input channels, 64 out
    ((2, 32, 12, 10), 16, (3, 3), (1, 1), (1, 1), False),     # small N: fp32 tiles
]


def _grads(x, wr, wi, geom, prep, monkeypatch):
    from sehip import functional as F
    _, cout, k, st, pad, tr = geom
    monkeypatch.setenv("SEHIP_DATA_PREP", "1" if prep else "0")
    xa = x.clone().requires_grad_(True)
    wra, wia = wr.clone().requires_grad_(True), wi.clone().requires_grad_(True)
    y = F.conv2d(xa, wra, wia, out_channels=cout, kernel=k, stride=st, padding=pad, transposed=tr)
    g = torch.randn(y.shape, device=x.device, generator=torch.Generator(x.device).manual_seed(3)).to(y.dtype)
    y.backward(g)
    torch.cuda.synchronize()
    return xa.grad, wra.grad, wia.grad


@pytest.mark.parametrize("math", ["f32", "bf16x3", "f16x3", "bf16", "fwd=bf16x6,data=bf16x6,weight=f32"])
@pytest.mark.parametrize("geom", GEOMS)
def test_forward_built_data_image_bit_identical(gpu_device, geom, math, monkeypatch):
    from sehip import functional as F
    prev = F.get_conv_math()
    F.set_conv_math(math)
    try:
        torch.manual_seed(0)
        xs, cout, k, _, _, tr = geom
        cin = xs[1]
        wshape = (cin // 2, cout // 2) + k if tr else (cout // 2, cin // 2) + k
        x = torch.randn(xs, device=gpu_device)
        wr, wi = torch.randn(wshape, device=gpu_device) * 0.05, torch.randn(wshape, device=gpu_device) * 0.05
        n0 = F.DATA_IMG_CALLS[0]
        a = _grads(x, wr, wi, geom, True, monkeypatch)
        assert F.DATA_IMG_CALLS[0] == n0 + 1
        b = _grads(x, wr, wi, geom, False, monkeypatch)
        assert F.DATA_IMG_CALLS[0] == n0 + 1
        for name, u, v in zip(("dx", "dwr", "dwi"), a, b):
            assert torch.equal(u, v), (math, name, (u - v).abs().max().item())
    finally:
        F.set_conv_math(prev)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_forward_built_data_image_16bit_storage(gpu_device, dtype, monkeypatch):
    from sehip import functional as F
    torch.manual_seed(0)
    geom = ((2, 128, 33, 21), 128, (5, 2), (2, 1), (2, 0), False)   # N % 16 == 0: native 16-bit
    xs, cout, k = geom[0], geom[1], geom[2]
    x = torch.randn(xs, device=gpu_device).to(dtype)
    wr = (torch.randn((cout // 2, xs[1] // 2) + k, device=gpu_device) * 0.05).to(dtype)
    wi = (torch.randn((cout // 2, xs[1] // 2) + k, device=gpu_device) * 0.05).to(dtype)
    n16, n0 = F.NATIVE16_CALLS[0], F.DATA_IMG_CALLS[0]
    a = _grads(x, wr, wi, geom, True, monkeypatch)
    assert F.NATIVE16_CALLS[0] > n16 and F.DATA_IMG_CALLS[0] == n0 + 1
    b = _grads(x, wr, wi, geom, False, monkeypatch)
    for name, u, v in zip(("dx", "dwr", "dwi"), a, b):
        assert torch.equal(u, v), (dtype, name)


@pytest.mark.parametrize("math", ["f16x3", "bf16x3", "bf16", "f32"])
def test_forward_built_data_image_joined(gpu_device, math, monkeypatch):
    """The decoder's joined convT (se_conv2d_bwd_data_joined, and its materialising
    fallback for f32) reads the same image."""
    from sehip import functional as F
    prev = F.get_conv_math()
    F.set_conv_math(math)
    try:
        torch.manual_seed(2)
        xs, ss, cout = (2, 128, 8, 38), (2, 128, 9, 37), 128
        x, s = torch.randn(xs, device=gpu_device), torch.randn(ss, device=gpu_device)
        wr = torch.randn(128, 64, 5, 2, device=gpu_device) * 0.05
        wi = torch.randn(128, 64, 5, 2, device=gpu_device) * 0.05
        outs = []
        for prep in (True, False):
            monkeypatch.setenv("SEHIP_DATA_PREP", "1" if prep else "0")
            xa, sa = x.clone().requires_grad_(True), s.clone().requires_grad_(True)
            wra, wia = wr.clone().requires_grad_(True), wi.clone().requires_grad_(True)
            y = F.conv2d_joined(xa, sa, wra, wia, out_channels=cout, kernel=(5, 2), stride=(2, 1), transposed=True)
            y.backward(torch.randn(y.shape, device=gpu_device, generator=torch.Generator(gpu_device).manual_seed(5)))
            torch.cuda.synchronize()
            outs.append((xa.grad, sa.grad, wra.grad, wia.grad))
        for name, u, v in zip(("dx", "dskip", "dwr", "dwi"), *outs):
            assert torch.equal(u, v), (math, name, (u - v).abs().max().item())
    finally:
        F.set_conv_math(prev)
