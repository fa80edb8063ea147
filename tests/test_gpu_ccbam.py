"""Fused CCBAM (csrc/ccbam.hip + the sub-modules' HIP conv/CBN) against the
oracle's restatement of models/modules/ccbam.py on the CPU (fp32):
forward output, input gradient, every parameter gradient and the spatial
CBN's running statistics. Tolerance: rel-L2 <= 1e-5 forward, <= 1e-4 for
gradients (reduction order only; the gate's sigmoid/CBN chain is smooth).

Ties: the fused kernels send max-pool gradients to the first maximal index
(AdaptiveMaxPool2d, torch.max(dim)); continuous random inputs have no ties,
so the comparison is exact in structure."""
import pytest
import torch

from conftest import rel_l2

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return rel_l2(a.detach().double().cpu().numpy(), b.detach().double().cpu().numpy())


@pytest.mark.parametrize("B,C,H,W", [(2, 32, 9, 13), (3, 128, 7, 403), (2, 128, 2, 403), (1, 4, 5, 5)])
def test_ccbam_matches_oracle(gpu_device, B, C, H, W):
    from oracle.ccbam import CCBAM as OCCBAM
    from sehip.ccbam import CCBAM
    torch.manual_seed(B * 1000 + C + H)
    ref = OCCBAM(C).train()
    mod = CCBAM(C).train()
    mod.load_state_dict(ref.state_dict())
    x = torch.randn(B, C, H, W)
    g = torch.randn(B, C, H, W)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    (yr * g).sum().backward()
    mod = mod.to(gpu_device)
    xd = x.to(gpu_device).requires_grad_(True)
    yd = mod(xd)
    assert _rel(yd, yr) < 1e-5
    (yd * g.to(gpu_device)).sum().backward()
    assert _rel(xd.grad, xr.grad) < 1e-4
    rp = dict(ref.named_parameters())
    for n, p in mod.named_parameters():
        assert p.grad is not None, n
        assert _rel(p.grad, rp[n].grad) < 1e-4, (n, _rel(p.grad, rp[n].grad))
    rb = dict(ref.named_buffers())
    for n, b in mod.named_buffers():
        if b.dtype.is_floating_point:
            assert _rel(b, rb[n]) < 1e-5, n


def test_ccbam_eval_and_no_grad(gpu_device):
    from oracle.ccbam import CCBAM as OCCBAM
    from sehip.ccbam import CCBAM
    torch.manual_seed(5)
    ref = OCCBAM(32).eval()
    mod = CCBAM(32).eval()
    mod.load_state_dict(ref.state_dict())
    x = torch.randn(2, 32, 6, 20)
    with torch.no_grad():
        yd = mod.to(gpu_device)(x.to(gpu_device))
    assert _rel(yd, ref(x)) < 1e-5


def test_ccbam_fused_matches_unfused_on_gpu(gpu_device):
    """The fused path against the module's own op-by-op formulation on the GPU
    at an FRCRN skip shape (B=8 of the B=64 decoder input, F=37)."""
    from sehip.ccbam import CCBAM
    torch.manual_seed(7)
    mod = CCBAM(128).to(gpu_device).train()
    x = torch.randn(8, 128, 37, 403, device=gpu_device)
    g = torch.randn_like(x)
    x1 = x.clone().requires_grad_(True)
    y1 = mod.forward_unfused(x1)
    (y1 * g).sum().backward()
    g1 = {n: p.grad.clone() for n, p in mod.named_parameters()}
    mod.zero_grad(set_to_none=True)
    x2 = x.clone().requires_grad_(True)
    y2 = mod(x2)
    (y2 * g).sum().backward()
    assert _rel(y2, y1) < 1e-5
    assert _rel(x2.grad, x1.grad) < 1e-4
    for n, p in mod.named_parameters():
        assert _rel(p.grad, g1[n]) < 1e-4, n


@pytest.mark.parametrize("B,C,Hd", [(64, 128, 8), (3, 32, 4), (2, 4, 2)])
def test_ccbam_mlp_kernels_vs_fp64(B, C, Hd, gpu_device):
    """se_ccbam_mlp_fwd / _bwd (the channel branch's shared MLP + sigmoid in one launch
    each way) against the same math in fp64 on the CPU: ca, dmean, dmax and the four
    weight gradients at rel-L2 1e-5 (fp32 sums in index order vs fp64)."""
    from sehip import _native as N
    gen = torch.Generator().manual_seed(B + C)
    mean, mx = torch.randn(B, C, generator=gen), torch.randn(B, C, generator=gen) + 1.0
    w = [torch.randn(Hd // 2, C // 2, generator=gen) * 0.3, torch.randn(Hd // 2, C // 2, generator=gen) * 0.3,
         torch.randn(C // 2, Hd // 2, generator=gen) * 0.3, torch.randn(C // 2, Hd // 2, generator=gen) * 0.3]
    dca = torch.randn(B, C, generator=gen)
    # fp64 reference: ComplexLinear -> ReLU -> ComplexLinear on [mean; max], sigmoid(a + m)
    p = torch.cat([mean, mx]).double().requires_grad_(True)
    w64 = [t.double().requires_grad_(True) for t in w]
    h = torch.relu(torch.cat([p[:, :C // 2] @ w64[0].t(), p[:, C // 2:] @ w64[1].t()], 1))
    o = torch.cat([h[:, :Hd // 2] @ w64[2].t(), h[:, Hd // 2:] @ w64[3].t()], 1)
    ca64 = torch.sigmoid(o[:B] + o[B:])
    ca64.backward(dca.double())
    dev = gpu_device
    md, xd, wd = mean.to(dev), mx.to(dev), [t.to(dev) for t in w]
    ca = torch.empty(B, C, device=dev)
    hs = torch.empty(2 * B, Hd, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    lib = N.lib()
    N.check(lib.se_ccbam_mlp_fwd(md.data_ptr(), xd.data_ptr(), *(t.data_ptr() for t in wd), B, C, Hd,
                                 ca.data_ptr(), hs.data_ptr(), st), "se_ccbam_mlp_fwd")
    dm, dx = torch.empty(B, C, device=dev), torch.empty(B, C, device=dev)
    dws = [torch.empty_like(t) for t in wd]
    N.check(lib.se_ccbam_mlp_bwd(dca.to(dev).data_ptr(), ca.data_ptr(), md.data_ptr(), xd.data_ptr(), hs.data_ptr(),
                                 *(t.data_ptr() for t in wd), B, C, Hd, dm.data_ptr(), dx.data_ptr(),
                                 *(t.data_ptr() for t in dws), st), "se_ccbam_mlp_bwd")
    torch.cuda.synchronize()
    assert _rel(ca, ca64) < 1e-6
    assert _rel(dm, p.grad[:B]) < 1e-5 and _rel(dx, p.grad[B:]) < 1e-5
    for got, ref in zip(dws, w64):
        assert _rel(got, ref.grad) < 1e-5


def test_ccbam_fused_mlp_matches_module_mlp(gpu_device, monkeypatch):
    """The fused MLP launch (default) against the MLP run as its own modules
    (SEHIP_CCBAM_MLP=0) inside the fused CCBAM: outputs and every gradient."""
    from sehip.ccbam import CCBAM
    torch.manual_seed(11)
    mod = CCBAM(128).to(gpu_device).train()
    x = torch.randn(4, 128, 17, 403, device=gpu_device)
    g = torch.randn_like(x)
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("SEHIP_CCBAM_MLP", flag)
        mod.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        y = mod(xi)
        (y * g).sum().backward()
        res.append((y.detach(), xi.grad, {n: p.grad.clone() for n, p in mod.named_parameters()}))
    (y0, dx0, g0), (y1, dx1, g1) = res
    assert _rel(y1, y0) < 1e-6 and _rel(dx1, dx0) < 1e-5
    for n in g0:
        assert _rel(g1[n], g0[n]) < 1e-5, n


@pytest.mark.parametrize("HW", [160 * 404, 10 * 403, 37])
def test_bwd_sa_sigmoid_bit_identical(gpu_device, HW):
    """se_ccbam_bwd_sa_sigmoid == se_ccbam_bwd_sa then torch's sigmoid backward, to the bit
    (16-B path where HW % 4 == 0, guarded scalar path otherwise)."""
    from sehip import _native as N
    torch.manual_seed(7)
    B, C = 3, 128
    g = torch.randn(B, C, HW, device=gpu_device)
    z = torch.randn(B, 2, HW, device=gpu_device, requires_grad=True)
    sa = torch.sigmoid(z)
    lib, st = N.lib(), N.stream_of(g)
    dsa = torch.empty(B, 2, HW, device=gpu_device)
    N.check(lib.se_ccbam_bwd_sa(g.data_ptr(), dsa.data_ptr(), B, C, HW, st), "se_ccbam_bwd_sa")
    ref, = torch.autograd.grad(sa, z, dsa)
    dz = torch.empty(B, 2, HW, device=gpu_device)
    sad = sa.detach().contiguous()
    N.check(lib.se_ccbam_bwd_sa_sigmoid(g.data_ptr(), sad.data_ptr(), dz.data_ptr(), B, C, HW, st),
            "se_ccbam_bwd_sa_sigmoid")
    torch.cuda.synchronize()
    assert torch.equal(dz, ref)


@pytest.mark.parametrize("shape", [(3, 4, 160, 404), (2, 4, 37, 70), (1, 4, 5, 403)])
def test_spatial_conv_stencil_bit_identical(gpu_device, monkeypatch, shape):
    """The CCBAM spatial ComplexConv2d(4 -> 2, k7, pad 3) forward and data-grad on the LDS
    stencil (gather_stencil_kernel) equal gather_smalln_kernel (SEHIP_STENCIL=0) to the
    bit (same products, same order), including partial edge tiles."""
    from sehip import functional as F
    torch.manual_seed(11)
    x = torch.randn(shape, device=gpu_device)
    wr = torch.randn(1, 2, 7, 7, device=gpu_device) * 0.1
    wi = torch.randn(1, 2, 7, 7, device=gpu_device) * 0.1
    g = torch.randn(shape[0], 2, shape[2], shape[3], device=gpu_device)
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("SEHIP_STENCIL", flag)
        xa = x.clone().requires_grad_(True)
        y = F.conv2d(xa, wr, wi, out_channels=2, kernel=(7, 7), padding=(3, 3))
        y.backward(g)
        torch.cuda.synchronize()
        outs.append((y.detach(), xa.grad))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    ref = torch.nn.functional.conv2d(x.double().cpu(),
                                     torch.cat([torch.cat([wr, -wi], 1), torch.cat([wi, wr], 1)], 0).double().cpu(),
                                     padding=3)
    assert ((outs[0][0].double().cpu() - ref).norm() / ref.norm()).item() < 1e-6


@pytest.mark.parametrize("overlap", ["0", "1"])
def test_deferred_gate_input_grad_bit_identical(gpu_device, monkeypatch, overlap):
    """FRCRN's CCBAM gates read forked encoder outputs: their input gradient is formed inside
    the forked CBN backward (se_cbn_bwd_ccbam, ABI 11) instead of being written by
    se_ccbam_bwd_dx and read back. Two train steps give bit-identical losses and parameters
    with the deferral on and off (the kernel forms bwd_dx_kernel's expression term for term),
    with the gates inline and on the side stream; the five forked-CBN gates (encoder layers
    1-5; layer 0's output comes from the first-block op) take the deferred form."""
    import paramfill
    from sehip import functional as F
    from sehip import models as M
    from sehip.train import make_optimizer, train_step
    monkeypatch.setenv("SEHIP_OVERLAP", overlap)
    noisy, clean = paramfill.structured_pair(2, 16000, seed=8)
    x, c = torch.from_numpy(noisy).cuda(), torch.from_numpy(clean).cuda()
    res = []
    for defer in ("0", "1"):
        monkeypatch.setenv("SEHIP_CCBAM_DEFER_DX", defer)
        m = paramfill.fill_(M.FRCRN(), seed=9).cuda().train()
        opt = make_optimizer(m)
        n0 = F.CCBAM_DX_FUSED[0]
        losses = [train_step(m, opt, x, c) for _ in range(2)]
        torch.cuda.synchronize()
        assert F.CCBAM_DX_FUSED[0] - n0 == (10 if defer == "1" else 0)
        res.append(losses + [p.detach().clone() for p in m.parameters()])
    assert not F._CCBAM_DX
    for a, b in zip(*res):
        assert torch.equal(a, b)
