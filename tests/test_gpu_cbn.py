"""GPU parity: ComplexBatchNorm2d kernels (csrc/cbn.hip) vs reference goldens:
train-mode forward, running-stat update, backward (dx and all 5 affine
params), eval-mode forward/backward; plus fused LeakyReLU vs oracle."""
import numpy as np
import pytest
import torch

from conftest import golden, rel_l2
import paramfill

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,C,seed", [("c5", 10, 0), ("c1", 2, 1)])
def test_cbn_golden(name, C, seed, gpu_device):
    from sehip.complex_nn import ComplexBatchNorm2d
    g = golden("cbn")
    m = paramfill.fill_(ComplexBatchNorm2d(C), seed=seed).cuda().train()
    x = torch.from_numpy(g[f"{name}_x"]).cuda().requires_grad_(True)
    y = m(x)
    assert rel_l2(y.detach().cpu().numpy(), g[f"{name}_y"]) < 1e-5
    (y * torch.from_numpy(g[f"{name}_gy"]).cuda()).sum().backward()
    assert rel_l2(x.grad.cpu().numpy(), g[f"{name}_dx"]) < 1e-5
    dp = torch.cat([m.Wrr.grad, m.Wri.grad, m.Wii.grad, m.Br.grad, m.Bi.grad]).cpu().numpy()
    assert rel_l2(dp, g[f"{name}_dparams"]) < 1e-5
    run = torch.cat([m.RMr, m.RMi, m.RVrr, m.RVri, m.RVii]).cpu().numpy()
    np.testing.assert_allclose(run, g[f"{name}_run1"], rtol=1e-5, atol=1e-6)
    assert int(m.num_batches_tracked) == 1
    m2 = paramfill.fill_(ComplexBatchNorm2d(C), seed=seed).cuda().eval()
    xe = torch.from_numpy(g[f"{name}_x"]).cuda().requires_grad_(True)
    ye = m2(xe)
    assert rel_l2(ye.detach().cpu().numpy(), g[f"{name}_yeval"]) < 1e-5
    (ye * torch.from_numpy(g[f"{name}_gy"]).cuda()).sum().backward()
    assert rel_l2(xe.grad.cpu().numpy(), g[f"{name}_dxeval"]) < 1e-5
    dpe = torch.cat([m2.Wrr.grad, m2.Wri.grad, m2.Wii.grad, m2.Br.grad, m2.Bi.grad]).cpu().numpy()
    assert rel_l2(dpe, g[f"{name}_dparamseval"]) < 1e-5


def test_cbn_leaky_fused_vs_oracle(gpu_device):
    """FRCRN-shaped CBN(128) + LeakyReLU(0.2), fused in one kernel, vs oracle."""
    from sehip.complex_nn import ComplexBatchNorm2d, norm_act
    from oracle.complex_nn import ComplexBatchNorm2d as OCBN
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(3, 128, 17, 41, generator=gen) * 2 + 0.5
    gy = torch.randn(x.shape, generator=gen)
    mo = paramfill.fill_(OCBN(128), seed=2).train()
    xo = x.clone().requires_grad_(True)
    yo = torch.nn.functional.leaky_relu(mo(xo), 0.2)
    yo.backward(gy)
    m = paramfill.fill_(ComplexBatchNorm2d(128), seed=2).cuda().train()
    xg = x.cuda().requires_grad_(True)
    y = norm_act(m, torch.nn.LeakyReLU(0.2), xg)
    y.backward(gy.cuda())
    assert rel_l2(y.detach().cpu().numpy(), yo.detach().numpy()) < 1e-5
    assert rel_l2(xg.grad.cpu().numpy(), xo.grad.numpy()) < 1e-4
    for n in ("Wrr", "Wri", "Wii", "Br", "Bi"):
        assert rel_l2(getattr(m, n).grad.cpu().numpy(), getattr(mo, n).grad.numpy()) < 1e-4, n
    for n in ("RMr", "RMi", "RVrr", "RVri", "RVii"):
        np.testing.assert_allclose(getattr(m, n).cpu().numpy(), getattr(mo, n).detach().numpy(),
                                   rtol=1e-5, atol=1e-6)


def test_cbn_whitening_full_size(gpu_device):
    """Known answer: with W = I, B = 0 the train-mode output is
    whitened — zero mean, identity covariance — at an FRCRN activation size."""
    from sehip.complex_nn import ComplexBatchNorm2d
    m = ComplexBatchNorm2d(128).cuda().train()
    with torch.no_grad():
        m.Wri.zero_()
    x = torch.randn(8, 128, 77, 403, device="cuda") * 3 + 1.5
    x[:, 64:] += 0.7 * x[:, :64]          # correlate real / imag
    y = m(x).double()
    yr, yi = y[:, :64], y[:, 64:]
    assert yr.mean(dim=(0, 2, 3)).abs().max() < 1e-5
    assert (yr.pow(2).mean(dim=(0, 2, 3)) - 1).abs().max() < 1e-3
    assert (yi.pow(2).mean(dim=(0, 2, 3)) - 1).abs().max() < 1e-3
    assert (yr * yi).mean(dim=(0, 2, 3)).abs().max() < 1e-3


@pytest.mark.parametrize("act", [0, 1, 2])
def test_cbn_amax_bounds(act, gpu_device):
    """The SE_MATH_F16X3 scale sources se_cbn_fwd / se_cbn_bwd emit with no extra
    pass: an upper bound of max |y| and of max |dx| (never below the true
    maximum, at most a small factor above it)."""
    from sehip import functional as F
    from sehip.complex_nn import ComplexBatchNorm2d
    seen = {}

    class Probe(torch.autograd.Function):   # sees dx with the address the CBN backward registered
        @staticmethod
        def forward(ctx, t):
            return t.view(t.shape)

        @staticmethod
        def backward(ctx, g):
            seen["dx"], seen["dx_amax"] = g.clone(), F.amax_get(g)
            return g

    m = paramfill.fill_(ComplexBatchNorm2d(128), seed=3).cuda().train()
    gen = torch.Generator(device=gpu_device).manual_seed(9)
    x = (torch.randn(4, 128, 37, 50, device=gpu_device, generator=gen) * 3 + 0.5).requires_grad_(True)
    y = m.forward_act(Probe.apply(x), act, 0.2)
    ya = F.amax_get(y)
    assert ya is not None
    true_y = y.detach().abs().max().item()
    assert true_y <= ya.item() <= 4 * true_y, (true_y, ya.item())
    gy = torch.randn(y.shape, device=gpu_device, generator=gen) * 1e-7
    y.backward(gy)
    assert seen["dx_amax"] is not None
    true_dx = seen["dx"].abs().max().item()
    assert true_dx <= seen["dx_amax"].item() <= 16 * true_dx, (true_dx, seen["dx_amax"].item())


@pytest.mark.parametrize("used", ["both", "first", "second"])
def test_cbn_fork_sums_both_gradients(used, gpu_device):
    """fork=True (FRCRN encoder outputs: next conv + decoder skip) sums the two output
    gradients inside se_cbn_bwd2; bit-identical to autograd's add followed by se_cbn_bwd,
    and either consumer alone (the other gradient absent) matches the plain backward."""
    from sehip.complex_nn import ComplexBatchNorm2d, norm_act
    gen = torch.Generator().manual_seed(11)
    x = (torch.randn(4, 128, 13, 37, generator=gen) * 1.5 + 0.3).cuda()
    g1 = torch.randn(x.shape, generator=gen).cuda()
    g2 = torch.randn(x.shape, generator=gen).cuda()
    grads = {"both": (g1, g2), "first": (g1, None), "second": (None, g2)}[used]
    act = torch.nn.LeakyReLU(0.2)

    m0 = paramfill.fill_(ComplexBatchNorm2d(128), seed=4).cuda().train()
    x0 = x.clone().requires_grad_(True)
    y0 = norm_act(m0, act, x0)
    y0.backward(sum(g for g in grads if g is not None))

    m1 = paramfill.fill_(ComplexBatchNorm2d(128), seed=4).cuda().train()
    x1 = x.clone().requires_grad_(True)
    ya, yb = norm_act(m1, act, x1, fork=True)
    assert yb.data_ptr() == ya.data_ptr() and torch.equal(ya, y0)
    outs = [(t, g) for t, g in zip((ya, yb), grads) if g is not None]
    torch.autograd.backward([t for t, _ in outs], [g for _, g in outs])
    assert torch.equal(x1.grad, x0.grad)
    for n in ("Wrr", "Wri", "Wii", "Br", "Bi"):
        assert torch.equal(getattr(m1, n).grad, getattr(m0, n).grad), n


@pytest.mark.parametrize("shape,act,train", [((3, 128, 19, 41), 1, True), ((2, 128, 5, 2), 1, True),
                                             ((2, 16, 7, 300), 2, True), ((3, 128, 19, 41), 1, False),
                                             ((2, 32, 11, 70), 0, True)])
def test_cbn_head_fused_vs_fp64(shape, act, train, gpu_device):
    """se_cbn_head_*: final_conv(act(CBN(x))) (frcrn.py:115, 140) with the activation never
    written, vs the fp64 oracle CBN + activation + conv2d on the CPU: the head output, dx,
    the 5 CBN parameter gradients, the head's weight gradient and the running statistics."""
    from sehip import functional as F
    from sehip.complex_nn import ComplexBatchNorm2d
    from oracle.complex_nn import ComplexBatchNorm2d as OCBN
    tf = torch.nn.functional
    b, c, h, w = shape
    gen = torch.Generator().manual_seed(21)
    x = torch.randn(shape, generator=gen) * 1.7 + 0.4
    x[:, c // 2:] += 0.5 * x[:, :c // 2]
    wh = torch.randn(2, c, 1, 2, generator=gen) / c ** 0.5
    gout = torch.randn(b, 2, h, w - 1, generator=gen)
    acts = {0: lambda t: t, 1: lambda t: tf.leaky_relu(t, 0.2), 2: tf.relu}

    mo = paramfill.fill_(OCBN(c), seed=7).double()
    mo.train(train)
    if not train:   # non-trivial running statistics
        with torch.no_grad():
            mo.RMr.uniform_(-0.5, 0.5); mo.RMi.uniform_(-0.5, 0.5)
            mo.RVrr.uniform_(1, 3); mo.RVii.uniform_(1, 3); mo.RVri.uniform_(-0.5, 0.5)
    m = paramfill.fill_(ComplexBatchNorm2d(c), seed=7).cuda()
    m.load_state_dict({k: v.float() for k, v in mo.state_dict().items()})
    m.train(train)
    xo = x.double().requires_grad_(True)
    who = wh.double().requires_grad_(True)
    yo = tf.conv2d(acts[act](mo(xo)), who)
    yo.backward(gout.double())

    xg = x.cuda().requires_grad_(True)
    whg = wh.cuda().requires_grad_(True)
    running = (m.RMr, m.RMi, m.RVrr, m.RVri, m.RVii)
    y = F.complex_batch_norm_head(xg, m.Wrr, m.Wri, m.Wii, m.Br, m.Bi, whg, running, m.num_batches_tracked,
                                  train, m.eps, m.momentum, act, 0.2)
    y.backward(gout.cuda())
    assert y.shape == yo.shape
    assert rel_l2(y.detach().cpu().numpy(), yo.detach().numpy()) < 1e-5
    assert rel_l2(xg.grad.cpu().numpy(), xo.grad.numpy()) < 1e-5
    assert rel_l2(whg.grad.cpu().numpy(), who.grad.numpy()) < 1e-5
    for n in ("Wrr", "Wri", "Wii", "Br", "Bi"):
        assert rel_l2(getattr(m, n).grad.cpu().numpy(), getattr(mo, n).grad.numpy()) < 1e-5, n
    for n in ("RMr", "RMi", "RVrr", "RVri", "RVii"):
        np.testing.assert_allclose(getattr(m, n).cpu().numpy(), getattr(mo, n).detach().numpy(),
                                   rtol=1e-5, atol=1e-6)
    assert int(m.num_batches_tracked) == int(mo.num_batches_tracked)


def test_frcrn_head_fused_matches_unfused(gpu_device, monkeypatch):
    """FRCRN train step with the head fused (default) vs SEHIP_HEAD=0 (CBN apply + the
    real final_conv on the conv kernels): same enhanced output and gradients to fp32
    rounding (different summation orders only)."""
    from sehip import models as M
    noisy, _ = paramfill.structured_pair(2, 16000, seed=3)
    x = torch.from_numpy(noisy).cuda()
    res = []
    for flag in ("1", "0"):
        monkeypatch.setenv("SEHIP_HEAD", flag)
        m = paramfill.fill_(M.FRCRN(), seed=3).cuda().train()
        spec, wav = m(x)
        (spec.square().sum() + wav.sum()).backward()
        torch.cuda.synchronize()
        res.append((spec.detach(), wav.detach(), {n: p.grad.clone() for n, p in m.named_parameters()},
                    {n: b.clone() for n, b in m.named_buffers()}))
    (s1, w1, g1, b1), (s0, w0, g0, b0) = res
    assert rel_l2(s1.cpu().numpy(), s0.cpu().numpy()) < 1e-6
    assert rel_l2(w1.cpu().numpy(), w0.cpu().numpy()) < 1e-6
    for n in g0:
        # the CCBAM spatial gates' CBN has one complex channel: each of its five scalar
        # parameter gradients is one sum over a whole skip map whose terms largely cancel,
        # so a summation-order change moves it ~1e-4 relative (measured 1.6e-4 on Br)
        tol = 1e-3 if "spatial_attention_branch.conv.norm" in n else 1e-4
        assert rel_l2(g1[n].cpu().numpy(), g0[n].cpu().numpy()) < tol, n
    for n in b0:
        if b0[n].is_floating_point():
            np.testing.assert_allclose(b1[n].cpu().numpy(), b0[n].cpu().numpy(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("fork", [False, True])
@pytest.mark.parametrize("shape", [(3, 2, 40, 37), (2, 2, 320, 101)])
def test_first_block_fused_vs_fp64(shape, fork, gpu_device):
    """se_cbn_bwd_first_conv: FRCRN's first block (causal pad (1, 0) + ComplexConv2d(2, 128,
    (5, 2), stride (2, 1), no bias) + ComplexBatchNorm2d + LeakyReLU, frcrn.py:11-34) with
    the conv's weight gradient accumulated inside the CBN backward apply (no dy tensor),
    against the fp64 oracle modules on the CPU: the output, the conv's dWr / dWi, the 5
    CBN parameter gradients and the running statistics; fork=True sums two consumers'
    gradients (the encoder output feeds the next block and the decoder skip)."""
    from sehip import functional as F
    from sehip.complex_nn import ComplexBatchNorm2d, ComplexConv2d
    from oracle.complex_nn import ComplexBatchNorm2d as OCBN, ComplexConv2d as OConv
    tf = torch.nn.functional
    gen = torch.Generator().manual_seed(31)
    x = torch.randn(shape, generator=gen) * 0.8
    co = paramfill.fill_(OConv(2, 128, (5, 2), stride=(2, 1), bias=False), seed=5).double()
    no = paramfill.fill_(OCBN(128), seed=6).double().train()
    # the device modules start from the same state, copied before the oracle's forward
    # updates its running statistics
    c = ComplexConv2d(2, 128, (5, 2), stride=(2, 1), bias=False).cuda()
    c.load_state_dict({k: v.float() for k, v in co.state_dict().items()})
    n = ComplexBatchNorm2d(128).cuda()
    n.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in no.state_dict().items()})
    yo = tf.leaky_relu(no(co(tf.pad(x.double(), (1, 0, 0, 0)))), 0.2)
    g1 = torch.randn(yo.shape, generator=gen, dtype=torch.float64)
    g2 = torch.randn(yo.shape, generator=gen, dtype=torch.float64)
    (yo * g1 + (yo * g2 if fork else 0)).sum().backward()
    xg = x.cuda()
    assert F.first_block_supported(xg, c.real_conv.weight, None, True, (5, 2))
    out = F.first_block(xg, c.real_conv.weight, c.imag_conv.weight, n.Wrr, n.Wri, n.Wii, n.Br, n.Bi,
                        (n.RMr, n.RMi, n.RVrr, n.RVri, n.RVii), n.num_batches_tracked, n.eps, n.momentum,
                        F.ACT_LEAKY, 0.2, kernel=(5, 2), stride=(2, 1), padding=(0, 1), padding_end=(0, 0),
                        dilation=(1, 1), fork=fork)
    if fork:
        y, y2 = out
        (y * g1.float().cuda() + y2 * g2.float().cuda()).sum().backward()
    else:
        y = out
        (y * g1.float().cuda()).sum().backward()
    assert rel_l2(y.detach().cpu().numpy(), yo.detach().numpy()) < 1e-5
    for name, a, b in (("dWr", c.real_conv.weight, co.real_conv.weight), ("dWi", c.imag_conv.weight, co.imag_conv.weight)):
        e = rel_l2(a.grad.cpu().numpy(), b.grad.numpy())
        print(f"{shape} fork={fork} {name}: {e:.2e}")
        assert e < 1e-5, (name, e)
    for k in ("Wrr", "Wri", "Wii", "Br", "Bi"):
        assert rel_l2(getattr(n, k).grad.cpu().numpy(), getattr(no, k).grad.numpy()) < 1e-5, k
    for k in ("RMr", "RMi", "RVrr", "RVri", "RVii"):
        np.testing.assert_allclose(getattr(n, k).cpu().numpy(), getattr(no, k).detach().numpy(), rtol=1e-5, atol=1e-6)


def test_frcrn_first_block_fused_matches_unfused(gpu_device, monkeypatch):
    """FRCRN train-mode forward + backward with the fused first block (default) vs
    SEHIP_FIRST_FUSED=0 (conv weight-grad GEMM on a written dy): same output, gradients
    to fp32 rounding for the first conv's weights (summed in another order, exact fp32
    products either way), bit-identical for every other parameter."""
    from sehip import models as M
    from sehip.losses import SI_SNR_loss
    noisy, clean = paramfill.structured_pair(2, 16000, seed=13)
    x, cl = torch.from_numpy(noisy).cuda(), torch.from_numpy(clean).cuda()
    res = []
    for flag in ("1", "0"):
        monkeypatch.setenv("SEHIP_FIRST_FUSED", flag)
        m = paramfill.fill_(M.FRCRN(), seed=14).cuda().train()
        _, wav = m(x)
        SI_SNR_loss(wav, cl).backward()
        torch.cuda.synchronize()
        res.append((wav.detach(), {k: p.grad.detach() for k, p in m.named_parameters()}))
    assert torch.equal(res[0][0], res[1][0])
    for k in res[0][1]:   # only the first conv's weight gradient is computed differently
        assert k.startswith("encoder.layers.0.conv") or torch.equal(res[0][1][k], res[1][1][k]), k
    e0 = [((res[0][1][k] - res[1][1][k]).norm() / res[1][1][k].norm()).item()
          for k in res[0][1] if k.startswith("encoder.layers.0.conv")]
    print("encoder.layers.0.conv weight grads fused vs unfused:", e0)
    assert max(e0) < 1e-5


@pytest.mark.parametrize("dtype,tol", [(torch.bfloat16, 1.5e-2), (torch.float16, 2e-3)])
@pytest.mark.parametrize("train", [True, False])
def test_cbn_low_precision_storage(dtype, tol, train, gpu_device):
    """model.to(bfloat16) / .half() (BASELINE configs 2 / 3 / 5): the CBN kernels read
    and write bf16 / fp16 activations, parameters and running statistics directly
    (fp32 arithmetic, fp64 moments, no cast passes). Against the fp64 oracle on the
    same rounded inputs: output, dx, parameter gradients within the storage's rounding;
    every result in the storage dtype."""
    from sehip.complex_nn import ComplexBatchNorm2d
    from oracle.complex_nn import ComplexBatchNorm2d as OCBN
    tf = torch.nn.functional
    gen = torch.Generator().manual_seed(41)
    b, c, h, w = 4, 16, 9, 44
    x = (torch.randn(b, c, h, w, generator=gen) * 1.3 + 0.2).to(dtype)
    gy = torch.randn(b, c, h, w, generator=gen).to(dtype)
    mo = paramfill.fill_(OCBN(c), seed=9).to(dtype).double().train(train)
    if not train:
        with torch.no_grad():
            # values the storage dtype holds exactly: both sides see the same statistics
            mo.RVrr.fill_(1.5); mo.RVii.fill_(0.6875); mo.RMr.fill_(0.125)
    m = ComplexBatchNorm2d(c).cuda()
    m.load_state_dict({k: v.to(dtype) if v.is_floating_point() else v for k, v in mo.state_dict().items()})
    m = m.to(dtype).train(train)
    xo = x.double().requires_grad_(True)
    yo = tf.leaky_relu(mo(xo), 0.2)
    yo.backward(gy.double())
    xg = x.cuda().requires_grad_(True)
    from sehip import functional as F
    y = m.forward_act(xg, F.ACT_LEAKY, 0.2)
    y.backward(gy.cuda())
    assert y.dtype == dtype and xg.grad.dtype == dtype and m.Wrr.grad.dtype == dtype
    assert rel_l2(y.detach().float().cpu().numpy(), yo.detach().numpy()) < tol
    assert rel_l2(xg.grad.float().cpu().numpy(), xo.grad.numpy()) < tol
    for k in ("Wrr", "Wri", "Wii", "Br", "Bi"):
        assert rel_l2(getattr(m, k).grad.float().cpu().numpy(), getattr(mo, k).grad.numpy()) < tol, k
    if train:
        for k in ("RMr", "RVrr", "RVri"):
            assert getattr(m, k).dtype == dtype
            np.testing.assert_allclose(getattr(m, k).float().cpu().numpy(), getattr(mo, k).detach().numpy(),
                                       rtol=2 * tol, atol=2 * tol)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1.5e-2)])
def test_cbn_prelu_fused(dtype, tol, gpu_device):
    """DCCRN's block ends in CBN -> nn.PReLU() (one weight, dccrn.py:21,45): the PReLU runs
    inside the CBN kernels with its slope read on the device, and its weight gradient is a
    7th sum of the backward moments pass. Against fp64 CBN + PReLU on the CPU."""
    from sehip.complex_nn import ComplexBatchNorm2d, norm_act
    from oracle.complex_nn import ComplexBatchNorm2d as OCBN
    gen = torch.Generator().manual_seed(43)
    b, c, h, w = 3, 32, 17, 40
    x = (torch.randn(b, c, h, w, generator=gen) * 0.9).to(dtype)
    gy = torch.randn(b, c, h, w, generator=gen).to(dtype)
    mo = paramfill.fill_(OCBN(c), seed=10).to(dtype).double().train()
    po = torch.nn.PReLU().double()
    with torch.no_grad():
        po.weight.fill_(0.3)
    xo = x.double().requires_grad_(True)
    yo = po(mo(xo))
    yo.backward(gy.double())
    m = ComplexBatchNorm2d(c)
    m.load_state_dict({k: v.to(dtype) if v.is_floating_point() else v for k, v in mo.state_dict().items()})
    m = m.cuda().to(dtype).train()
    p = torch.nn.PReLU().cuda().to(dtype)
    with torch.no_grad():
        p.weight.fill_(0.3)
    xg = x.cuda().requires_grad_(True)
    y = norm_act(m, p, xg)
    y.backward(gy.cuda())
    assert rel_l2(y.detach().float().cpu().numpy(), yo.detach().numpy()) < tol
    assert rel_l2(xg.grad.float().cpu().numpy(), xo.grad.numpy()) < tol
    assert rel_l2(p.weight.grad.float().cpu().numpy(), po.weight.grad.numpy()) < tol
    for k in ("Wrr", "Wri", "Br"):
        assert rel_l2(getattr(m, k).grad.float().cpu().numpy(), getattr(mo, k).grad.numpy()) < tol, k


def test_cbn_fp32_module_on_bf16_input_promotes(gpu_device):
    """An fp32 ComplexBatchNorm2d fed bf16 activations (autocast-style) returns the promoted
    type, fp32, as the reference's pure-torch CBN does (complex_nn.py:300-320: Z * x + B
    against fp32 parameters), and is at least as close to an fp64 evaluation on the same
    (bf16-valued) input as the oracle's own mixed-precision run. Eval mode: in training the
    reference's fp32 running-stat lerp_ against bf16 batch means raises (complex_nn.py:250)."""
    from sehip.complex_nn import ComplexBatchNorm2d
    from oracle.complex_nn import ComplexBatchNorm2d as OCBN
    gen = torch.Generator().manual_seed(9)
    x = (torch.randn(2, 16, 9, 37, generator=gen) * 2 + 0.3).to(torch.bfloat16)
    m = paramfill.fill_(ComplexBatchNorm2d(16), seed=4).cuda().eval()
    y = m(x.cuda())
    assert y.dtype == torch.float32
    mo = paramfill.fill_(OCBN(16), seed=4).eval()
    yo = mo(x)
    assert yo.dtype == torch.float32
    y64 = paramfill.fill_(OCBN(16), seed=4).double().eval()(x.double())
    e_h = rel_l2(y.detach().cpu().numpy(), y64.detach().numpy())
    e_o = rel_l2(yo.detach().numpy(), y64.detach().numpy())
    assert e_h <= max(e_o, 1e-5), (e_h, e_o)
