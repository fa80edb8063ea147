"""Train-step glue on the HIP kernels (csrc/step.hip):
SI-SNR loss forward/backward with the pad / truncate folded in
(losses.py:62-84, utils.py:105-121), clip_grad_norm_ and AdamW
(trainer.py:216-221).

Oracle: oracle/train.py's restatement of the reference loss (checked against
the reference's train-step golden in test_oracle_golden.py), evaluated in
fp64 on the CPU with autograd; torch.nn.utils.clip_grad_norm_ and
torch.optim.AdamW (fp32, the ops the reference calls) on the same GPU for the
update. Tolerances: loss |d| <= 1e-5 |loss| + 1e-5 (fp64 sums vs fp32
rounding of the reference formula), gradients rel-L2 <= 1e-5; clip and AdamW
per element <= 1e-6 relative (same fp32 formulas, fp64 norm)."""
import os

import pytest
import torch

from conftest import rel_l2

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return rel_l2(a.detach().double().cpu().numpy(), b.detach().double().cpu().numpy())


@pytest.mark.parametrize("B,le,lt,zero_mean,chan", [
    (4, 16000, 16000, False, False),
    (3, 15840, 16000, False, True),     # estimate shorter: zero-padded (iSTFT length)
    (2, 16400, 16000, True, False),     # estimate longer: truncated; zero-mean form
    (1, 64000, 64000, False, False),
    (64, 64000, 64000, False, True),    # the bench batch, [B, 1, L] estimate
])
def test_sisnr_matches_oracle(gpu_device, B, le, lt, zero_mean, chan):
    from oracle.train import pad_or_truncate_wav as o_pad, si_snr_loss as o_loss
    from sehip.losses import si_snr_loss_aligned
    g = torch.Generator().manual_seed(B * 7 + le)
    tgt = torch.randn(B, lt, generator=g) * 0.3
    est = torch.randn(B, le, generator=g) * 0.2
    est[:, :min(le, lt)] += 0.8 * tgt[:, :min(le, lt)]
    e64 = est.double().requires_grad_(True)
    ref = o_loss(o_pad(e64, tgt.double()), tgt.double(), zero_mean=zero_mean)
    ref.backward()
    ed = est.to(gpu_device)
    ed = (ed[:, None] if chan else ed).requires_grad_(True)
    loss = si_snr_loss_aligned(ed, tgt.to(gpu_device), zero_mean=zero_mean)
    assert loss.shape == ()
    assert abs(loss.item() - ref.item()) <= 1e-5 * abs(ref.item()) + 1e-5
    loss.backward()
    gd = ed.grad.reshape(B, le)
    assert _rel(gd, e64.grad) < 1e-5
    if le > lt:
        assert torch.count_nonzero(gd[:, lt:]) == 0


def test_sisnr_drop_in_equal_lengths(gpu_device):
    """SI_SNR_loss (the reference's signature) on [B, L] CUDA fp32 uses the kernel
    and agrees with the plain-PyTorch fp32 formula."""
    from sehip.losses import SI_SNR_loss
    torch.manual_seed(0)
    t = torch.randn(8, 4000, device=gpu_device)
    e = (0.7 * t + 0.3 * torch.randn_like(t)).requires_grad_(True)
    loss = SI_SNR_loss(e, t)
    te = t.pow(2).sum(1, keepdim=True)
    e2 = e.detach().clone().requires_grad_(True)
    proj = (e2 * t).sum(1, keepdim=True) * t / te
    ref = -torch.mean(10 * torch.log10((proj.pow(2).sum(1) + 1e-8) / ((e2 - proj).pow(2).sum(1) + 1e-8)))
    assert abs(loss.item() - ref.item()) < 1e-5 * abs(ref.item())
    loss.backward()
    ref.backward()
    assert _rel(e.grad, e2.grad) < 1e-5


def _params(dev, seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(64, 128, 5, 2), (64,), (1,), (3, 7), (1024, 257), (2,)]
    ps = [torch.nn.Parameter(torch.randn(s, generator=g).to(dev)) for s in shapes]
    for p in ps:
        p.grad = (torch.randn(p.shape, generator=g) * 0.05).to(dev)
    return ps


def test_clip_grad_norm_matches_torch(gpu_device):
    from sehip.optim import clip_grad_norm_
    for max_norm in (0.5, 1e6):          # clipping and not clipping (coef clamped to 1)
        a, b = _params(gpu_device, 1), _params(gpu_device, 1)
        ta = torch.nn.utils.clip_grad_norm_(a, max_norm)
        tb = clip_grad_norm_(b, max_norm)
        assert abs(ta.item() - tb.item()) <= 1e-6 * ta.item()
        for pa, pb in zip(a, b):
            assert torch.allclose(pa.grad, pb.grad, rtol=1e-6, atol=0)


def test_adamw_matches_torch_over_steps(gpu_device):
    from sehip.optim import AdamW
    a, b = _params(gpu_device, 2), _params(gpu_device, 2)
    oa = torch.optim.AdamW(a, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2)
    ob = AdamW(b, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2)
    g = torch.Generator().manual_seed(3)
    for step in range(4):
        oa.step()
        ob.step()
        for pa, pb in zip(a, b):
            d = (pa - pb).abs().max().item()
            assert d <= 1e-6 * max(pa.abs().max().item(), 1.0), (step, d)
            ng = (torch.randn(pa.shape, generator=g) * 0.05).to(gpu_device)
            pa.grad.copy_(ng)
            pb.grad.copy_(ng)
    # state layout interchangeable with torch's
    sa, sb = oa.state_dict(), ob.state_dict()
    assert set(sa["state"][0]) == set(sb["state"][0])
    oc = torch.optim.AdamW(_params(gpu_device, 2), lr=1e-3)
    oc.load_state_dict(sb)
    assert float(oc.state_dict()["state"][0]["step"]) == 4.0


def test_train_step_uses_fused_glue(gpu_device):
    """make_optimizer returns the fused AdamW for CUDA fp32 models; over FRCRN's
    279 parameter tensors (the slot table of a real step) the fused clip +
    AdamW equals torch's on the same gradients; and train_step runs on it."""
    from sehip import models as M
    from sehip import optim
    from sehip.train import make_optimizer, train_step, ADAMW, CLIP_NORM
    from sehip.losses import si_snr_loss_aligned
    import paramfill
    noisy, clean = paramfill.structured_pair(2, 16000, seed=11)
    x, c = torch.from_numpy(noisy).to(gpu_device), torch.from_numpy(clean).to(gpu_device)
    m = paramfill.fill_(M.FRCRN(), seed=12).to(gpu_device).train()
    assert isinstance(make_optimizer(m), optim.AdamW)
    _, wav = m(x)
    si_snr_loss_aligned(wav, c).backward()
    pa = [torch.nn.Parameter(p.detach().clone()) for p in m.parameters()]
    pb = [torch.nn.Parameter(p.detach().clone()) for p in m.parameters()]
    for p, a, b in zip(m.parameters(), pa, pb):
        a.grad, b.grad = p.grad.clone(), p.grad.clone()
    na = torch.nn.utils.clip_grad_norm_(pa, CLIP_NORM)
    nb = optim.clip_grad_norm_(pb, CLIP_NORM)
    assert abs(na.item() - nb.item()) <= 1e-6 * na.item()
    oa, ob = torch.optim.AdamW(pa, **ADAMW), optim.AdamW(pb, **ADAMW)
    for _ in range(2):
        oa.step()
        ob.step()
    for a, b in zip(pa, pb):
        assert torch.allclose(a.grad, b.grad, rtol=1e-6, atol=0)
        assert (a - b).abs().max().item() <= 1e-6 * max(a.abs().max().item(), 1e-2)
    m2 = paramfill.fill_(M.FRCRN(), seed=12).to(gpu_device).train()
    loss = train_step(m2, make_optimizer(m2), x, c)
    assert torch.isfinite(loss)

def test_clip_grad_norm_error_if_nonfinite(gpu_device):
    """error_if_nonfinite=True: finite gradients clip as usual, a non-finite one raises
    (as torch.nn.utils.clip_grad_norm_)."""
    from sehip.optim import clip_grad_norm_
    a, b = _params(gpu_device, 5), _params(gpu_device, 5)
    ta = torch.nn.utils.clip_grad_norm_(a, 0.5, error_if_nonfinite=True)
    tb = clip_grad_norm_(b, 0.5, error_if_nonfinite=True)
    assert abs(ta.item() - tb.item()) <= 1e-6 * ta.item()
    b[1].grad[3] = float("inf")
    with pytest.raises(RuntimeError, match="non-finite"):
        clip_grad_norm_(b, 0.5, error_if_nonfinite=True)


def test_adamw_parameters_at_different_steps_match_torch(gpu_device):
    """A parameter without a gradient on some steps falls behind the others' step
    count; torch keeps a step per parameter, and so does sehip AdamW (one launch per
    distinct step count): both agree after every step."""
    from sehip.optim import AdamW
    a, b = _params(gpu_device, 6), _params(gpu_device, 6)
    oa = torch.optim.AdamW(a, lr=1e-3, weight_decay=1e-2)
    ob = AdamW(b, lr=1e-3, weight_decay=1e-2)
    g = torch.Generator().manual_seed(8)
    for step in range(5):
        for i, (pa, pb) in enumerate(zip(a, b)):
            if i == 1 and step in (0, 2):     # parameter 1 has no gradient on steps 0 and 2
                pa.grad = pb.grad = None
            else:
                ng = (torch.randn(pa.shape, generator=g) * 0.05).to(gpu_device)
                pa.grad, pb.grad = ng.clone(), ng.clone()
        oa.step()
        ob.step()
        for pa, pb in zip(a, b):
            d = (pa - pb).abs().max().item()
            assert d <= 1e-6 * max(pa.abs().max().item(), 1.0), (step, d)
    assert int(ob.state[b[1]]["step"]) == 3 and int(ob.state[b[0]]["step"]) == 5


def test_frcrn_mask_fused_vs_torch(gpu_device):
    """se_mask_fwd / _bwd (FRCRN's tanh mask x noisy, frcrn.py:140-152) against the
    reference's pad / tanh / mul / pad / reshape in torch on the same device: est equal
    to fp32 rounding (the same ops, tanhf vs torch's tanh), the gradient into h likewise,
    rows 0 and 1 of est exactly 0."""
    from sehip import functional as F
    tf = torch.nn.functional
    g = torch.Generator().manual_seed(5)
    B, half, T = 3, 321, 77
    h = torch.randn(B, 2, half - 2, T, generator=g).cuda().requires_grad_(True)
    spec = torch.randn(B, 2 * half, T, generator=g).cuda()
    est = F.complex_mask(h, spec, half)
    noisy = spec.view(B, 2, half, T)[:, :, 1:]
    h2 = h.detach().clone().requires_grad_(True)
    ref = tf.pad(torch.tanh(tf.pad(h2, (0, 0, 1, 0))) * noisy, (0, 0, 1, 0)).reshape(B, 2 * half, T)
    assert (est - ref).abs().max().item() <= 1e-6 * ref.abs().max().item()
    v = est.view(B, 2, half, T)
    assert torch.all(v[:, :, :2] == 0)
    gest = torch.randn(B, 2 * half, T, generator=g).cuda()
    est.backward(gest)
    ref.backward(gest)
    assert ((h.grad - h2.grad).norm() / h2.grad.norm()).item() < 1e-6


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_sisnr_16bit_storage(gpu_device, dtype):
    """ABI 10: a model.to(bfloat16) / .half() run's SI-SNR reads and writes its own dtype
    (no cast kernels): the loss within one rounding of the fp64 value of the same 16-bit
    inputs, the gradient within 2 roundings (rel-L2), zero past the target length."""
    from oracle.train import pad_or_truncate_wav as o_pad, si_snr_loss as o_loss
    from sehip.losses import si_snr_loss_aligned
    g = torch.Generator().manual_seed(9)
    B, le, lt = 4, 16100, 16000
    tgt = (torch.randn(B, lt, generator=g) * 0.3).to(dtype)
    est = (torch.randn(B, le, generator=g) * 0.2)
    est[:, :lt] += 0.8 * tgt.float()
    est = est.to(dtype)
    e64 = est.double().requires_grad_(True)
    ref = o_loss(o_pad(e64, tgt.double()), tgt.double())
    ref.backward()
    ed = est.to(gpu_device).requires_grad_(True)
    loss = si_snr_loss_aligned(ed, tgt.to(gpu_device))
    assert loss.dtype == dtype
    eps = torch.finfo(dtype).eps
    assert abs(loss.item() - ref.item()) <= eps * abs(ref.item()) + 1e-6
    loss.backward()
    assert ed.grad.dtype == dtype
    assert _rel(ed.grad, e64.grad) < 2 * eps
    assert torch.count_nonzero(ed.grad[:, lt:]) == 0


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_clip_and_adamw_16bit_match_torch(gpu_device, dtype):
    """ABI 10: clip_grad_norm_ + AdamW over bf16 / fp16 parameters against torch's own
    (foreach) implementations on the same tensors: the total norm within 1 rounding, every
    clipped gradient and every updated parameter / state element within 1 ulp of the format
    (torch rounds per foreach op; the kernel reproduces that sequence, the one freedom being
    the fp32 summation order of the norms)."""
    from sehip.optim import AdamW, clip_grad_norm_
    a = _params(gpu_device, 4)
    for p in a:
        p.data = p.data.to(dtype)
        p.grad = p.grad.to(dtype)
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    for p, q in zip(a, b):
        q.grad = p.grad.clone()
    ulp = lambda t: torch.finfo(dtype).eps * t.float().abs().clamp_min(torch.finfo(dtype).tiny)
    ta = torch.nn.utils.clip_grad_norm_(a, 0.5)
    tb = clip_grad_norm_(b, 0.5)
    assert abs(ta.float().item() - tb.item()) <= torch.finfo(dtype).eps * ta.float().item()
    for p, q in zip(a, b):   # the coefficient may differ by one rounding: <= 2 ulp per product
        assert ((p.grad.float() - q.grad.float()).abs() <= 2 * ulp(p.grad)).all()
        q.grad.copy_(p.grad)   # the optimizer comparison starts from identical gradients
    oa = torch.optim.AdamW(a, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, foreach=True)
    ob = AdamW(b, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2)
    g = torch.Generator().manual_seed(5)
    for step in range(3):
        oa.step()
        ob.step()
        for p, q in zip(a, b):
            assert q.dtype == dtype and ob.state[q]["exp_avg"].dtype == dtype
            bad = (p.float() - q.float()).abs() > ulp(p)
            assert not bad.any(), (step, p.float()[bad][:4].tolist(), q.float()[bad][:4].tolist(), bad.sum().item())
            for k in ("exp_avg", "exp_avg_sq"):
                sa, sb = oa.state[p][k].float(), ob.state[q][k].float()
                bad = (sa - sb).abs() > ulp(sa) + 1e-30
                assert not bad.any(), (step, k, sa[bad][:4].tolist(), sb[bad][:4].tolist(), bad.sum().item())
            ng = (torch.randn(p.shape, generator=g) * 0.05).to(dtype).to(gpu_device)
            p.grad.copy_(ng)
            q.grad.copy_(ng)
