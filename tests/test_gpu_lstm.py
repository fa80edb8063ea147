"""Parity of the persistent HIP LSTM recurrence (csrc/lstm.hip via
se_lstm_fwd / se_lstm_bwd) with torch.nn.LSTM, the op the reference's
ComplexLSTM calls (models/modules/complex_nn.py:115-145).

Oracle: PyTorch's CPU nn.LSTM in fp32 (small shapes, seconds) and
oracle/complex_nn.ComplexLSTM (the reference's four-call formulation).
At FRCRN's full size (64 utterances x 403 frames) the reference point is
nn.LSTM on the GPU in fp32 (MIOpen), the plain-PyTorch fp32 reference of
the same op. Tolerances: forward rel-L2 <= 2e-6, gradients <= 1e-5 (fp32
re-association only; the recurrence is a fixed 128-term dot per gate)."""
import pytest
import torch

from conftest import rel_l2

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return rel_l2(a.detach().double().cpu().numpy(), b.detach().double().cpu().numpy())


def _grads(m):
    return {n: p.grad.detach().clone() for n, p in m.named_parameters()}


@pytest.mark.parametrize("H,I,B,T,bidir,layers", [
    (128, 128, 4, 37, False, 2),      # FRCRN ComplexLSTM half (256 -> 256 complex)
    (64, 96, 6, 23, True, 1),         # DCCRN-like bidirectional
    (128, 64, 2, 5, True, 2),         # bidirectional, stacked layers, short sequence
    (64, 64, 2, 1, False, 1),         # single step
    (64, 32, 3, 7, False, 1),         # odd batch (partial last sequence group)
])
def test_stacked_lstms_match_nn_lstm(gpu_device, H, I, B, T, bidir, layers):
    from sehip.complex_nn import stacked_lstms
    torch.manual_seed(0)
    mods = [torch.nn.LSTM(I, H, num_layers=layers, batch_first=True, bidirectional=bidir) for _ in range(2)]
    x = torch.randn(B, T, I)
    # oracle: CPU nn.LSTM, each module separately
    xr = x.clone().requires_grad_(True)
    ref = [m(xr)[0] for m in mods]
    gys = [torch.randn_like(r) for r in ref]
    sum((r * g).sum() for r, g in zip(ref, gys)).backward()
    ref_g = [_grads(m) for m in mods]
    for m in mods:
        m.zero_grad(set_to_none=True)
    # HIP path
    dmods = [m.to(gpu_device) for m in mods]
    xd = x.to(gpu_device).requires_grad_(True)
    outs = stacked_lstms(xd, dmods, batch_first=True)
    for o, r in zip(outs, ref):
        assert o.shape == r.shape
        assert _rel(o, r) < 2e-6
    sum((o * g.to(gpu_device)).sum() for o, g in zip(outs, gys)).backward()
    assert _rel(xd.grad, xr.grad) < 1e-5
    for m, rg in zip(dmods, ref_g):
        for n, p in m.named_parameters():
            assert _rel(p.grad, rg[n]) < 1e-5, n


def test_lstm_layer_time_major_and_per_lstm_input(gpu_device):
    """batch_first=False input and a per-LSTM [L, B, T, I] layer input."""
    from sehip.complex_nn import stacked_lstms
    from sehip import functional as F
    torch.manual_seed(1)
    m = torch.nn.LSTM(32, 64, num_layers=1)
    x = torch.randn(9, 4, 32)                          # [T, B, I]
    ref = m(x)[0]
    out = stacked_lstms(x.to(gpu_device), [m.to(gpu_device)], batch_first=False)[0]
    assert _rel(out, ref) < 2e-6
    # per-LSTM inputs: two different sequences through two weight sets
    w_ih, w_hh = torch.randn(2, 256, 32) * 0.1, torch.randn(2, 256, 64) * 0.1
    xs = torch.randn(2, 4, 9, 32)
    h = F.lstm_layer(xs.to(gpu_device), w_ih.to(gpu_device), w_hh.to(gpu_device))
    for l in range(2):
        r = torch.nn.LSTM(32, 64, bias=False, batch_first=True)
        with torch.no_grad():
            r.weight_ih_l0.copy_(w_ih[l])
            r.weight_hh_l0.copy_(w_hh[l])
        assert _rel(h[l], r(xs[l])[0]) < 2e-6


def test_complex_lstm_matches_oracle(gpu_device):
    """sehip ComplexLSTM (stacked HIP recurrence) vs the oracle's four-call
    ComplexLSTM on the CPU, FRCRN configuration."""
    from oracle.complex_nn import ComplexLSTM as OracleCLSTM
    from sehip.complex_nn import ComplexLSTM
    torch.manual_seed(2)
    ref = OracleCLSTM(256, 256, num_layers=2, bidirectional=False, batch_first=True)
    mod = ComplexLSTM(256, 256, num_layers=2, bidirectional=False, batch_first=True)
    mod.load_state_dict(ref.state_dict())
    x = torch.randn(3, 41, 256)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    gy = torch.randn_like(yr)
    (yr * gy).sum().backward()
    mod = mod.to(gpu_device)
    xd = x.to(gpu_device).requires_grad_(True)
    yd = mod(xd)
    assert _rel(yd, yr) < 2e-6
    (yd * gy.to(gpu_device)).sum().backward()
    assert _rel(xd.grad, xr.grad) < 1e-5
    rg = dict(ref.named_parameters())
    for n, p in mod.named_parameters():
        assert _rel(p.grad, rg[n].grad) < 1e-5, n


def test_frcrn_size_against_gpu_nn_lstm(gpu_device):
    """FRCRN B=64 at 4 s: 128 stacked sequences x 403 frames, H = 128, two
    layers — against nn.LSTM (MIOpen fp32) on the same GPU."""
    from sehip.complex_nn import stacked_lstms
    torch.manual_seed(3)
    mods = [torch.nn.LSTM(128, 128, num_layers=2, batch_first=True).to(gpu_device) for _ in range(2)]
    x = torch.randn(128, 403, 128, device=gpu_device)
    xr = x.clone().requires_grad_(True)
    ref = [m(xr)[0] for m in mods]
    gys = [torch.randn_like(r) for r in ref]
    sum((r * g).sum() for r, g in zip(ref, gys)).backward()
    ref_g = [_grads(m) for m in mods]
    for m in mods:
        m.zero_grad(set_to_none=True)
    xd = x.clone().requires_grad_(True)
    outs = stacked_lstms(xd, mods, batch_first=True)
    for o, r in zip(outs, ref):
        assert _rel(o, r) < 2e-6
    sum((o * g).sum() for o, g in zip(outs, gys)).backward()
    assert _rel(xd.grad, xr.grad) < 1e-5
    for m, rg in zip(mods, ref_g):
        for n, p in m.named_parameters():
            assert _rel(p.grad, rg[n]) < 1e-5, n


def test_lstm_rejects_cpu_and_bad_shapes(gpu_device):
    from sehip import functional as F
    w_ih, w_hh = torch.zeros(1, 512, 16), torch.zeros(1, 512, 128)
    with pytest.raises(RuntimeError, match="GPU only"):
        F.lstm_layer(torch.zeros(2, 3, 16), w_ih, w_hh)
    with pytest.raises(ValueError):
        F.lstm_layer(torch.zeros(2, 3, 8, device=gpu_device), w_ih.to(gpu_device), w_hh.to(gpu_device))


@pytest.mark.parametrize("gemm", ["hip", "torch"])
def test_bias_grads_do_not_share_storage(gpu_device, monkeypatch, gemm):
    """b_ih and b_hh get the same gradient (sum over t of dgates) but must own separate
    storage, as nn.LSTM's do: shared storage made clip_grad_norm_'s in-place kernel scale
    it twice, racing (run-to-run differences in the LSTM biases after a train step)."""
    from sehip.complex_nn import ComplexLSTM
    from sehip.optim import clip_grad_norm_
    monkeypatch.setenv("SEHIP_LSTM_GEMM", gemm)
    torch.manual_seed(0)
    m = ComplexLSTM(64, 64, num_layers=1, batch_first=True).to(gpu_device)
    x = torch.randn(2, 7, 64, device=gpu_device)
    (m(x) ** 2).sum().backward()
    ptrs = [p.grad.untyped_storage().data_ptr() for p in m.parameters()]
    assert len(set(ptrs)) == len(ptrs)
    for lstm in (m.real_lstm, m.imag_lstm):
        g_ih, g_hh = lstm.bias_ih_l0.grad.clone(), lstm.bias_hh_l0.grad.clone()
        assert torch.equal(g_ih, g_hh)
    # clipping scales each gradient once
    ref = [p.grad.clone() for p in m.parameters()]
    norm = clip_grad_norm_(m.parameters(), 1e-3)
    s = 1e-3 / (norm.item() + 1e-6)
    for p, r in zip(m.parameters(), ref):
        assert torch.allclose(p.grad, r * s, rtol=1e-6, atol=0)
