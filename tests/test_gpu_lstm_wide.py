"""Parity of the wide-hidden HIP LSTM recurrence (csrc/lstm_wide.hip via
se_lstm_wide_fwd / se_lstm_wide_bwd: H = 256 / 512 / 1024, a group of H/32
(H/16 at 1024) workgroups per sequence block exchanging h_t / dgates_t every
step) with torch.nn.LSTM, the op CARN calls (models/_2104_05267_carn.py:132,
nn.LSTM(512, 512, num_layers=2, batch_first=True)) and CRN calls
(models/_1809_01405_crn.py:90, nn.LSTM(1024, 1024, num_layers=2)).

Oracle: PyTorch's CPU nn.LSTM in fp32 at small shapes; at config 5's length
(one 30 s @ 48 kHz utterance = 9002 frames, H = 512, two layers) nn.LSTM on
the same GPU in fp32 (MIOpen). Tolerances: rel-L2 <= 5e-6 forward and
<= 2e-5 for gradients at small T (fp32 re-association of 256/512-term dots);
at T = 9002 the recurrence compounds rounding over 9002 steps on both sides,
so 1e-4 (forward) / 1e-3 (gradients)."""
import pytest
import torch

from conftest import rel_l2

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return rel_l2(a.detach().double().cpu().numpy(), b.detach().double().cpu().numpy())


def _grads(m):
    return {n: p.grad.detach().clone() for n, p in m.named_parameters()}


def _status(dev):
    from sehip import functional as F
    return F.lstm_wide_status(dev)


@pytest.mark.parametrize("H,I,B,T,bidir,layers", [
    (512, 512, 2, 33, False, 2),     # CARN's LSTM
    (256, 128, 3, 17, True, 1),      # bidirectional, odd batch
    (512, 64, 1, 1, False, 1),       # single step, one sequence
    (256, 256, 9, 12, False, 2),     # BS > 1 groups with a partial last block
    (512, 96, 40, 6, False, 1),      # many groups (BS = 8)
    (1024, 1024, 2, 9, False, 2),    # CRN's LSTM: 64-member groups over two XCD ids
    (1024, 48, 3, 6, True, 1),       # bidirectional at H = 1024
    (1024, 32, 20, 4, False, 1),     # three groups of 8 sequences
    (1024, 32, 40, 3, False, 1),     # more groups than fit at once: two batch-slice launches
])
def test_wide_lstm_matches_nn_lstm(gpu_device, H, I, B, T, bidir, layers):
    from sehip.complex_nn import stacked_lstms
    torch.manual_seed(0)
    mods = [torch.nn.LSTM(I, H, num_layers=layers, batch_first=True, bidirectional=bidir)]
    x = torch.randn(B, T, I)
    xr = x.clone().requires_grad_(True)
    ref = mods[0](xr)[0]
    gy = torch.randn_like(ref)
    (ref * gy).sum().backward()
    ref_g = _grads(mods[0])
    mods[0].zero_grad(set_to_none=True)
    dm = mods[0].to(gpu_device)
    xd = x.to(gpu_device).requires_grad_(True)
    out = stacked_lstms(xd, [dm], batch_first=True)[0]
    assert out.shape == ref.shape
    assert _rel(out, ref) < 5e-6
    (out * gy.to(gpu_device)).sum().backward()
    assert _rel(xd.grad, xr.grad) < 2e-5
    for n, p in dm.named_parameters():
        assert _rel(p.grad, ref_g[n]) < 2e-5, n
    assert _status(gpu_device) == 0


def test_lstm_module_states_and_fp16(gpu_device):
    """complex_nn.LSTM (nn.LSTM subclass): output and (h_n, c_n) as nn.LSTM;
    fp16 parameters / input (model.half(), config 5) compute in fp32."""
    from sehip.complex_nn import LSTM
    torch.manual_seed(1)
    ref = torch.nn.LSTM(64, 256, num_layers=2, batch_first=True, bidirectional=True)
    mod = LSTM(64, 256, num_layers=2, batch_first=True, bidirectional=True)
    mod.load_state_dict(ref.state_dict())
    x = torch.randn(2, 11, 64)
    yr, (hr, cr) = ref(x)
    mod = mod.to(gpu_device)
    y, (h, c) = mod(x.to(gpu_device))
    assert _rel(y, yr) < 5e-6 and _rel(h, hr) < 5e-6 and _rel(c, cr) < 5e-6
    assert h.shape == hr.shape and c.shape == cr.shape
    yh, _ = mod.half()(x.to(gpu_device).half())
    assert yh.dtype == torch.float16
    assert _rel(yh.float(), yr) < 2e-3
    assert _status(gpu_device) == 0


def test_carn_config5_length_against_gpu_nn_lstm(gpu_device):
    """Config 5's recurrence: 1 x 9002 frames, nn.LSTM(512, 512, 2 layers),
    forward and backward, against MIOpen fp32 on the same GPU."""
    from sehip.complex_nn import LSTM
    torch.manual_seed(2)
    ref = torch.nn.LSTM(512, 512, num_layers=2, batch_first=True).to(gpu_device)
    mod = LSTM(512, 512, num_layers=2, batch_first=True).to(gpu_device)
    mod.load_state_dict(ref.state_dict())
    x = torch.randn(1, 9002, 512, device=gpu_device) * 0.5
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)[0]
    gy = torch.randn_like(yr)
    (yr * gy).sum().backward()
    xd = x.clone().requires_grad_(True)
    y = mod(xd)[0]
    assert _rel(y, yr) < 1e-4
    (y * gy).sum().backward()
    assert _rel(xd.grad, xr.grad) < 1e-3
    rg = dict(ref.named_parameters())
    for n, p in mod.named_parameters():
        assert _rel(p.grad, rg[n].grad) < 1e-3, n
    assert _status(gpu_device) == 0
