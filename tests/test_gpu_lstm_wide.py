"""Parity of the wide-hidden HIP LSTM recurrence (csrc/lstm_wide.hip via
se_lstm_wide_fwd / se_lstm_wide_bwd: H = 256 / 512 / 1024, a group of H/32
(H/16 at 1024) workgroups per sequence block exchanging h_t / dgates_t every
step) with torch.nn.LSTM, the op CARN calls (models/_2104_05267_carn.py:132,
nn.LSTM(512, 512, num_layers=2, batch_first=True)) and CRN calls
(models/_1809_01405_crn.py:90, nn.LSTM(1024, 1024, num_layers=2)).

Oracle: PyTorch's CPU nn.LSTM in fp32 at small shapes; at config 5's length
(one 30 s @ 48 kHz utterance = 9002 frames, H = 512, two layers) the CPU
nn.LSTM in fp64, with the CPU fp32 run's own error as the bar. Tolerances: rel-L2 <= 5e-6 forward and
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


@pytest.mark.timeout(400)
def test_carn_config5_length_against_cpu_fp64(gpu_device):
    """Config 5's recurrence: 1 x 9002 frames (one 30 s @ 48 kHz utterance),
    nn.LSTM(512, 512, 2 layers) (carn.py:132), forward and backward, against the
    CPU nn.LSTM in fp64. Bar: within 2x the CPU fp32 nn.LSTM's own error against
    the same fp64 run (both compound fp32 rounding over 9002 steps), and the
    north-star 1e-4 for the forward."""
    from sehip.complex_nn import LSTM
    torch.manual_seed(2)
    ref = torch.nn.LSTM(512, 512, num_layers=2, batch_first=True)
    x = torch.randn(1, 9002, 512) * 0.5

    def run(m, xin, gy=None):
        xin = xin.clone().requires_grad_(True)
        y = m(xin)[0]
        gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(3)) if gy is None else gy
        (y * gy.to(y.device, y.dtype)).sum().backward()
        return y.detach().double().cpu(), xin.grad.double().cpu(), \
            {n: p.grad.double().cpu() for n, p in m.named_parameters()}, gy

    m64 = torch.nn.LSTM(512, 512, num_layers=2, batch_first=True)
    m64.load_state_dict(ref.state_dict())
    y64, dx64, g64, gy = run(m64.double(), x.double())
    y32, dx32, g32, _ = run(ref, x, gy)
    mod = LSTM(512, 512, num_layers=2, batch_first=True)
    mod.load_state_dict(ref.state_dict())
    yh, dxh, gh, _ = run(mod.to(gpu_device), x.to(gpu_device), gy)
    e = lambda a, b: ((a - b).norm() / b.norm()).item()
    print(f"9002-frame H=512 LSTM vs fp64: y hip {e(yh, y64):.2e} cpu32 {e(y32, y64):.2e}; "
          f"dx hip {e(dxh, dx64):.2e} cpu32 {e(dx32, dx64):.2e}; "
          + " ".join(f"{n} {e(gh[n], g64[n]):.1e}/{e(g32[n], g64[n]):.1e}" for n in g64))
    assert e(yh, y64) < 1e-4 and e(yh, y64) < 2 * e(y32, y64) + 1e-7
    assert e(dxh, dx64) < 2 * e(dx32, dx64) + 1e-7
    for n in g64:
        assert e(gh[n], g64[n]) < 2 * e(g32[n], g64[n]) + 1e-7, n
    assert _status(gpu_device) == 0


def test_wide_lstm_two_streams_concurrently(gpu_device):
    """Two wide-LSTM launches on different streams at once: each (device, stream)
    has its own group counters, so the launches cannot reset or advance each
    other's barriers; both match a serial run bit for bit."""
    from sehip import functional as F
    torch.manual_seed(4)
    L, B, T, H, I = 1, 2, 40, 256, 64
    args = [(torch.randn(B, T, I, device=gpu_device), torch.randn(L, 4 * H, I, device=gpu_device) * 0.05,
             torch.randn(L, 4 * H, H, device=gpu_device) * 0.05) for _ in range(2)]
    serial = [F.lstm_layer(x, wi, wh) for x, wi, wh in args]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(gpu_device) for _ in range(2)]
    outs = [None, None]
    for i, st in enumerate(streams):
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            outs[i] = F.lstm_layer(*args[i])
    for st in streams:
        torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    for a, b in zip(outs, serial):
        assert torch.equal(a, b)
    F.lstm_wide_poll(block=True)
    assert _status(gpu_device) == 0


def test_wide_lstm_timeout_raises(gpu_device):
    """A wide launch whose status word reports a barrier timeout makes the next
    poll (before the next wide launch, after every train_step) raise instead of
    letting NaN outputs through silently. The status word is set by hand here."""
    from sehip import _native as N
    from sehip import functional as F
    x = torch.randn(1, 3, 16, device=gpu_device)
    wi = torch.randn(1, 1024, 16, device=gpu_device) * 0.05
    wh = torch.randn(1, 1024, 256, device=gpu_device) * 0.05
    F.lstm_layer(x, wi, wh)
    F.lstm_wide_poll(block=True)
    _, status = F._wide_ws(x.device, N.stream_of(x))
    status.fill_(1)
    try:
        F.lstm_layer(x, wi, wh)
        with pytest.raises(F.LstmWideTimeout):
            F.lstm_wide_poll(block=True)
    finally:
        status.zero_()
        F._WIDE_PENDING.clear()
