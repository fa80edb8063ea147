"""se_complex_join(_bwd) (the FRCRN decoder's align + complex_concat,
frcrn.py:93-100) against the reference formulation on the CPU: forward and
both gradients must be bit-identical (pure data movement)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(x, s):
    from oracle.complex_nn import complex_concat
    if x.shape[-1] > s.shape[-1]:
        x = x[..., :-1]
    if x.shape[-2] < s.shape[-2]:
        x = torch.nn.functional.pad(x, (0, 0, 0, 1))
    return complex_concat([x, s], dim=1)


JOINED = [   # (x shape, skip shape): decoder state vs skip, FRCRN alignments
    ((2, 64, 9, 38), (2, 64, 9, 37)),            # time crop
    ((2, 64, 8, 38), (2, 64, 9, 37)),            # time crop + frequency pad
    ((3, 64, 7, 21), (3, 64, 7, 21)),            # aligned
    ((2, 128, 17, 41), (2, 128, 17, 40)),        # FRCRN width (jh = 64)
]


@pytest.mark.parametrize("cout", [128, 64])
@pytest.mark.parametrize("math", ["f16x3", "bf16x3", "fwd=bf16x6,data=bf16x3,weight=bf16x3", "bf16", "f16", "f32"])
@pytest.mark.parametrize("xs,ss", JOINED)
def test_joined_conv_matches_materialised_join(gpu_device, xs, ss, math, cout):
    """The decoder convT over complex_join(x, skip) with the join folded into
    the GEMMs (se_conv2d_*_joined) gives bit-identical outputs and gradients to
    the materialised join + plain conv (same K order, same MFMA sequence); f32
    has no joined kernel and takes the materialising fallback. cout = 64: the
    weight-grad's gathered operand (dy, 64 channels) is not tap-uniform, so the
    joined weight-grad runs on the per-row tap table (DCCRN's 128 -> 64 / 64 -> 32
    decoder layers)."""
    from sehip import functional as F
    prev = F.get_conv_math()
    F.set_conv_math(math)
    try:
        torch.manual_seed(1)
        cin = 2 * xs[1]
        x, s = torch.randn(xs, device=gpu_device), torch.randn(ss, device=gpu_device)
        wr = (torch.randn(cin // 2, cout // 2, 5, 2, device=gpu_device) * 0.05)
        wi = (torch.randn(cin // 2, cout // 2, 5, 2, device=gpu_device) * 0.05)
        kw = dict(out_channels=cout, kernel=(5, 2), stride=(2, 1), transposed=True)
        outs = []
        for joined in (False, True):
            xa, sa = x.clone().requires_grad_(True), s.clone().requires_grad_(True)
            wra, wia = wr.clone().requires_grad_(True), wi.clone().requires_grad_(True)
            if joined:
                y = F.conv2d_joined(xa, sa, wra, wia, **kw)
            else:
                y = F.conv2d(F.complex_join(xa, sa), wra, wia, **kw)
            g = torch.randn(y.shape, device=gpu_device, generator=torch.Generator(gpu_device).manual_seed(5))
            y.backward(g)
            outs.append((y.detach(), xa.grad, sa.grad, wra.grad, wia.grad))
        torch.cuda.synchronize()
        for name, a, b in zip(("y", "dx", "dskip", "dwr", "dwi"), *outs):
            assert torch.equal(a, b), (math, name, (a - b).abs().max().item())
    finally:
        F.set_conv_math(prev)


JOIN_TOL = {"f32": 1e-5, "f16x3": 1e-5, "fwd=bf16x6,data=bf16x3,weight=bf16x3": 3e-5, "bf16x3": 3e-5}


@pytest.mark.parametrize("math", sorted(JOIN_TOL))
@pytest.mark.parametrize("xs,ss", [((2, 128, 17, 41), (2, 128, 17, 40)),     # dec3-like: time crop
                                   ((2, 128, 77, 41), (2, 128, 78, 40))])    # dec5-like: crop + freq pad
def test_joined_conv_vs_fp64_oracle(gpu_device, xs, ss, math):
    """The joined decoder passes (forward, both input gradients, both weight
    gradients) against the fp64 oracle of the reference's trim / pad /
    complex_concat + ComplexConvTranspose2d (frcrn.py:93-101), per MFMA form:
    fp32-class forms at 1e-5, the bf16x3 passes at 3e-5."""
    from oracle import complex_nn as O_cnn
    import paramfill
    from conftest import rel_l2
    from sehip import functional as F
    cin, cout = 2 * xs[1], 128
    m = paramfill.fill_(O_cnn.ComplexConvTranspose2d(cin, cout, (5, 2), stride=(2, 1), bias=False), seed=4).double()
    gen = torch.Generator().manual_seed(2)
    x = torch.randn(xs, generator=gen, dtype=torch.float64)
    s = torch.randn(ss, generator=gen, dtype=torch.float64)
    xo, so = x.clone().requires_grad_(True), s.clone().requires_grad_(True)
    yo = m(_ref(xo, so))
    g = torch.randn(yo.shape, generator=gen, dtype=torch.float64)
    yo.backward(g)
    ref = dict(y=yo.detach(), dx=xo.grad, ds=so.grad, dwr=m.real_conv.weight.grad, dwi=m.imag_conv.weight.grad)
    prev = F.get_conv_math()
    F.set_conv_math(math)
    try:
        xa = x.float().to(gpu_device).requires_grad_(True)
        sa = s.float().to(gpu_device).requires_grad_(True)
        wr = m.real_conv.weight.detach().float().to(gpu_device).requires_grad_(True)
        wi = m.imag_conv.weight.detach().float().to(gpu_device).requires_grad_(True)
        y = F.conv2d_joined(xa, sa, wr, wi, out_channels=cout, kernel=(5, 2), stride=(2, 1), transposed=True)
        y.backward(g.float().to(gpu_device))
        torch.cuda.synchronize()
        got = dict(y=y.detach(), dx=xa.grad, ds=sa.grad, dwr=wr.grad, dwi=wi.grad)
    finally:
        F.set_conv_math(prev)
    for k, r in ref.items():
        e = rel_l2(got[k].cpu().numpy(), r.numpy())
        print(math, xs, k, f"{e:.2e}")
        assert e < JOIN_TOL[math], (math, k, e)


def test_joined_entry_points_run_their_own_kernels(gpu_device):
    """bf16x3 / bf16x6 / bf16 have joined kernels (rc 0, no fallback); f32 reports
    SE_E_UNSUPPORTED so the host materialises the join."""
    import ctypes
    from sehip import functional as F, _native as N
    B, C, F_, T = 2, 64, 9, 37
    d = F.conv_desc((B, 2 * C, F_, T), 128, (5, 2), (2, 1), (0, 0), (1, 1), (0, 0), True, True)
    lib = N.lib()
    ho, wo = ctypes.c_int(), ctypes.c_int()
    lib.se_conv2d_out_shape(ctypes.byref(d), ctypes.byref(ho), ctypes.byref(wo))
    x = torch.randn(B, C, F_ - 1, T + 1, device=gpu_device)
    s = torch.randn(B, C, F_, T, device=gpu_device)
    w = torch.randn(C, 64, 5, 2, device=gpu_device)
    y = torch.empty(B, 128, ho.value, wo.value, device=gpu_device)
    ws = torch.empty(lib.se_conv2d_workspace_size(ctypes.byref(d)), dtype=torch.uint8, device=gpu_device)
    st = N.stream_of(y)
    for mode, want in (("bf16x3", 0), ("bf16x6", 0), ("bf16", 0), ("f16x3", 0), ("f32", -3)):
        d.math = F._MATH_CODES[mode]
        rc = lib.se_conv2d_fwd_joined(ctypes.byref(d), x.data_ptr(), F_ - 1, T + 1, s.data_ptr(), w.data_ptr(),
                                      w.data_ptr(), None, None, y.data_ptr(), ws.data_ptr(), ws.numel(), st)
        assert rc == want, (mode, rc)
    torch.cuda.synchronize()


@pytest.mark.parametrize("xs,ss", [
    ((2, 8, 7, 14), (2, 6, 7, 13)),      # time crop only (every decoder layer)
    ((2, 8, 6, 14), (2, 8, 7, 13)),      # crop + freq pad (157 -> 158 in FRCRN)
    ((3, 4, 5, 9), (3, 4, 5, 9)),        # already aligned (first decoder layer)
    ((1, 2, 4, 10), (1, 6, 5, 10)),      # pad only
])
def test_complex_join_matches_reference(gpu_device, xs, ss):
    from sehip import functional as F
    torch.manual_seed(0)
    x, s = torch.randn(xs), torch.randn(ss)
    xr, sr = x.clone().requires_grad_(True), s.clone().requires_grad_(True)
    yr = _ref(xr, sr)
    g = torch.randn_like(yr)
    (yr * g).sum().backward()
    xd, sd = x.to(gpu_device).requires_grad_(True), s.to(gpu_device).requires_grad_(True)
    yd = F.complex_join(xd, sd)
    assert torch.equal(yd.cpu(), yr.detach())
    (yd * g.to(gpu_device)).sum().backward()
    assert torch.equal(xd.grad.cpu(), xr.grad)
    assert torch.equal(sd.grad.cpu(), sr.grad)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("xs,ss", JOINED)
def test_complex_join_16bit_storage_bit_exact(gpu_device, xs, ss, dtype):
    """se_complex_join(_bwd) on bf16 / fp16 tensors (ABI 4 dtype argument; DCCRN's bf16
    decoder): the same bits as the reference formulation's crop / pad / complex_concat in
    that dtype, forward and both gradients."""
    from sehip import functional as F
    torch.manual_seed(3)
    x = torch.randn(xs).to(dtype)
    s = torch.randn(ss).to(dtype)
    xr, sr = x.clone().requires_grad_(True), s.clone().requires_grad_(True)
    yr = _ref(xr, sr)
    g = torch.randn(yr.shape).to(dtype)
    yr.backward(g)
    xd, sd = x.to(gpu_device).requires_grad_(True), s.to(gpu_device).requires_grad_(True)
    yd = F.complex_join(xd, sd)
    yd.backward(g.to(gpu_device))
    assert yd.dtype == dtype and xd.grad.dtype == dtype
    assert torch.equal(yd.detach().cpu(), yr.detach())
    assert torch.equal(xd.grad.cpu(), xr.grad) and torch.equal(sd.grad.cpu(), sr.grad)


CAT_JOINED = [   # (x shape, skip shape, kernel, stride, padding): DCUNet decoder alignments
    ((2, 64, 8, 20), (2, 64, 9, 21), (5, 3), (2, 1), (2, 1)),     # x padded in both dims
    ((2, 64, 9, 21), (2, 64, 9, 21), (5, 3), (2, 2), (2, 1)),     # aligned
    ((1, 128, 16, 31), (1, 128, 17, 33), (7, 5), (2, 2), (3, 2)), # DCUNet-16 width (jh = 64)
    ((2, 128, 8, 20), (2, 128, 9, 21), (5, 3), (2, 1), (2, 1), 64),   # 64 outputs (DCUNet-16 dec.)
    ((2, 64, 8, 20), (2, 64, 9, 21), (5, 3), (2, 1), (2, 1), 32),     # 32 outputs
    ((2, 64, 16, 31), (2, 64, 17, 33), (7, 5), (2, 2), (3, 2), 2),   # DCUNet-16 mask layer: stencil
]


def _cat_ref(x, s):
    """dcunet.py:89-93: x zero-padded to the skip's grid, then a plain torch.cat."""
    if x.shape != s.shape:
        x = torch.nn.functional.pad(x, (0, s.shape[3] - x.shape[3], 0, s.shape[2] - x.shape[2]))
    return torch.cat([x, s], dim=1)


def _joined_pair(gpu_device, xs, ss, kernel, stride, padding, cat, dtype, cout=128):
    """(y, dx, dskip, dwr, dwi) of the materialised join + plain conv and of the joined
    conv (se_conv2d_*_joined), same inputs, the storage type dtype throughout."""
    from sehip import functional as F
    torch.manual_seed(1)
    cin = 2 * xs[1]
    x, s = torch.randn(xs, device=gpu_device).to(dtype), torch.randn(ss, device=gpu_device).to(dtype)
    wr = (torch.randn(cin // 2, cout // 2, *kernel, device=gpu_device) * 0.05).to(dtype)
    wi = (torch.randn(cin // 2, cout // 2, *kernel, device=gpu_device) * 0.05).to(dtype)
    kw = dict(out_channels=cout, kernel=kernel, stride=stride, padding=padding, transposed=True)
    outs = []
    for joined in (False, True):
        xa, sa = x.clone().requires_grad_(True), s.clone().requires_grad_(True)
        wra, wia = wr.clone().requires_grad_(True), wi.clone().requires_grad_(True)
        if joined:
            y = F.conv2d_joined(xa, sa, wra, wia, cat=cat, **kw)
        else:
            y = F.conv2d(_cat_ref(xa, sa) if cat else F.complex_join(xa, sa), wra, wia, **kw)
        g = torch.randn(y.shape, device=gpu_device, generator=torch.Generator(gpu_device).manual_seed(5)).to(dtype)
        y.backward(g)
        outs.append((y.detach(), xa.grad, sa.grad, wra.grad, wia.grad))
    torch.cuda.synchronize()
    return outs


@pytest.mark.parametrize("math", ["f16x3", "bf16x3", "bf16"])
@pytest.mark.parametrize("case", CAT_JOINED)
def test_cat_joined_conv_matches_materialised_cat(gpu_device, case, math):
    """DCUNet's decoder join (torch.cat order, x padded to the skip's grid in both
    dimensions, se_conv2d_desc.join_cat) folded into the GEMMs: outputs and all four
    gradients bit-identical to pad + torch.cat + the plain conv."""
    from sehip import functional as F
    prev = F.get_conv_math()
    F.set_conv_math(math)
    try:
        xs, ss, kernel, stride, padding = case[:5]
        cout = case[5] if len(case) > 5 else 128
        ref, got = _joined_pair(gpu_device, xs, ss, kernel, stride, padding, True, torch.float32, cout)
        for name, a, b in zip(("y", "dx", "dskip", "dwr", "dwi"), ref, got):
            assert a.shape == b.shape and torch.equal(a, b), (math, name, (a - b).abs().max().item())
    finally:
        F.set_conv_math(prev)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("cat", [False, True])
@pytest.mark.parametrize("cout", [128, 64])
def test_joined_conv_16bit_storage_matches_materialised(gpu_device, dtype, cat, cout):
    """16-bit storage (model.to(bfloat16) / .half(): BASELINE configs 2 / 3) on the joined
    GEMMs, the one-term MFMA of the storage format reading and writing x, s, dx and ds as
    they are: bit-identical to materialise-then-conv in the same storage type, for the
    complex_concat join (DCCRN) and the torch.cat join (DCUNet)."""
    from sehip import functional as F
    if cat:
        xs, ss, k, st, p = (2, 64, 8, 20), (2, 64, 9, 21), (5, 3), (2, 1), (2, 1)
    else:
        xs, ss, k, st, p = (2, 64, 8, 22), (2, 64, 9, 21), (5, 2), (2, 1), (2, 0)
    n0 = F.NATIVE16_CALLS[0]
    ref, got = _joined_pair(gpu_device, xs, ss, k, st, p, cat, dtype, cout)
    assert F.NATIVE16_CALLS[0] > n0   # the joined form ran natively, not on fp32 copies
    for name, a, b in zip(("y", "dx", "dskip", "dwr", "dwi"), ref, got):
        assert a.dtype == dtype and b.dtype == dtype
        assert a.shape == b.shape and torch.equal(a, b), (dtype, cat, name, (a.float() - b.float()).abs().max().item())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_mask_layer_join_runs_on_the_chunked_stencil(gpu_device, dtype, monkeypatch):
    """DCUNet's 2-output mask layer over its decoder join (dcunet.py:89-93 + the final convT):
    the forward gathers x (zero-padded) and the skip straight into the chunked stencil's LDS
    tiles, no materialised torch.cat; bit-identical to pad + cat + the plain conv in the
    storage type, gradients included (the weight-grad of N = 2 materialises its join)."""
    from sehip import functional as F
    calls = []
    raw = F._join_raw
    monkeypatch.setattr(F, "_join_raw", lambda *a, **k: calls.append(1) or raw(*a, **k))
    torch.manual_seed(2)
    x = torch.randn(2, 64, 16, 31, device=gpu_device).to(dtype)
    s = torch.randn(2, 64, 17, 33, device=gpu_device).to(dtype)
    wr = (torch.randn(64, 1, 7, 5, device=gpu_device) * 0.05).to(dtype)
    wi = (torch.randn(64, 1, 7, 5, device=gpu_device) * 0.05).to(dtype)
    kw = dict(out_channels=2, kernel=(7, 5), stride=(2, 2), padding=(3, 2), transposed=True)
    with torch.no_grad():
        y = F.conv2d_joined(x, s, wr, wi, cat=True, **kw)
        y_ref = F.conv2d(_cat_ref(x, s), wr, wi, **kw)
    assert not calls, "the mask layer's joined forward materialised the cat"
    assert torch.equal(y, y_ref), (y.float() - y_ref.float()).abs().max().item()
    ref, got = _joined_pair(gpu_device, (2, 64, 16, 31), (2, 64, 17, 33), (7, 5), (2, 2), (3, 2), True, dtype, 2)
    for name, a, b in zip(("y", "dx", "dskip", "dwr", "dwi"), ref, got):
        assert a.shape == b.shape and torch.equal(a, b), (dtype, name, (a.float() - b.float()).abs().max().item())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_complex_concat_join_on_the_chunked_stencil(gpu_device, dtype, monkeypatch):
    """DCCRN's last decoder layer (2 output channels over the complex_concat join,
    _2008_00264_dccrn.py:106-117; stride (2, 1), kernel (5, 2), x one frame wider than the
    skip): the forward gathers x and the skip straight into the chunked stencil's LDS tiles in
    complex_concat's chunk order (round 6; torch.cat order only before), no materialised join;
    bit-identical to complex_join + the plain conv, gradients included."""
    from sehip import functional as F
    calls = []
    raw = F._join_raw
    monkeypatch.setattr(F, "_join_raw", lambda *a, **k: calls.append(1) or raw(*a, **k))
    torch.manual_seed(4)
    x = torch.randn(2, 32, 9, 24, device=gpu_device).to(dtype)
    s = torch.randn(2, 32, 9, 23, device=gpu_device).to(dtype)
    wr = (torch.randn(32, 1, 5, 2, device=gpu_device) * 0.05).to(dtype)
    wi = (torch.randn(32, 1, 5, 2, device=gpu_device) * 0.05).to(dtype)
    kw = dict(out_channels=2, kernel=(5, 2), stride=(2, 1), padding=(2, 0), output_padding=(1, 0),
              transposed=True)
    with torch.no_grad():
        y = F.conv2d_joined(x, s, wr, wi, **kw)
        y_ref = F.conv2d(F.complex_join(x, s), wr, wi, **kw)
    assert not calls, "the joined forward materialised the join"
    assert torch.equal(y, y_ref), (y.float() - y_ref.float()).abs().max().item()
