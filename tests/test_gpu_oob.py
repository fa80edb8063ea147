"""Guard-region out-of-bounds regression. Every operand of a conv pass / the LSTM recurrence lives in the
middle of a buffer padded on both sides: inputs' padding is filled with 0 in
one run and NaN in another (an out-of-bounds READ changes the result or makes
it non-finite), outputs' padding with a sentinel (an out-of-bounds WRITE
changes it). Covers every conv math mode at FRCRN / DCCRN / DCUNet layer
shapes, and the se_lstm_bwd scalar-load fault fixed in round 1 (its shapes:
DCCRN's L 2, B 4, T 162, H 128 among them)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

PAD = 4 << 20          # floats on each side (16 MB)
SENT = 12345.0


def _padded(dev, shape, fill):
    n = 1
    for s in shape:
        n *= s
    buf = torch.full((n + 2 * PAD,), float(fill), device=dev)
    return buf, buf[PAD:PAD + n].view(shape)


def _guards_intact(buf, n):
    return bool(torch.all(buf[:PAD] == SENT)) and bool(torch.all(buf[PAD + n:] == SENT))


CONV_LAYERS = [   # (transposed, cin, cout, h, w, pad, output_pad, kernel, stride)
    (False, 2, 128, 320, 41, (0, 0), (0, 0), (5, 2), (2, 1)),     # FRCRN enc0
    (False, 128, 128, 40, 41, (0, 0), (0, 0), (5, 2), (2, 1)),    # FRCRN enc
    (True, 256, 128, 9, 40, (0, 0), (0, 0), (5, 2), (2, 1)),      # FRCRN dec
    (True, 256, 128, 77, 40, (0, 0), (0, 0), (5, 2), (2, 1)),
    (False, 2, 32, 256, 163, (2, 0), (0, 0), (5, 2), (2, 1)),     # DCCRN enc0
    (False, 128, 256, 32, 163, (2, 0), (0, 0), (5, 2), (2, 1)),
    (True, 512, 256, 8, 162, (2, 0), (1, 0), (5, 2), (2, 1)),     # DCCRN dec
    (True, 64, 2, 128, 162, (2, 0), (1, 0), (5, 2), (2, 1)),
    (False, 64, 64, 257, 126, (3, 2), (0, 0), (7, 5), (2, 2)),    # DCUNet-16
    (True, 256, 64, 33, 63, (3, 2), (0, 0), (7, 5), (2, 2)),
]


@pytest.mark.parametrize("math", ["f16x3", "bf16x3", "bf16x6", "bf16", "f32"])
@pytest.mark.parametrize("layer", CONV_LAYERS, ids=[f"{'T' if l[0] else 'C'}{l[1]}-{l[2]}h{l[3]}" for l in CONV_LAYERS])
def test_conv_passes_stay_in_bounds(layer, math, gpu_device):
    from sehip import functional as F, _native as N
    tr, cin, cout, h, w, pad, op, k, s = layer
    lib = N.lib()
    B = 2
    d = F.conv_desc((B, cin, h, w), cout, k, s, pad, (1, 1), op, tr, True)
    d.math = F._MATH_CODES[math]
    ho, wo = ctypes.c_int(), ctypes.c_int()
    assert lib.se_conv2d_out_shape(ctypes.byref(d), ctypes.byref(ho), ctypes.byref(wo)) == 0
    xs, ys = (B, cin, h, w), (B, cout, ho.value, wo.value)
    wsh = (cin // 2, cout // 2, *k) if tr else (cout // 2, cin // 2, *k)
    g = torch.Generator(device=gpu_device).manual_seed(0)
    x0, dy0 = torch.randn(xs, device=gpu_device, generator=g), torch.randn(ys, device=gpu_device, generator=g)
    wr0 = torch.randn(wsh, device=gpu_device, generator=g) * .05
    wi0 = torch.randn(wsh, device=gpu_device, generator=g) * .05
    ws = torch.empty(lib.se_conv2d_workspace_size(ctypes.byref(d)), dtype=torch.uint8, device=gpu_device)
    st = N.stream_of(x0)
    res, bad = {}, []
    for fill in (0.0, float("nan")):
        _, x = _padded(gpu_device, xs, fill); x.copy_(x0)
        _, dy = _padded(gpu_device, ys, fill); dy.copy_(dy0)
        _, wr = _padded(gpu_device, wsh, fill); wr.copy_(wr0)
        _, wi = _padded(gpu_device, wsh, fill); wi.copy_(wi0)
        outs = {n: _padded(gpu_device, shp, SENT) for n, shp in (("y", ys), ("dx", xs), ("dwr", wsh), ("dwi", wsh))}
        b = ctypes.byref(d)
        rc = [lib.se_conv2d_fwd(b, x.data_ptr(), wr.data_ptr(), wi.data_ptr(), None, None, outs["y"][1].data_ptr(),
                                ws.data_ptr(), ws.numel(), st),
              lib.se_conv2d_bwd_data(b, dy.data_ptr(), wr.data_ptr(), wi.data_ptr(), outs["dx"][1].data_ptr(),
                                     ws.data_ptr(), ws.numel(), st),
              lib.se_conv2d_bwd_weight(b, x.data_ptr(), dy.data_ptr(), outs["dwr"][1].data_ptr(),
                                       outs["dwi"][1].data_ptr(), None, None, ws.data_ptr(), ws.numel(), st)]
        torch.cuda.synchronize()
        assert rc == [0, 0, 0], rc
        for n, (buf, t) in outs.items():
            if not _guards_intact(buf, t.numel()):
                bad.append(f"out-of-bounds write around {n} (fill {fill})")
            res.setdefault(n, []).append(t.clone())
    for n, (a, c) in res.items():
        if not torch.isfinite(c).all() or not torch.equal(a, c):
            bad.append(f"out-of-bounds read into {n}")
    assert not bad, bad


@pytest.mark.parametrize("L,B,T,H", [(2, 4, 162, 128), (2, 2, 9, 128), (4, 6, 23, 64), (2, 128, 403, 128)])
def test_lstm_recurrence_stays_in_bounds(L, B, T, H, gpu_device):
    """se_lstm_fwd / se_lstm_bwd inside guard regions (bwd reads dgates back
    with scalar loads: the round-1 memory-aperture fault)."""
    from sehip import _native as N
    lib = N.lib()
    G = 4 * H
    g = torch.Generator(device=gpu_device).manual_seed(0)
    src = {"xproj": torch.randn(B * T * L * G, device=gpu_device, generator=g),
           "w_hh": torch.randn(L * G * H, device=gpu_device, generator=g) * 0.05,
           "dy": torch.randn(L * B * T * H, device=gpu_device, generator=g)}
    res, bad = {}, []
    for fill in (0.0, float("nan")):
        ins = {k: _padded(gpu_device, (v.numel(),), fill) for k, v in src.items()}
        for k, (_, t) in ins.items():
            t.copy_(src[k])
        _, zero = _padded(gpu_device, (H,), fill)
        zero.zero_()
        outs = {k: _padded(gpu_device, (n,), SENT) for k, n in (("h", L * B * T * H), ("c", L * B * T * H),
                                                                ("gates", L * B * T * G))}
        # dgates is read back (scalar loads) as well as written: its padding holds the probe fill
        outs["dgates"] = _padded(gpu_device, (L * B * T * G,), fill)
        st = N.stream_of(zero)
        rc1 = lib.se_lstm_fwd(ins["xproj"][1].data_ptr(), G, L * G, ins["w_hh"][1].data_ptr(), zero.data_ptr(),
                              outs["h"][1].data_ptr(), outs["c"][1].data_ptr(), outs["gates"][1].data_ptr(),
                              L, B, T, H, 0, st)
        rc2 = lib.se_lstm_bwd(ins["dy"][1].data_ptr(), ins["w_hh"][1].data_ptr(), outs["gates"][1].data_ptr(),
                              outs["c"][1].data_ptr(), outs["dgates"][1].data_ptr(), L, B, T, H, 0, st)
        torch.cuda.synchronize()
        assert rc1 == 0 and rc2 == 0, (rc1, rc2)
        for k, (buf, t) in outs.items():
            n = t.numel()
            if k == "dgates":
                guard = torch.cat([buf[:PAD], buf[PAD + n:]])
                ok = bool(torch.isnan(guard).all()) if fill != fill else bool((guard == fill).all())
            else:
                ok = _guards_intact(buf, n)
            if not ok:
                bad.append(f"out-of-bounds write around {k} (fill {fill})")
            res.setdefault(k, []).append(t.clone())
    for k, (a, c) in res.items():
        if not torch.isfinite(c).all() or not torch.equal(a, c):
            bad.append(f"out-of-bounds read into {k}")
    assert not bad, bad
