"""CPU-only checks of the C-ABI library: it loads, exports every symbol
include/sehip.h declares, and its host-side planning/validation entry points
(no kernel launches) behave like the reference's shape rules."""
import ctypes
import os

import pytest
import torch

from sehip import _native as N
from sehip import functional as F


def test_library_exports_header_symbols():
    lib = N.lib()
    syms = N.header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), f"libsehip.so does not export {s}"
    assert N.MISSING == []
    assert lib.se_abi_version() == N.ABI_VERSION


def test_strerror():
    lib = N.lib()
    assert lib.se_strerror(0) == b"ok"
    for code in (-1, -2, -3, -4, -5):
        assert lib.se_strerror(code) not in (b"ok", b"unknown sehip error")
    assert lib.se_strerror(-99) == b"unknown sehip error"


CONV_GEOMS = [
    # (transposed, x shape, cout, kernel, stride, padding, dilation, output_padding)
    (False, (2, 2, 320, 404), 128, (5, 2), (2, 1), (0, 0), (1, 1), (0, 0)),     # FRCRN enc0
    (False, (3, 8, 17, 11), 6, (5, 3), (2, 2), (2, 1), (1, 1), (0, 0)),
    (False, (1, 4, 9, 10), 2, (7, 7), (1, 1), (3, 3), (1, 1), (0, 0)),         # CCBAM k7
    (False, (1, 6, 20, 30), 4, (3, 3), (1, 2), (1, 1), (2, 1), (0, 0)),        # dilation
    (True, (2, 256, 77, 403), 128, (5, 2), (2, 1), (0, 0), (1, 1), (0, 0)),    # FRCRN dec
    (True, (2, 8, 6, 7), 6, (5, 2), (2, 1), (2, 0), (1, 1), (1, 0)),           # DCCRN dec
    (True, (2, 8, 6, 5), 6, (5, 3), (2, 2), (2, 1), (1, 1), (0, 0)),           # DCUNet dec
    (True, (1, 4, 5, 7), 2, (1, 3), (2, 1), (0, 1), (1, 1), (1, 0)),           # CARN-like k1 s2
]


@pytest.mark.parametrize("g", CONV_GEOMS)
def test_conv_out_shape_matches_torch(g):
    tr, xs, cout, k, s, p, d, op = g
    desc = F.conv_desc(xs, cout, k, s, p, d, op, tr, True)
    ho, wo = ctypes.c_int(), ctypes.c_int()
    assert N.lib().se_conv2d_out_shape(ctypes.byref(desc), ctypes.byref(ho), ctypes.byref(wo)) == 0
    cls = torch.nn.ConvTranspose2d if tr else torch.nn.Conv2d
    kw = dict(stride=s, padding=p, dilation=d)
    if tr:
        kw["output_padding"] = op
    ref = cls(xs[1], cout, k, bias=False, **kw)(torch.zeros(xs)).shape
    assert (ho.value, wo.value) == tuple(ref[2:])
    assert N.lib().se_conv2d_workspace_size(ctypes.byref(desc)) > 0


def test_conv_argument_errors_need_no_gpu():
    lib = N.lib()
    d = F.conv_desc((1, 3, 8, 8), 4, (3, 3), (1, 1), (1, 1), (1, 1), (0, 0), False, True)
    # odd channel count with complex weights
    assert lib.se_conv2d_out_shape(ctypes.byref(d), None, None) == -2
    d = F.conv_desc((1, 4, 8, 8), 4, (3, 3), (0, 1), (1, 1), (1, 1), (0, 0), False, True)
    assert lib.se_conv2d_out_shape(ctypes.byref(d), None, None) == -1   # stride 0
    d = F.conv_desc((1, 4, 8, 8), 4, (3, 3), (1, 1), (1, 1), (1, 1), (0, 0), False, True)
    assert lib.se_conv2d_fwd(ctypes.byref(d), None, None, None, None, None, None, None, 0, None) == -1
    d = F.conv_desc((1, 4, 8, 8), 4, (9, 9), (1, 1), (1, 1), (1, 1), (0, 0), False, True)
    assert lib.se_conv2d_out_shape(ctypes.byref(d), None, None) == -3   # 81 taps > 64


def test_data_weight_image_validation_needs_no_gpu():
    """se_conv2d_prep_data_weights (ABI 5): sized per desc, and a split-fp16 image
    needs the caller's weight bound (it is baked in) -- rejected before any launch."""
    lib = N.lib()
    d = F.conv_desc((2, 180, 80, 40), 180, (5, 2), (2, 1), (2, 0), (1, 1), (0, 0), False, True)
    d.math = 4   # SE_MATH_F16X3, 180 input channels: the split tiles
    nb = lib.se_conv2d_data_weights_size(ctypes.byref(d))
    assert nb > 0
    fake = ctypes.c_void_p(256)   # never dereferenced: the call returns before launching
    assert lib.se_conv2d_prep_data_weights(ctypes.byref(d), fake, fake, fake, nb, None) == -1
    assert lib.se_conv2d_prep_data_weights(ctypes.byref(d), None, fake, fake, nb, None) == -1
    d.math = 0
    assert lib.se_conv2d_prep_data_weights(ctypes.byref(d), fake, fake, fake, 16, None) == -5   # image too small
    assert lib.se_conv2d_data_weights_size(None) == 0


@pytest.mark.parametrize("L,win,hop,nfft,center", [
    (64000, 320, 160, 640, 1), (64000, 400, 100, 512, 1), (32000, 512, 128, 512, 1),
    (16000, 320, 160, 320, 1), (1440000, 320, 160, 512, 1), (4000, 320, 160, 640, 0)])
def test_stft_num_frames_matches_conv1d(L, win, hop, nfft, center):
    pad = nfft // 2 if center else 0
    expect = (L + 2 * pad - win) // hop + 1
    assert N.lib().se_stft_num_frames(L, win, hop, nfft, center) == expect


def test_stft_validation_needs_no_gpu():
    lib = N.lib()
    # nfft with a factor 7 is not supported by the radix-2/3/4/5 FFT
    assert lib.se_stft_fwd(None, None, None, 1, 4000, 320, 160, 7 * 64, 1, 0, None, None, 0, None) == -3
    assert lib.se_stft_fwd(None, None, None, 1, 4000, 320, 160, 642, 1, 0, None, None, 0, None) == -3
    assert lib.se_stft_fwd(None, None, None, 1, 4000, 700, 160, 640, 1, 0, None, None, 0, None) == -1
    assert lib.se_istft_fwd(None, None, 1, 10, 320, 160, 640, 0, 10 ** 6, None, None, 0, None) == -2


def test_cbn_workspace():
    assert N.lib().se_cbn_workspace_size(64, 128, 77 * 403) > 0
    assert N.lib().se_cbn_workspace_size(0, 128, 10) == 0


def test_cpu_tensors_are_rejected():
    """The product path must fail loudly instead of falling back to the CPU."""
    from sehip.complex_nn import ComplexConv2d
    m = ComplexConv2d(4, 4, 3, padding=1)
    with pytest.raises(RuntimeError, match="GPU only"):
        m(torch.zeros(1, 4, 8, 8))


def test_lstm_validation_needs_no_gpu():
    lib = N.lib()
    assert lib.se_lstm_supported(128) == 1 and lib.se_lstm_supported(64) == 1
    assert lib.se_lstm_supported(96) == 0 and lib.se_lstm_supported(1024) == 0
    # (xproj, x_lstm, x_row, w_hh, zero, h, c, gates, L, B, T, H, rev_mask, stream)
    assert lib.se_lstm_fwd(None, 0, 512, None, None, None, None, None, 2, 128, 403, 96, 0, None) == -3
    assert lib.se_lstm_fwd(None, 0, 512, None, None, None, None, None, 0, 128, 403, 128, 0, None) == -1
    assert lib.se_lstm_fwd(None, 0, 512, None, None, None, None, None, 2, 128, 403, 128, 0, None) == -1
    assert lib.se_lstm_fwd(None, 0, 100, None, None, None, None, None, 2, 128, 403, 128, 0, None) == -1
    assert lib.se_lstm_bwd(None, None, None, None, None, 2, 128, 403, 64, 0, None) == -1
    assert lib.se_lstm_bwd(None, None, None, None, None, 2, 0, 403, 64, 0, None) == -1


def test_complex_lstm_state_dict_matches_reference_layout():
    """ComplexLSTM keeps the reference's parameter names (real_lstm / imag_lstm
    nn.LSTM modules) although the HIP path does not call them."""
    from sehip.complex_nn import ComplexLSTM
    from oracle.complex_nn import ComplexLSTM as O
    a = ComplexLSTM(256, 256, num_layers=2, batch_first=True).state_dict()
    b = O(256, 256, num_layers=2, batch_first=True).state_dict()
    assert list(a) == list(b)
    assert all(a[k].shape == b[k].shape for k in a)


@pytest.mark.parametrize("tr,xs,pb,pe", [
    (False, (2, 8, 20, 31), (0, 1), (0, 0)),      # FRCRN causal time pad folded into the conv
    (False, (1, 4, 9, 10), (2, 0), (1, 3)),
    (True, (2, 8, 6, 7), (1, 0), (0, 1)),
])
def test_asymmetric_padding_out_shape(tr, xs, pb, pe):
    k, s = (5, 2), (2, 1)
    desc = F.conv_desc(xs, 6, k, s, pb, (1, 1), (0, 0), tr, True, padding_end=pe)
    ho, wo = ctypes.c_int(), ctypes.c_int()
    assert N.lib().se_conv2d_out_shape(ctypes.byref(desc), ctypes.byref(ho), ctypes.byref(wo)) == 0
    if tr:   # convT with crop (pb, pe): full output cropped at begin/end
        full = torch.nn.ConvTranspose2d(xs[1], 6, k, stride=s, bias=False)(torch.zeros(xs)).shape
        ref = (full[2] - pb[0] - pe[0], full[3] - pb[1] - pe[1])
    else:    # conv of the zero-padded input
        xp = torch.nn.functional.pad(torch.zeros(xs), (pb[1], pe[1], pb[0], pe[0]))
        ref = tuple(torch.nn.Conv2d(xs[1], 6, k, stride=s, bias=False)(xp).shape[2:])
    assert (ho.value, wo.value) == tuple(ref)


def test_joined_conv_validation_needs_no_gpu():
    """se_conv2d_*_joined shape rules (frcrn.py:95-100 alignments) are checked
    on the host before any launch."""
    lib = N.lib()
    d = F.conv_desc((2, 256, 9, 37), 128, (5, 2), (2, 1), (0, 0), (1, 1), (0, 0), True, True)
    b = ctypes.byref(d)
    # x taller than the joined grid (only F.pad rows may be missing) -> SE_E_SHAPE
    assert lib.se_conv2d_fwd_joined(b, None, 10, 38, None, None, None, None, None, None, None, 0, None) == -2
    # x narrower than the joined grid (only x[..., :-1] crops) -> SE_E_SHAPE
    assert lib.se_conv2d_bwd_data_joined(b, None, None, None, None, 9, 36, None, None, 0, None) == -2
    # valid shapes, null pointers -> SE_E_ARG
    assert lib.se_conv2d_fwd_joined(b, None, 8, 38, None, None, None, None, None, None, None, 0, None) == -1
    assert lib.se_conv2d_bwd_weight_joined(b, None, 9, 37, None, None, None, None, None, None, None, 0,
                                           None) == -1
    # join chunks of 24 channels (not a multiple of 32): no joined kernel
    d2 = F.conv_desc((2, 96, 9, 37), 128, (5, 2), (2, 1), (0, 0), (1, 1), (0, 0), True, True)
    assert lib.se_conv2d_fwd_joined(ctypes.byref(d2), None, 9, 38, None, None, None, None, None, None, None, 0,
                                    None) == -3


def test_ccbam_and_join_validation_need_no_gpu():
    lib = N.lib()
    assert lib.se_ccbam_workspace_size(64, 128, 158 * 403) > 0
    assert lib.se_ccbam_workspace_size(64, 127, 100) == 0          # odd channel count
    # (x, mean, max, amax, B, C, HW, stream): odd C -> SE_E_SHAPE, null -> SE_E_ARG
    assert lib.se_ccbam_channel_pool(None, None, None, None, 2, 7, 10, None) == -2
    assert lib.se_ccbam_channel_pool(None, None, None, None, 2, 8, 10, None) == -1
    assert lib.se_ccbam_apply(None, None, None, None, 2, 8, 10, None, None) == -1
    ws = lib.se_ccbam_workspace_size(2, 8, 10)
    assert lib.se_ccbam_bwd_dca(None, None, None, None, None, 2, 8, 10, None, ws, None) == -1
    # join: (x, Cx, Fx, Tx, s, Cs, F, T, out, B, stream)
    assert lib.se_complex_join(None, 3, 4, 5, None, 4, 4, 5, None, 1, 0, None) == -2   # odd Cx
    assert lib.se_complex_join(None, 4, 4, 5, None, 4, 4, 5, None, 1, 0, None) == -1   # null pointers
    assert lib.se_complex_join_bwd(None, None, 4, 4, 5, None, 4, 0, 5, 1, 0, None) == -1


def test_python_call_sites_match_the_ctypes_signatures():
    """Every `<lib>.se_*(...)` call in the host package, the tools, bench.py and the tests
    passes as many arguments as its ctypes signature (and so the C header) declares: an ABI
    change that misses a call site fails here on the CPU instead of on the GPU box."""
    import ast
    import glob
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = (glob.glob(os.path.join(root, "speech-enhancement_amd", "sehip", "**", "*.py"), recursive=True)
             + glob.glob(os.path.join(root, "tools", "*.py")) + glob.glob(os.path.join(root, "tests", "*.py"))
             + [os.path.join(root, "bench.py")])
    bad, n = [], 0
    for f in files:
        for node in ast.walk(ast.parse(open(f).read())):
            if not (isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute)
                    and node.func.attr.startswith("se_") and node.func.attr in N._SIGNATURES):
                continue
            if any(isinstance(a, ast.Starred) for a in node.args) or node.keywords:
                continue
            n += 1
            want = len(N._SIGNATURES[node.func.attr][1])
            if len(node.args) != want:
                bad.append(f"{os.path.relpath(f, root)}:{node.lineno} {node.func.attr}: {len(node.args)} args, "
                           f"signature has {want}")
    assert n > 50, n
    assert not bad, bad
