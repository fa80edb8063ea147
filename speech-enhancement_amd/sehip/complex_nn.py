"""Complex layers on channel-stacked [re; im] tensors, HIP path.

Drop-in for /root/reference/models/modules/complex_nn.py: same class names,
constructor signatures and state_dict keys (``real_conv``/``imag_conv`` stay
real nn.Conv2d / nn.ConvTranspose2d parameter holders so utils.py:47-84
``initialize_params`` still finds them). Forward passes run the fused
kernels of csrc/cconv.hip and csrc/cbn.hip; the holders' own forward is never
called.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import functional as F
from . import glue


# ----------------------------------------------------------- layout helpers
def split_complex(x, dim=1):
    """complex_nn.py:18-30."""
    if isinstance(x, (tuple, list)):
        real, imag = x
        return real, imag
    if torch.is_complex(x):
        return x.real, x.imag
    if isinstance(x, torch.Tensor):
        return torch.chunk(x, 2, dim=dim)
    raise ValueError("Input must be a complex tensor or a tuple of real and imaginary tensors")


def merge_real_imag(x, real, imag, dim=1):
    """complex_nn.py:32-42: output in the container kind of x."""
    if isinstance(x, (tuple, list)):
        return [real, imag]
    if torch.is_complex(x):
        return torch.complex(real, imag)
    return torch.cat([real, imag], dim=dim)


def complex_concat(inputs, dim=1):
    """complex_nn.py:4-16: concat real halves, then imag halves."""
    halves = [torch.chunk(t, 2, dim=dim) for t in inputs]
    return torch.cat([h[0] for h in halves] + [h[1] for h in halves], dim=dim)


def _stacked(x):
    """(stacked tensor, rebuild fn) for any of the reference's complex containers."""
    if isinstance(x, (tuple, list)):
        return torch.cat([x[0], x[1]], dim=1), lambda y: list(torch.chunk(y, 2, dim=1))
    if torch.is_complex(x):
        return torch.cat([x.real, x.imag], dim=1), lambda y: torch.complex(*torch.chunk(y, 2, dim=1))
    return x, lambda y: y


def _f32(t):
    """fp16 / bf16 storage (the reference's model.half() / .to(bfloat16) configs)
    runs on the fp32-storage kernels; results go back in the caller's dtype."""
    return t if t is None or t.dtype == torch.float32 else t.float()


def _check_even(n, what):
    assert n % 2 == 0, f"{what} must be a factor of 2, current channels: {n}"
    return n // 2


# ---------------------------------------------------------------- conv ops
def _fold_pad(padding, input_pad, transposed):
    """(begin, end) conv padding equivalent to zero-padding the input by
    input_pad = (left, right, top, bottom) and then applying `padding`."""
    ph, pw = padding
    if not input_pad or not any(input_pad):
        return (ph, pw), None
    if transposed:
        raise NotImplementedError("sehip: input padding folds into plain convs only")
    left, right, top, bottom = input_pad
    return (ph + top, pw + left), (ph + bottom, pw + right)


class _FusedComplexConv(nn.Module):
    """Shared forward of ComplexConv2d / ComplexConvTranspose2d
    (complex_nn.py:44-65): one GEMM against the block weight instead of four
    real convs + sub/add/cat."""

    transposed = False
    # set by a model on its first conv, whose input is the raw spectrum (the batch's
    # whole level spread): its f16x3 GEMMs run exact fp32 (functional._pass_math)
    exact_fp32 = False

    def _geometry(self):
        c = self.real_conv
        if c.groups != 1:
            raise NotImplementedError("sehip complex conv: groups != 1")
        if getattr(c, "padding_mode", "zeros") != "zeros":
            raise NotImplementedError("sehip complex conv: padding_mode must be 'zeros'")
        if isinstance(c.padding, str):
            raise NotImplementedError("sehip complex conv: string padding")
        return c

    def forward(self, x, input_pad=None):
        """input_pad = (left, right, top, bottom) zeros around x (TF.pad order),
        folded into the conv's own padding instead of materialised (plain
        convs only)."""
        xs, rebuild = _stacked(x)
        c = self._geometry()
        begin, end = _fold_pad(c.padding, input_pad, self.transposed)
        y = F.conv2d(xs, c.weight, self.imag_conv.weight, c.bias, self.imag_conv.bias,
                     out_channels=2 * c.out_channels, kernel=c.kernel_size, stride=c.stride,
                     padding=begin, padding_end=end, dilation=c.dilation,
                     output_padding=getattr(c, "output_padding", (0, 0)),
                     transposed=self.transposed, exact=self.exact_fp32)
        return rebuild(y)

    def forward_joined(self, x, skip, cat=False):
        """self(complex_concat([align(x), skip])) with the FRCRN decoder's
        trim / pad / concat (frcrn.py:93-100) folded into the GEMMs; cat=True:
        self(torch.cat([F.pad(x, to skip's grid), skip])) (DCUNet, dcunet.py:89-93)."""
        c = self._geometry()
        return F.conv2d_joined(x, skip, c.weight, self.imag_conv.weight, c.bias, self.imag_conv.bias,
                               out_channels=2 * c.out_channels, kernel=c.kernel_size, stride=c.stride,
                               padding=c.padding, dilation=c.dilation,
                               output_padding=getattr(c, "output_padding", (0, 0)),
                               transposed=self.transposed, cat=cat)


class ComplexConv2d(_FusedComplexConv):
    """complex_nn.py:67-78."""

    def __init__(self, in_channels, out_channels, kernel_size, **kwargs):
        super().__init__()
        cin = _check_even(in_channels, "in_channels")
        cout = _check_even(out_channels, "out_channels")
        self.real_conv = nn.Conv2d(cin, cout, kernel_size, **kwargs)
        self.imag_conv = nn.Conv2d(cin, cout, kernel_size, **kwargs)


class ComplexConvTranspose2d(_FusedComplexConv):
    """complex_nn.py:80-91."""

    transposed = True

    def __init__(self, in_channels, out_channels, kernel_size, **kwargs):
        super().__init__()
        cin = _check_even(in_channels, "in_channels")
        cout = _check_even(out_channels, "out_channels")
        self.real_conv = nn.ConvTranspose2d(cin, cout, kernel_size, **kwargs)
        self.imag_conv = nn.ConvTranspose2d(cin, cout, kernel_size, **kwargs)


def real_conv2d(conv: nn.Module, x, input_pad=None):
    """A plain nn.Conv2d / nn.ConvTranspose2d evaluated by the same HIP GEMM
    (e.g. FRCRN's real final_conv, frcrn.py:115); input_pad as in
    _FusedComplexConv.forward. A conv flagged `sehip_exact_fp32` (a model's first,
    data-fed conv) runs exact fp32 where the mode is f16x3."""
    tr = isinstance(conv, nn.ConvTranspose2d)
    if conv.groups != 1 or isinstance(conv.padding, str):
        raise NotImplementedError("sehip real conv: groups / string padding")
    begin, end = _fold_pad(conv.padding, input_pad, tr)
    return F.conv2d(x, conv.weight, None, conv.bias, None, out_channels=conv.out_channels,
                    kernel=conv.kernel_size, stride=conv.stride, padding=begin, padding_end=end,
                    dilation=conv.dilation, output_padding=getattr(conv, "output_padding", (0, 0)),
                    transposed=tr, exact=getattr(conv, "sehip_exact_fp32", False))


# ------------------------------------------------------------- linear / LSTM
class ComplexLinear(nn.Module):
    """complex_nn.py:93-113 (separate real / imag linears, no cross terms) on the
    hand-written GEMM (sehip.linear: se_gemm fwd, input-, weight- and bias-grad).
    The real_linear / imag_linear nn.Linear modules are the parameter holders.
    feature_major_out: produce the output as the transposed view of a [B, out, T]
    storage (the same values and shape), for a consumer that transposes it back
    (DCCRN's LSTMBlock -> decoder hand-off, dccrn.py:169-171)."""

    feature_major_out = False

    def __init__(self, in_channels, out_channels, **kwargs):
        super().__init__()
        cin = _check_even(in_channels, "in_channels")
        cout = _check_even(out_channels, "out_channels")
        self.real_linear = nn.Linear(cin, cout, **kwargs)
        self.imag_linear = nn.Linear(cin, cout, **kwargs)

    def forward(self, x):
        from .linear import linear, linear_halves
        rl, il = self.real_linear, self.imag_linear
        if isinstance(x, torch.Tensor) and not torch.is_complex(x):
            # both halves of the last axis in place (complex_nn.py:106-113 without chunk / cat)
            return linear_halves(x, [rl.weight, il.weight], [rl.bias, il.bias], self.feature_major_out)
        re, im = split_complex(x, dim=-1)
        return merge_real_imag(x, linear(re, rl), linear(im, il), dim=-1)


# hidden sizes of the HIP recurrence: se_lstm_* (64, 128), se_lstm_wide_* (256, 512, 1024)
HIP_LSTM_HIDDEN = (64, 128, 256, 512, 1024)


def _wide_group_fits(m: nn.LSTM) -> bool:
    """The wide recurrence (H = 256 / 512 / 1024) runs one group of H/32 (H/16 at 1024)
    workgroups that must all be resident: a device with fewer CUs than one group runs
    nn.LSTM's own forward instead (se_lstm_wide_* would return SE_E_UNSUPPORTED)."""
    H = m.hidden_size
    if H not in (256, 512, 1024):
        return True
    p = next(m.parameters(), None)
    if p is None or not p.is_cuda:
        return True
    members = H // (16 if H == 1024 else 32)
    return torch.cuda.get_device_properties(p.device).multi_processor_count >= members


def _hip_lstm_ok(m: nn.LSTM) -> bool:
    return (m.proj_size == 0 and m.hidden_size in HIP_LSTM_HIDDEN
            and (m.dropout == 0 or not m.training) and m.mode == "LSTM" and _wide_group_fits(m))


def stacked_lstms(x, lstms, batch_first=True, with_state=False, raw=False):
    """Run several nn.LSTMs (same shape) over the same input x on the HIP
    recurrence, all of them in the same launches: per layer one projection
    GEMM, one se_lstm_fwd over every (LSTM, direction), and in backward one
    se_lstm_bwd. Returns one output per LSTM, shaped like nn.LSTM's output[0]
    (with_state: and per LSTM nn.LSTM's (h_n, c_n), [layers * dirs, B, H]).
    raw=True (unidirectional): the fp32 [len(lstms), B, T, H] output of the last layer
    as it is, for a consumer that reads it directly (ComplexLSTM's combine).
    The modules keep their own parameters (state_dict keys unchanged); their bf16 /
    fp16 weights are stacked in fp32 by one HIP copy per tensor (glue.stack), the
    recurrence runs in fp32 and the outputs come back in x's dtype (glue.contiguous)."""
    m0 = lstms[0]
    nd = 2 if m0.bidirectional else 1
    H = m0.hidden_size
    dt = x.dtype                                  # bf16 / fp16 models: fp32 recurrence, caller's dtype out
    xb = x if batch_first else x.transpose(0, 1)
    inp = glue.contiguous(xb, torch.float32)      # layer 0: [B, T, I] shared by every LSTM
    rev_mask = sum(1 << (i * nd + 1) for i in range(len(lstms))) if nd == 2 else 0
    out = None
    h_layers, c_layers = [], []
    f32 = torch.float32
    for k in range(m0.num_layers):
        sfx = [f"_l{k}", f"_l{k}_reverse"][:nd]
        w_ih = glue.stack([getattr(m, "weight_ih" + s) for m in lstms for s in sfx], f32)
        w_hh = glue.stack([getattr(m, "weight_hh" + s) for m in lstms for s in sfx], f32)
        b_ih = b_hh = None
        if m0.bias:
            b_ih = glue.stack([getattr(m, "bias_ih" + s) for m in lstms for s in sfx], f32)
            b_hh = glue.stack([getattr(m, "bias_hh" + s) for m in lstms for s in sfx], f32)
        h, c = F.lstm_layer(inp, w_ih, w_hh, b_ih, b_hh, rev_mask, with_cell=True)   # [len*nd, B, T, H]
        if with_state:
            h_layers.append(h)
            c_layers.append(c)
        Bn, T = h.shape[1], h.shape[2]
        if nd == 2:   # per LSTM: cat(forward, reverse) on features, fed to both directions
            out = h.view(len(lstms), 2, Bn, T, H).permute(0, 2, 3, 1, 4).reshape(len(lstms), Bn, T, 2 * H)
        else:
            out = h
        if k + 1 < m0.num_layers:
            if m0.dropout > 0 and m0.training:
                out = torch.nn.functional.dropout(out, m0.dropout, True)
            inp = out.repeat_interleave(nd, dim=0) if nd == 2 else out
    if raw and nd == 1 and not with_state:
        return out
    outs = [glue.contiguous(o, dt) for o in out.unbind(0)]
    outs = outs if batch_first else [o.transpose(0, 1) for o in outs]
    if not with_state:
        return outs
    # per LSTM: [layers * dirs, B, H] in nn.LSTM's (layer, direction) order; the last step in
    # processing order: t = T-1 forward, t = 0 reverse
    states = []
    for i in range(len(lstms)):
        hn = [hl[i * nd + d, :, -1 if d == 0 else 0] for hl in h_layers for d in range(nd)]
        cn = [cl[i * nd + d, :, -1 if d == 0 else 0] for cl in c_layers for d in range(nd)]
        states.append((glue.stack(hn, dt), glue.stack(cn, dt)))
    return outs, states


class LSTM(nn.LSTM):
    """torch.nn.LSTM (same constructor, parameters and state_dict keys) whose
    recurrence runs on the HIP kernels (stacked_lstms) when the configuration
    is covered: hidden 64 / 128 / 256 / 512 / 1024, no proj_size, no initial state,
    a dense [B, T, I] (batch_first) or [T, B, I] CUDA input. fp16 / bf16
    parameters and inputs (model.half()) compute in fp32 and return the
    caller's dtype. Anything else is nn.LSTM's own forward."""

    def forward(self, input, hx=None):
        if (hx is None and _hip_lstm_ok(self) and isinstance(input, torch.Tensor) and input.is_cuda
                and input.dim() == 3):
            outs, states = stacked_lstms(input, [self], batch_first=self.batch_first, with_state=True)
            return outs[0], states[0]
        return super().forward(input, hx)


class ComplexLSTM(nn.Module):
    """complex_nn.py:115-145. The reference makes four LSTM calls; the real
    and imaginary inputs are independent sequences through the SAME weights,
    so re and im are stacked on the batch axis, and real_lstm / imag_lstm run
    together in the stacked HIP recurrence (stacked_lstms): per layer one
    launch forward and one backward instead of MIOpen's per-time-step kernels.
    Configurations the HIP recurrence does not cover (hidden size other than
    64 / 128, proj_size) run each nn.LSTM once over the stacked batch."""

    # batch_first: return the output as the transposed view of a [B, 2H, T] storage (same
    # values and shape) for a caller that transposes it back (FRCRN, frcrn.py:137)
    feature_major_out = False

    def __init__(self, in_channels, hidden_channels, **kwargs):
        super().__init__()
        cin = _check_even(in_channels, "in_channels")
        hid = _check_even(hidden_channels, "hidden_channels")
        self.real_lstm = nn.LSTM(cin, hid, **kwargs)
        self.imag_lstm = nn.LSTM(cin, hid, **kwargs)
        self._bdim = 0 if kwargs.get("batch_first", False) else 1

    def forward(self, x):
        if (isinstance(x, torch.Tensor) and not torch.is_complex(x) and x.is_cuda and x.dim() == 3
                and _hip_lstm_ok(self.real_lstm) and not self.real_lstm.bidirectional):
            # re / im stacked on the batch axis in fp32 (one HIP copy), both LSTMs in the same
            # launches, the four outputs combined into (re, im) in x's dtype (one HIP pass)
            xb = x if self._bdim == 0 else x.transpose(0, 1)
            h = stacked_lstms(glue.stack_re_im(xb), [self.real_lstm, self.imag_lstm], batch_first=True, raw=True)
            out = glue.complex_lstm_combine(h, x.dtype, self.feature_major_out and self._bdim == 0)
            return out if self._bdim == 0 else out.transpose(0, 1)
        re, im = split_complex(x, dim=-1)
        both = torch.cat([re, im], dim=self._bdim)
        if _hip_lstm_ok(self.real_lstm):
            r_out, i_out = stacked_lstms(both, [self.real_lstm, self.imag_lstm],
                                         batch_first=self._bdim == 0)
        else:
            r_out = self.real_lstm(both)[0]
            i_out = self.imag_lstm(both)[0]
        rr, ir = torch.chunk(r_out, 2, dim=self._bdim)     # real_lstm(re), real_lstm(im)
        ri, ii = torch.chunk(i_out, 2, dim=self._bdim)     # imag_lstm(re), imag_lstm(im)
        return merge_real_imag(x, rr - ii, ri + ir, dim=-1)

    def flatten_parameters(self):
        self.real_lstm.flatten_parameters()
        self.imag_lstm.flatten_parameters()


# ------------------------------------------------------------- batch norm
class ComplexBatchNorm2d(nn.Module):
    """complex_nn.py:148-329 — whitening complex BN on the HIP kernels."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True,
                 track_running_stats=True, complex_axis=1):
        super().__init__()
        if complex_axis != 1:
            raise NotImplementedError("sehip ComplexBatchNorm2d: complex_axis must be 1")
        self.num_features = num_features // 2
        self.eps, self.momentum, self.affine = eps, momentum, affine
        self.track_running_stats, self.complex_axis = track_running_stats, complex_axis
        c = self.num_features
        for name in ("Wrr", "Wri", "Wii", "Br", "Bi"):
            if affine:
                setattr(self, name, nn.Parameter(torch.empty(c)))
            else:
                self.register_parameter(name, None)
        if track_running_stats:
            self.register_buffer("RMr", torch.zeros(c))
            self.register_buffer("RMi", torch.zeros(c))
            self.register_buffer("RVrr", torch.ones(c))
            self.register_buffer("RVri", torch.zeros(c))
            self.register_buffer("RVii", torch.ones(c))
            self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))
        else:
            for name in ("RMr", "RMi", "RVrr", "RVri", "RVii", "num_batches_tracked"):
                self.register_parameter(name, None)
        self.reset_parameters()

    def reset_running_stats(self):
        if self.track_running_stats:
            self.RMr.zero_(); self.RMi.zero_(); self.RVri.zero_()
            self.RVrr.fill_(1); self.RVii.fill_(1)
            self.num_batches_tracked.zero_()

    def reset_parameters(self):                               # complex_nn.py:202-209
        self.reset_running_stats()
        if self.affine:
            with torch.no_grad():
                self.Br.zero_(); self.Bi.zero_()
                self.Wrr.fill_(1); self.Wii.fill_(1)
                self.Wri.uniform_(-.9, +.9)

    def forward_act(self, x, act=F.ACT_NONE, slope=0.0, fork=False, prelu=None):
        """BN followed by a fused activation (LeakyReLU / ReLU, or the weight of a
        one-parameter nn.PReLU). fork=True returns (y, alias of y) for two consumers
        (see functional.complex_batch_norm). x may be fp32, bf16 or fp16 storage, with
        the module in the same dtype (model.to(bfloat16) / .half()). A module whose dtype
        differs from x's (e.g. an fp32 module fed bf16 activations under autocast) runs
        its kernels on x cast to the module dtype and returns the result in the promoted
        type of x and the parameters, as the reference's pure-torch CBN does (its
        `Zrr * xr + ... + Br` promotes against the fp32 parameters, complex_nn.py:300-320)."""
        mdt = _module_dtype(self, x.dtype)
        if mdt != x.dtype:
            y = self.forward_act(x.to(mdt), act, slope, False, None if prelu is None else prelu.to(mdt))
            y = y.to(torch.promote_types(x.dtype, mdt))
            return (y, y) if fork else y
        running = (self.RMr, self.RMi, self.RVrr, self.RVri, self.RVii) if self.track_running_stats else None
        training = self.training or not self.track_running_stats    # complex_nn.py:234
        return F.complex_batch_norm(
            x, self.Wrr, self.Wri, self.Wii, self.Br, self.Bi, running,
            self.num_batches_tracked if self.track_running_stats else None,
            training, self.eps, self.momentum, act, slope, fork, prelu)

    def forward(self, inputs):
        return self.forward_act(inputs)

    def extra_repr(self):
        return ("{num_features}, eps={eps}, momentum={momentum}, affine={affine}, "
                "track_running_stats={track_running_stats}".format(**self.__dict__))


def _module_dtype(m: nn.Module, default):
    for t in list(m.parameters(recurse=False)) + list(m.buffers(recurse=False)):
        if t is not None and t.is_floating_point():
            return t.dtype
    return default


def norm_act(norm: nn.Module, act: nn.Module, x, fork: bool = False):
    """act(norm(x)) with the activation fused into the CBN kernel when both are
    the kinds the kernel knows; otherwise the two modules are applied in turn.
    fork=True returns (y, y2) for two consumers of y: with the CBN kernel y2 is an
    alias whose gradient the CBN backward sums itself; otherwise y2 is y."""
    if isinstance(norm, ComplexBatchNorm2d):     # forward_act casts a dtype mismatch itself
        if isinstance(act, nn.LeakyReLU):
            return norm.forward_act(x, F.ACT_LEAKY, act.negative_slope, fork)
        if isinstance(act, nn.ReLU):
            return norm.forward_act(x, F.ACT_RELU, 0.0, fork)
        if isinstance(act, nn.Identity):
            return norm.forward_act(x, fork=fork)
        if isinstance(act, nn.PReLU) and act.weight.numel() == 1:
            return norm.forward_act(x, fork=fork, prelu=act.weight)   # DCCRN, dccrn.py:21,45
    y = act(norm(x))
    return (y, y) if fork else y


class ComplexPReLU(nn.Module):
    """complex_nn.py:337-357."""

    def __init__(self, **kwargs):
        super().__init__()
        self.real_prelu = nn.PReLU(**kwargs)
        self.imag_prelu = nn.PReLU(**kwargs)

    def forward(self, x):
        re, im = split_complex(x, dim=1)
        out_re = self.real_prelu(re) - self.imag_prelu(im)
        out_im = self.imag_prelu(re) + self.real_prelu(im)
        return merge_real_imag(x, out_re, out_im, dim=1)


ComplexReLU = nn.ReLU            # complex_nn.py:359
ComplexLeakyReLU = nn.LeakyReLU  # complex_nn.py:360


def mark_data_fed(block: nn.Module) -> nn.Module:
    """mark_data_fed_conv on every conv inside `block` (a model's first block)."""
    for m in block.modules():
        if isinstance(m, (_FusedComplexConv, nn.Conv2d, nn.ConvTranspose2d)):
            mark_data_fed_conv(m)
    return block


def mark_data_fed_conv(conv: nn.Module) -> nn.Module:
    """Flag a model's first conv (its input is the raw spectrum or magnitude, which
    carries the whole level spread of the batch; every later conv operand is a
    per-channel normalised activation or a gradient of one): its passes run exact
    fp32 where the conv math is the per-tensor-scaled f16x3. This conv is HBM-bound
    (Cin = 2), so exact products cost nothing measurable."""
    if isinstance(conv, _FusedComplexConv):
        conv.exact_fp32 = True
    else:   # (the real_conv / imag_conv holders of a fused conv are flagged too, harmlessly)
        conv.sehip_exact_fp32 = True
    return conv
