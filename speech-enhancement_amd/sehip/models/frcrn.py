"""FRCRN on the HIP path (drop-in for models/_2206_07293_frcrn.py).

Constructor signature, module tree and state_dict keys (279 entries) match
the reference. The spectral front/back end (ConvSTFT/ConviSTFT), every
complex conv / transposed conv, every ComplexBatchNorm2d (+ fused
LeakyReLU), the real final_conv, the complex LSTM, the CCBAM skip gates, the
skip joins (folded into the decoder GEMMs), the tanh mask and the SI-SNR loss
run on csrc/*.hip kernels; a training step launches no ATen kernel
(profiles/r6_*_kernel_stats.csv, tools/aten_sources.py).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as TF

from ..ccbam import CCBAM
from ..complex_nn import (ComplexBatchNorm2d, ComplexConv2d, ComplexConvTranspose2d, ComplexLSTM,
                          complex_concat, mark_data_fed, norm_act, real_conv2d)
from .. import functional as F
from .. import glue
from ..conv_stft import ConvSTFT, ConviSTFT


_SIDE_STREAMS: dict = {}


def _side_stream(dev):
    s = _SIDE_STREAMS.get(dev)
    if s is None:
        s = _SIDE_STREAMS[dev] = torch.cuda.Stream(dev)
        F.SIDE_STREAMS.append(s)
    return s


def _overlap_ok(tensors) -> bool:
    """Side streams on: GPU tensors, SEHIP_OVERLAP != 0, and no hook-based torch DDP
    (sehip.train.FlatDataParallel reduces after backward and keeps them)."""
    if not tensors or not tensors[0].is_cuda or os.environ.get("SEHIP_OVERLAP", "1") == "0":
        return False
    return not F.DDP_HOOKS[0]


class _CausalConvBase(nn.Module):
    """frcrn.py:11-59: left-pad time by padding[1] ('causal') or both sides,
    then (transposed) conv -> norm -> act."""

    conv_attr = "conv"

    def _conv(self):
        return getattr(self, self.conv_attr)

    def forward(self, x, fork: bool = False):
        lp = self.padding[1]
        pad = (lp, 0 if self.causal else lp, 0, 0)
        conv = self._conv()
        fused = self._first_block(x, conv, pad if lp else None, fork)
        if fused is not None:
            return fused
        plain = isinstance(conv, (nn.Conv2d, nn.ConvTranspose2d))
        transposed = isinstance(conv, (nn.ConvTranspose2d, ComplexConvTranspose2d))
        if lp and transposed:                      # zero input columns of a convT: materialise
            x, pad = TF.pad(x, pad), None
        elif not lp:
            pad = None
        # the time pad of a plain conv is folded into its (asymmetric) padding
        y = real_conv2d(conv, x, pad) if plain else conv(x, pad)
        return norm_act(self.norm, self.act, y, fork)

    def _first_block(self, x, conv, input_pad, fork):
        """The model's first block in training (its conv flagged data-fed): conv + CBN +
        act as functional.first_block, whose backward computes the conv's weight
        gradient inside the CBN backward (no dy tensor, no weight-grad GEMM). None where
        that path does not apply."""
        n = self.norm
        if not (isinstance(conv, ComplexConv2d) and conv.exact_fp32 and isinstance(n, ComplexBatchNorm2d)
                and n.affine and n.track_running_stats and n.training):
            return None
        act = {nn.LeakyReLU: F.ACT_LEAKY, nn.ReLU: F.ACT_RELU, nn.Identity: F.ACT_NONE}.get(type(self.act))
        c = conv.real_conv
        if act is None or c.groups != 1 or c.padding_mode != "zeros" or isinstance(c.padding, str) or \
                not F.first_block_supported(x, c.weight, c.bias, True, c.kernel_size):
            return None
        from ..complex_nn import _fold_pad
        begin, end = _fold_pad(c.padding, input_pad, False)
        slope = self.act.negative_slope if act == F.ACT_LEAKY else 0.0
        return F.first_block(x, c.weight, conv.imag_conv.weight, n.Wrr, n.Wri, n.Wii, n.Br, n.Bi,
                             (n.RMr, n.RMi, n.RVrr, n.RVri, n.RVii), n.num_batches_tracked, n.eps, n.momentum, act,
                             slope, kernel=c.kernel_size, stride=c.stride, padding=begin, padding_end=end,
                             dilation=c.dilation, fork=fork)

    def forward_joined(self, x, skip):
        """self(complex_join(x, skip)) (frcrn.py:95-101) without writing the
        joined tensor: the conv GEMMs gather from x and skip directly."""
        conv = self._conv()
        if self.padding[1] or not isinstance(conv, (ComplexConv2d, ComplexConvTranspose2d)) \
                or x.shape[1] != skip.shape[1]:
            return self(F.complex_join(x, skip))
        y = conv.forward_joined(x, skip)
        return norm_act(self.norm, self.act, y)

    def forward_joined_head(self, x, skip, head: nn.Conv2d):
        """head(self(complex_join(x, skip))) for FRCRN's final_conv (frcrn.py:115, 140):
        the CBN + activation + head run as one fused op (se_cbn_head_*), so the block's
        output is never written; anything the fused op does not cover runs unfused."""
        conv = self._conv()
        act = {nn.LeakyReLU: F.ACT_LEAKY, nn.ReLU: F.ACT_RELU, nn.Identity: F.ACT_NONE}.get(type(self.act))
        w = head.weight
        fusable = (os.environ.get("SEHIP_HEAD", "1") != "0" and isinstance(self.norm, ComplexBatchNorm2d)
                   and act is not None and not self.padding[1] and x.is_cuda
                   and isinstance(conv, (ComplexConv2d, ComplexConvTranspose2d)) and x.shape[1] == skip.shape[1]
                   and type(head) is nn.Conv2d and head.bias is None and w.dtype == torch.float32
                   and x.dtype == torch.float32 and (w.shape[0], w.shape[2], w.shape[3]) in F.HEAD_SUPPORTED
                   and head.stride == (1, 1) and head.padding == (0, 0) and head.dilation == (1, 1)
                   and head.groups == 1)
        if not fusable:
            return real_conv2d(head, self.forward_joined(x, skip))
        y = conv.forward_joined(x, skip)
        if w.shape[1] != y.shape[1]:
            raise ValueError(f"head takes {w.shape[1]} channels, the block gives {y.shape[1]}")
        n = self.norm
        running = (n.RMr, n.RMi, n.RVrr, n.RVri, n.RVii) if n.track_running_stats else None
        slope = self.act.negative_slope if act == F.ACT_LEAKY else 0.0
        return F.complex_batch_norm_head(y, n.Wrr, n.Wri, n.Wii, n.Br, n.Bi, w, running,
                                         n.num_batches_tracked if n.track_running_stats else None,
                                         n.training or not n.track_running_stats, n.eps, n.momentum,
                                         act, slope)


def _make_block(block, transposed, in_channels, out_channels, kernel_size, padding, norm, act,
                causal, is_complex, kwargs):
    block.causal, block.padding = causal, padding
    slope = kwargs.pop("negative_slope", 0.2)
    if is_complex:
        conv_cls = ComplexConvTranspose2d if transposed else ComplexConv2d
        norm_m = ComplexBatchNorm2d(out_channels) if norm else nn.Identity()
    else:
        conv_cls = nn.ConvTranspose2d if transposed else nn.Conv2d
        norm_m = nn.BatchNorm2d(out_channels) if norm else nn.Identity()
    setattr(block, block.conv_attr, conv_cls(in_channels, out_channels, kernel_size,
                                             padding=(padding[0], 0), bias=not norm, **kwargs))
    block.norm = norm_m
    block.act = nn.LeakyReLU(slope) if act else nn.Identity()


class ConvBlock(_CausalConvBase):
    """frcrn.py:11-34."""

    def __init__(self, in_channels, out_channels, kernel_size, padding=(0, 0), norm=True, act=True,
                 causal=True, is_complex=True, **kwargs):
        super().__init__()
        _make_block(self, False, in_channels, out_channels, kernel_size, padding, norm, act, causal,
                    is_complex, kwargs)


class ConvTransposeBlock(_CausalConvBase):
    """frcrn.py:36-59."""

    conv_attr = "conv_transposed"

    def __init__(self, in_channels, out_channels, kernel_size, padding=(0, 0), norm=True, act=True,
                 causal=True, is_complex=True, **kwargs):
        super().__init__()
        _make_block(self, True, in_channels, out_channels, kernel_size, padding, norm, act, causal,
                    is_complex, kwargs)


class Encoder(nn.Module):
    """frcrn.py:62-76: six (5,2)/(2,1) causal complex conv blocks."""

    def __init__(self, in_channels=1, out_channels=128, num_repeats=6, is_complex=True):
        super().__init__()
        chans = [in_channels] + [out_channels] * num_repeats
        self.layers = nn.ModuleList(
            ConvBlock(chans[i], chans[i + 1], kernel_size=(5, 2), stride=(2, 1), padding=(0, 1),
                      causal=True, is_complex=is_complex) for i in range(num_repeats))

    def forward(self, x):
        # each block output feeds the next block and a decoder skip (frcrn.py:70-75): forked in
        # the CBN so the two gradients are summed inside its backward (se_cbn_bwd2)
        skips = []
        for layer in self.layers:
            x, skip = layer(x, fork=True)
            skips.append(skip)
        return x, skips


class Decoder(nn.Module):
    """frcrn.py:78-102: CCBAM on each skip, align, complex concat, convT block."""

    def __init__(self, in_channels=128, out_channels=128, num_repeats=6, reduction_ratio=16,
                 is_complex=True):
        super().__init__()
        self.skip_connection_attention_layers = nn.ModuleList()
        self.layers = nn.ModuleList()
        c = in_channels
        for _ in range(num_repeats):
            self.skip_connection_attention_layers.append(CCBAM(c, reduction_ratio))
            self.layers.append(ConvTransposeBlock(2 * c, out_channels, kernel_size=(5, 2), stride=(2, 1),
                                                  padding=(0, 0), causal=True, is_complex=is_complex))
            c = out_channels

    def gate_state(self, x):
        """Per-step state for gating the skips on a side HIP stream as the encoder produces
        them (attend_skip), or None to run them inline: off the GPU, with SEHIP_OVERLAP=0,
        or under DDP (its gradient-ready hooks would see the CCBAM parameter gradients on
        the side stream). The gates depend only on the encoder outputs; on the side stream
        they run beside the encoder's GEMMs and the latency-bound LSTM recurrence, and
        autograd runs their backward there too, beside the decoder's data-grad chain."""
        if not _overlap_ok([x]):
            return None
        n = len(self.skip_connection_attention_layers)
        return [None] * n, [None] * n

    def attend_skip(self, state, skip, i):
        """Start the gate of encoder output i (attention layer n-1-i) on the side stream."""
        dev = skip.device
        main, side = torch.cuda.current_stream(dev), _side_stream(dev)
        side.wait_stream(main)
        j = len(self.skip_connection_attention_layers) - 1 - i
        with torch.cuda.stream(side):
            skip.record_stream(side)
            state[0][j] = self.skip_connection_attention_layers[j](skip)
            ev = torch.cuda.Event()
            ev.record(side)
            state[1][j] = ev   # the decoder waits per gate, not for all six

    def attend_skips(self, encoder_outputs):
        """All six gates at once on the side stream (after the encoder): returns
        (gated skips in decoder order, their ready events) or None (see gate_state)."""
        state = self.gate_state(encoder_outputs[0])
        if state is not None:   # deepest (smallest, first needed) skip first
            for i, skip in reversed(list(enumerate(encoder_outputs))):
                self.attend_skip(state, skip, i)
        return state

    def forward(self, x, encoder_outputs, attended=None, head=None):
        """head: a conv applied to the last block's output (FRCRN's final_conv), fused
        into that block's CBN where the fused op covers it (forward_joined_head)."""
        if attended is not None:   # gated on the side stream (attend_skips)
            gated, ready = (list(reversed(t)) for t in attended)   # popped like encoder_outputs
            main = torch.cuda.current_stream(x.device)
        for attention, layer in zip(self.skip_connection_attention_layers, self.layers):
            if attended is not None:
                # join the side stream at this gate only: the later (larger) gates are still
                # running beside this decoder layer
                main.wait_event(ready.pop())
                skip = gated.pop()
                skip.record_stream(main)
            else:
                skip = attention(encoder_outputs.pop())
            # frcrn.py:95-99: x[..., :-1] if wider, F.pad(x, (0, 0, 0, 1)) if shorter, then
            # complex_concat([x, skip]): folded into the convT's GEMMs (se_conv2d_*_joined);
            # modes without a joined kernel materialise it in one pass (se_complex_join)
            if x.shape[-1] - skip.shape[-1] not in (0, 1) or skip.shape[-2] - x.shape[-2] not in (0, 1):
                raise ValueError(f"decoder/skip grids do not align: {tuple(x.shape)} vs {tuple(skip.shape)}")
            if head is not None and layer is self.layers[-1]:
                return layer.forward_joined_head(x, skip, head)
            x = layer.forward_joined(x, skip)
        return real_conv2d(head, x) if head is not None else x


class FRCRN(nn.Module):
    """frcrn.py:104-155."""

    def __init__(self, window_size=320, hop_size=160, fft_size=640, lstm_channels=256,
                 reduction_ratio=16, is_complex=True):
        super().__init__()
        self.stft = ConvSTFT(window_size, hop_size, fft_size)
        self.istft = ConviSTFT(window_size, hop_size, fft_size)
        self.encoder = Encoder(in_channels=2, out_channels=128, is_complex=is_complex)
        mark_data_fed(self.encoder.layers[0])        # the noisy spectrum enters here
        self.decoder = Decoder(in_channels=128, out_channels=128, is_complex=is_complex,
                               reduction_ratio=reduction_ratio)
        self.lstm = ComplexLSTM(256, lstm_channels, num_layers=2, bidirectional=False, batch_first=True)
        self.lstm.feature_major_out = True   # forward transposes it back to [b, c f, t] (:137): a view
        self.final_conv = nn.Conv2d(128, 2, kernel_size=(1, 2), bias=False)
        self.fft_size = fft_size

    def forward(self, x):
        half = self.fft_size // 2 + 1
        spec = self.stft(x)                                            # [B, N+2, T]
        noisy = spec.view(spec.shape[0], 2, half, spec.shape[-1])[:, :, 1:]   # drop DC (:123-127)
        h, skips = glue.contiguous(noisy), []
        attended = self.decoder.gate_state(h)
        for layer in self.encoder.layers:                              # Encoder.forward
            h, skip = layer(h, fork=True)
            skips.append(skip)
        # the six gates on the side stream after the encoder (beside the half-idle LSTM
        # recurrence; starting each beside the encoder's GEMMs measured 534 vs 538 utt/s),
        # in the decoder's order: the smallest, deepest skip first, so the decoder starts
        # right after the LSTM, beside the big gates
        if attended is not None:
            for i, skip in reversed(list(enumerate(skips))):
                self.decoder.attend_skip(attended, skip, i)
        b, c, f, t = h.shape                                           # :133-137
        h = self.lstm(h.reshape(b, c * f, t).transpose(1, 2))
        h = h.transpose(1, 2).reshape(b, c, f, t)
        # decoder + final_conv; the conv is fused into the last block's CBN (se_cbn_head_*)
        h = self.decoder(h, skips, attended, head=self.final_conv)
        if h.is_cuda and h.dtype == torch.float32 and tuple(h.shape[1:]) == (2, half - 2, spec.shape[-1]):
            est = F.complex_mask(h, spec, half)                        # :140-152 in one pass each way
        else:
            mask = torch.tanh(TF.pad(h, (0, 0, 1, 0)))                 # :140-144
            est = TF.pad(mask * noisy, (0, 0, 1, 0))                   # :145-146 (DC back as 0)
            est = est.reshape(b, 2 * half, est.shape[-1])              # cat(re, im) on dim 1 (:149-152)
        wav = self.istft(est)
        return est, glue.clamp(wav, -1, 1)                             # :153-155
