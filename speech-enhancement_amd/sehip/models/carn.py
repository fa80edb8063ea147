"""CARN / GCARN (drop-in for models/_2104_05267_carn.py).

A real-valued conv U-Net over stacked re/im. The spectral front and back end
(ConvSTFT / ConviSTFT) and every real conv / transposed conv (encoder, GLU
gates, decoder, attention gates) run on the HIP kernels (the real-weight form
of the conv GEMMs, complex_nn.real_conv2d); BatchNorm2d + PReLU run as one fused
HIP pass each way (norm.bn_act -> se_bn_*); the LSTM (H = 512) runs on the wide
HIP recurrence (complex_nn.LSTM -> se_lstm_wide_*); the Linear(512 -> 514) head
on the hand-written GEMM, reading the decoder output and writing the mask in
their conv layouts (sehip.linear); the attention gates, the decoder's cat, the
mask + cat, the clamp and the layout copies as HIP passes (sehip.glue).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import glue
from ..complex_nn import LSTM, mark_data_fed, real_conv2d, stacked_lstms, _hip_lstm_ok
from ..conv_stft import ConvSTFT, ConviSTFT
from ..linear import linear
from ..norm import bn_act


def _conv(m: nn.Module, x):
    """A plain nn.Conv2d / nn.ConvTranspose2d on the HIP GEMM; any other module as is."""
    return real_conv2d(m, x) if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)) else m(x)


class ConvGLU(nn.Module):
    """carn.py:9-17."""

    def __init__(self, in_channels, out_channels, kernel_size, **kwargs):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, out_channels, kernel_size, **kwargs)
        self.conv2 = nn.Conv2d(in_channels, out_channels, kernel_size, **kwargs)

    def forward(self, x):
        return glue.glu(_conv(self.conv1, x), _conv(self.conv2, x))


class DeConvGLU(nn.Module):
    """carn.py:19-27."""

    def __init__(self, in_channels, out_channels, kernel_size, **kwargs):
        super().__init__()
        self.conv_transpose1 = nn.ConvTranspose2d(in_channels, out_channels, kernel_size, **kwargs)
        self.conv_transpose2 = nn.ConvTranspose2d(in_channels, out_channels, kernel_size, **kwargs)

    def forward(self, x):
        return glue.glu(_conv(self.conv_transpose1, x), _conv(self.conv_transpose2, x))


class ConvBlock(nn.Module):
    """carn.py:30-42."""

    def __init__(self, in_channels, out_channels, kernel_size, norm=True, act=True, gate=False, **kwargs):
        super().__init__()
        cls = ConvGLU if gate else nn.Conv2d
        self.conv = cls(in_channels, out_channels, kernel_size, bias=not norm, **kwargs)
        self.norm = nn.BatchNorm2d(out_channels) if norm else nn.Identity()
        self.act = nn.PReLU() if act else nn.Identity()

    def forward(self, x):
        return bn_act(self.norm, self.act, _conv(self.conv, x))


class ConvTransposeBlock(nn.Module):
    """carn.py:44-56."""

    def __init__(self, in_channels, out_channels, kernel_size, norm=True, act=True, gate=False, **kwargs):
        super().__init__()
        cls = DeConvGLU if gate else nn.ConvTranspose2d
        self.conv_transposed = cls(in_channels, out_channels, kernel_size, bias=not norm, **kwargs)
        self.norm = nn.BatchNorm2d(out_channels) if norm else nn.Identity()
        self.act = nn.PReLU() if act else nn.Identity()

    def forward(self, x):
        return bn_act(self.norm, self.act, _conv(self.conv_transposed, x))


class Attention(nn.Module):
    """carn.py:59-76: sigmoid(conv3(sigmoid(conv1 x_u + conv2 x_c))) * x_c."""

    def __init__(self, in_channels):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, in_channels * 2, kernel_size=3, padding=1, bias=False)
        self.conv2 = nn.Conv2d(in_channels, in_channels * 2, kernel_size=3, padding=1, bias=False)
        self.conv3 = nn.Conv2d(in_channels * 2, in_channels, kernel_size=3, padding=1, bias=False)

    def gate_logits(self, x_u, x_c, pad_u=False):
        """conv3(sigmoid(conv1(x_u) + conv2(x_c))): the pre-sigmoid gate; pad_u = x_u zero-padded by
        one frequency row at the bottom (the decoder's F.pad, carn.py:108-109), folded into conv1."""
        a = real_conv2d(self.conv1, x_u, (0, 0, 0, 1) if pad_u else None)
        return _conv(self.conv3, glue.add_sigmoid(a, _conv(self.conv2, x_c)))

    def forward(self, x_u, x_c):
        return glue.glu(x_c, self.gate_logits(x_u, x_c))


class Encoder(nn.Module):
    def __init__(self, in_channels=2, gate=False):
        super().__init__()
        chans = [in_channels, 16, 32, 64, 96, 128, 128]
        self.layers = nn.ModuleList(
            ConvBlock(chans[i], chans[i + 1], kernel_size=(3, 3), stride=(2, 1), padding=(1, 1), gate=gate)
            for i in range(6))

    def forward(self, x):
        outs = []
        for layer in self.layers:
            x = layer(x)
            outs.append(x)
        return x, outs


class Decoder(nn.Module):
    def __init__(self, in_channels=128, gate=False):
        super().__init__()
        self.conv_transpose_layers = nn.ModuleList()
        self.attention_layers = nn.ModuleList()
        c = in_channels
        for out_c in [128, 96, 64, 32, 16, 2]:
            self.attention_layers.append(Attention(c))
            self.conv_transpose_layers.append(
                ConvTransposeBlock(2 * c, out_c, kernel_size=(1, 3), stride=(2, 1), padding=(0, 1),
                                   output_padding=(1, 0), gate=gate))
            c = out_c

    def forward(self, x, encoder_outputs):
        for attention, layer in zip(self.attention_layers, self.conv_transpose_layers):
            skip = encoder_outputs.pop()
            pad = x.shape[2] < skip.shape[2]      # carn.py:108-109, folded into conv1's padding
            # cat([sigmoid(gate) * skip, skip]) in one pass (carn.py:74-76, :112-113)
            x = layer(glue.gate_cat(attention.gate_logits(x, skip, pad), skip))
        return x


class CARN(nn.Module):
    """carn.py:121-172."""

    def __init__(self, window_size=320, hop_size=160, fft_size=512, lstm_channels=512, gate=False):
        super().__init__()
        self.fft_size = fft_size
        self.stft = ConvSTFT(window_size, hop_size, fft_size)
        self.istft = ConviSTFT(window_size, hop_size, fft_size)
        self.encoder = Encoder(in_channels=2, gate=gate)
        mark_data_fed(self.encoder.layers[0])        # the noisy spectrum enters here
        self.decoder = Decoder(in_channels=128, gate=gate)
        self.lstm = LSTM(input_size=lstm_channels, hidden_size=lstm_channels, num_layers=2, batch_first=True)
        self.linear = nn.Linear(in_features=fft_size, out_features=fft_size + 2)

    def forward(self, x):
        half = self.fft_size // 2 + 1
        spec = self.stft(x)
        h, skips = self.encoder(glue.contiguous(spec.view(spec.shape[0], 2, half, -1)[:, :, 1:]))
        b, c, f, t = h.shape
        seq = h.reshape(b, c * f, t).transpose(1, 2)            # [b, t, c f]: a view, read in place
        if _hip_lstm_ok(self.lstm) and not self.lstm.bidirectional and h.is_cuda:
            # the LSTM output back to the conv layout and the storage type in one copy
            raw = stacked_lstms(seq, [self.lstm], batch_first=True, raw=True)[0]   # fp32 [b, t, H]
            h = glue.contiguous(raw.transpose(1, 2), h.dtype).view(b, c, f, t)
        else:
            h = glue.contiguous(self.lstm(seq)[0].transpose(1, 2)).view(b, c, f, t)
        h = self.decoder(h, skips)
        # the Linear head reads the decoder output and writes the mask in their [b, C, t] layouts
        m = linear(h.reshape(b, c * f, t).transpose(1, 2), self.linear, feature_major_out=True)
        m = m.transpose(1, 2).reshape(b, 2, half, t)
        est = glue.carn_mask(m, spec, half)     # carn.py:161-168 (sign as-is) + the cat
        return est, glue.clamp(self.istft(est), -1, 1)


class GCARN(CARN):
    """carn.py:174-176."""

    def __init__(self, window_size=320, hop_size=160, fft_size=512, lstm_channels=512):
        super().__init__(window_size, hop_size, fft_size, lstm_channels, gate=True)
