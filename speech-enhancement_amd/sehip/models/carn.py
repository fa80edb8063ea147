"""CARN / GCARN (drop-in for models/_2104_05267_carn.py).

A real-valued conv U-Net over stacked re/im. The spectral front and back end
(ConvSTFT / ConviSTFT) and every real conv / transposed conv (encoder, GLU
gates, decoder, attention gates) run on the HIP kernels (the real-weight form
of the conv GEMMs, complex_nn.real_conv2d); BatchNorm2d + PReLU run as one fused
HIP pass each way (norm.bn_act -> se_bn_*); the LSTM (H = 512) runs on the wide
HIP recurrence (complex_nn.LSTM -> se_lstm_wide_*).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as TF

from ..complex_nn import LSTM, mark_data_fed, real_conv2d
from ..conv_stft import ConvSTFT, ConviSTFT
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
        return _conv(self.conv1, x) * torch.sigmoid(_conv(self.conv2, x))


class DeConvGLU(nn.Module):
    """carn.py:19-27."""

    def __init__(self, in_channels, out_channels, kernel_size, **kwargs):
        super().__init__()
        self.conv_transpose1 = nn.ConvTranspose2d(in_channels, out_channels, kernel_size, **kwargs)
        self.conv_transpose2 = nn.ConvTranspose2d(in_channels, out_channels, kernel_size, **kwargs)

    def forward(self, x):
        return _conv(self.conv_transpose1, x) * torch.sigmoid(_conv(self.conv_transpose2, x))


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

    def forward(self, x_u, x_c):
        gate = torch.sigmoid(_conv(self.conv3, torch.sigmoid(_conv(self.conv1, x_u) + _conv(self.conv2, x_c))))
        return gate * x_c


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
            if x.shape[2] < skip.shape[2]:
                x = TF.pad(x, (0, 0, 0, 1))
            x = layer(torch.cat([attention(x, skip), skip], dim=1))
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
        nr, ni = spec[:, :half], spec[:, half:]
        h, skips = self.encoder(spec.view(spec.shape[0], 2, half, -1)[:, :, 1:].contiguous())
        b, c, f, t = h.shape
        h = self.lstm(h.reshape(b, c * f, t).transpose(1, 2))[0].transpose(1, 2).reshape(b, c, f, t)
        h = self.decoder(h, skips)
        h = self.linear(h.reshape(b, c * f, t).transpose(1, 2)).transpose(1, 2).reshape(b, 2, half, t)
        mr, mi = h[:, 0], h[:, 1]
        est = torch.cat([mr * nr - mi * ni, mr * ni - mi * nr], dim=1)   # carn.py:165-166 (sign as-is)
        return est, torch.clamp_(self.istft(est), -1, 1)


class GCARN(CARN):
    """carn.py:174-176."""

    def __init__(self, window_size=320, hop_size=160, fft_size=512, lstm_channels=512):
        super().__init__(window_size, hop_size, fft_size, lstm_channels, gate=True)
