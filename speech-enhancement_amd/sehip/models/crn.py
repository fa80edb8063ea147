"""CRN (drop-in for models/_1809_01405_crn.py): magnitude-domain conv-LSTM
that exercises the mag/phase API of ConvSTFT / ConviSTFT (HIP kernels); its
real convs run on the real-weight form of the HIP conv GEMMs (real_conv2d),
BatchNorm2d + ELU as one fused HIP pass each way (norm.bn_act); the 1024-wide
two-layer LSTM (:90) on the wide HIP recurrence (se_lstm_wide_*, a group of 64
workgroups of 16 hidden units)."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as TF

from ..complex_nn import LSTM, mark_data_fed, real_conv2d
from ..conv_stft import ConvSTFT, ConviSTFT
from ..norm import bn_act


class ConvBlock(nn.Module):
    """crn.py:9-25: conv, drop the last padding[0] rows (causal), BN, ELU."""

    def __init__(self, in_channels, out_channels, kernel_size, norm=True, act=True, **kwargs):
        super().__init__()
        alpha = kwargs.get("alpha", 1)
        self.padding = kwargs.get("padding", (0, 0))
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, bias=not norm, **kwargs)
        self.norm = nn.BatchNorm2d(out_channels) if norm else nn.Identity()
        self.act = nn.ELU(alpha) if act else nn.Identity()

    def forward(self, x):
        return bn_act(self.norm, self.act, real_conv2d(self.conv, x)[:, :, :-self.padding[0], :])


class ConvTransposeBlock(nn.Module):
    """crn.py:27-41."""

    def __init__(self, in_channels, out_channels, kernel_size, norm=True, act=True, **kwargs):
        super().__init__()
        alpha = kwargs.get("alpha", 1)
        self.padding = kwargs.get("padding", (0, 0))
        self.conv_transposed = nn.ConvTranspose2d(in_channels, out_channels, kernel_size, bias=not norm, **kwargs)
        self.norm = nn.BatchNorm2d(out_channels) if norm else nn.Identity()
        self.act = nn.ELU(alpha) if act else nn.Identity()

    def forward(self, x):
        return bn_act(self.norm, self.act, real_conv2d(self.conv_transposed, x)[:, :, :-1, :])


class Encoder(nn.Module):
    def __init__(self, in_channels=1):
        super().__init__()
        chans = [in_channels, 16, 32, 64, 128, 256]
        self.layers = nn.ModuleList(
            ConvBlock(chans[i], chans[i + 1], kernel_size=(2, 3), stride=(1, 2), padding=(1, 0))
            for i in range(5))

    def forward(self, x):
        outs = []
        for layer in self.layers:
            x = layer(x)
            outs.append(x)
        return x, outs


class Decoder(nn.Module):
    def __init__(self, in_channels=512):
        super().__init__()
        self.layers = nn.ModuleList()
        c = in_channels
        for i, out_c in enumerate([128, 64, 32, 16, 1]):
            kw = dict(kernel_size=(2, 3), stride=(1, 2))
            if i == 3:
                kw["output_padding"] = (0, 1)
            if i == 4:
                kw.update(norm=False, act=False)
            self.layers.append(ConvTransposeBlock(c, out_c, **kw))
            c = out_c * 2

    def forward(self, x, encoder_outputs):
        for layer in self.layers:
            x = layer(torch.cat([x, encoder_outputs.pop()], dim=1))
        return x


class CRN(nn.Module):
    """crn.py:82-109."""

    def __init__(self, window_size=320, hop_size=160, fft_size=320):
        super().__init__()
        self.stft = ConvSTFT(window_size, hop_size, fft_size, return_mag_phase=True)
        self.istft = ConviSTFT(window_size, hop_size, fft_size)
        self.encoder = Encoder()
        mark_data_fed(self.encoder.layers[0])        # the noisy magnitude enters here
        self.lstm_layers = LSTM(input_size=1024, hidden_size=1024, num_layers=2, batch_first=True)
        self.decoder = Decoder()

    def forward(self, x):
        mag, phase = self.stft(x)
        h, skips = self.encoder(mag.transpose(1, 2).unsqueeze(1))
        b, c, t, f = h.shape
        h = self.lstm_layers(h.permute(0, 2, 1, 3).reshape(b, t, c * f))[0]
        h = self.decoder(h.reshape(b, t, c, f).permute(0, 2, 1, 3), skips)
        est = TF.softplus(h).squeeze(1).transpose(1, 2)
        return est, self.istft(est, phase)
