"""DCCRN on the HIP path (drop-in for models/_2008_00264_dccrn.py)."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as TF

from ..complex_nn import (ComplexBatchNorm2d, ComplexConv2d, ComplexConvTranspose2d, ComplexLinear,
                          ComplexLSTM, LSTM, complex_concat, mark_data_fed, norm_act,
                          real_conv2d)
from .. import functional as F
from .. import glue
from ..conv_stft import ConvSTFT, ConviSTFT
from ..linear import linear


class _Block(nn.Module):
    """dccrn.py:11-57: causal pad -> (T)conv -> CBN -> PReLU."""

    def __init__(self, transposed, in_channels, out_channels, kernel_size, padding, norm, act, causal,
                 is_complex, kwargs):
        super().__init__()
        self.causal, self.padding = causal, padding
        if is_complex:
            conv = (ComplexConvTranspose2d if transposed else ComplexConv2d)
            norm_cls = ComplexBatchNorm2d
        else:
            conv = (nn.ConvTranspose2d if transposed else nn.Conv2d)
            norm_cls = nn.BatchNorm2d
        self._attr = "conv_transposed" if transposed else "conv"
        setattr(self, self._attr, conv(in_channels, out_channels, kernel_size,
                                       padding=(padding[0], 0), bias=not norm, **kwargs))
        self.norm = norm_cls(out_channels) if norm else nn.Identity()
        self.act = nn.PReLU() if act else nn.Identity()

    def forward(self, x, fork: bool = False):
        """fork=True: (y, y2) for the two consumers of an encoder output (the next block
        and the decoder skip, dccrn.py:98-101), summed inside the CBN backward."""
        lp = self.padding[1]
        pad = (lp, 0 if self.causal else lp, 0, 0)
        conv = getattr(self, self._attr)
        plain = isinstance(conv, (nn.Conv2d, nn.ConvTranspose2d))
        transposed = isinstance(conv, (nn.ConvTranspose2d, ComplexConvTranspose2d))
        if lp and transposed:          # zero input columns of a convT: materialised
            x, pad = TF.pad(x, pad), None
        elif not lp:
            pad = None
        # a conv's causal time pad is folded into its (asymmetric) padding, not materialised
        y = real_conv2d(conv, x, pad) if plain else conv(x, pad)
        return norm_act(self.norm, self.act, y, fork)

    def forward_joined(self, x, skip):
        """self(complex_concat([x[..., :T], skip])) (dccrn.py:116-120) with the concat folded
        into the convT's GEMMs (se_conv2d_*_joined); None where that path does not apply."""
        conv = getattr(self, self._attr)
        if (self.padding[1] or not isinstance(conv, ComplexConvTranspose2d) or x.dtype != skip.dtype
                or x.shape[2] != skip.shape[2] or x.shape[1] != skip.shape[1]):
            return None
        y = conv.forward_joined(x, skip)
        return norm_act(self.norm, self.act, y)


class ConvBlock(_Block):
    def __init__(self, in_channels, out_channels, kernel_size, padding=(0, 0), norm=True, act=True,
                 causal=True, is_complex=True, **kwargs):
        super().__init__(False, in_channels, out_channels, kernel_size, padding, norm, act, causal,
                         is_complex, kwargs)


class ConvTransposeBlock(_Block):
    def __init__(self, in_channels, out_channels, kernel_size, padding=(0, 0), norm=True, act=True,
                 causal=True, is_complex=True, **kwargs):
        super().__init__(True, in_channels, out_channels, kernel_size, padding, norm, act, causal,
                         is_complex, kwargs)


class LSTMBlock(nn.Module):
    """dccrn.py:59-86."""

    def __init__(self, in_channels, hidden_channels, linear_channels, num_layers=2, is_complex=True,
                 **kwargs):
        super().__init__()
        nd = 2 if kwargs.get("bidirectional", True) else 1
        self.layers = nn.ModuleList()
        if is_complex:
            for _ in range(num_layers - 1):
                self.layers.append(ComplexLSTM(in_channels, hidden_channels, num_layers=1, **kwargs))
            self.layers.append(ComplexLSTM(nd * hidden_channels, hidden_channels, num_layers=1, **kwargs))
            self.layers.append(ComplexLinear(nd * hidden_channels, linear_channels))
        else:
            self.layers.append(LSTM(in_channels, hidden_channels, num_layers=num_layers, **kwargs))
            self.layers.append(nn.Linear(nd * hidden_channels, linear_channels))

    # the last Linear's output as the transposed view of a [B, out, T] storage: the layout
    # DCCRN.forward transposes it back to (dccrn.py:169-171), so that transpose is a view
    feature_major_out = False

    def forward(self, x):
        for i, layer in enumerate(self.layers):
            last = i == len(self.layers) - 1
            if isinstance(layer, nn.Linear) and isinstance(x, torch.Tensor) and x.is_cuda:
                x = linear(x, layer, feature_major_out=last and self.feature_major_out)
                continue
            x = layer(x)
            if isinstance(x, tuple):
                x = x[0]
        return x


class Encoder(nn.Module):
    def __init__(self, encoder_channels, in_channels=2, is_complex=True):
        super().__init__()
        chans = [in_channels] + list(encoder_channels)
        self.layers = nn.ModuleList(
            ConvBlock(chans[i], chans[i + 1], kernel_size=(5, 2), stride=(2, 1), padding=(2, 1),
                      causal=True, is_complex=is_complex) for i in range(len(encoder_channels)))

    def forward(self, x):
        outs = []
        for layer in self.layers:   # each output feeds the next block (or the LSTM) and a decoder skip
            x, skip = layer(x, fork=True)
            outs.append(skip)
        return x, outs


class Decoder(nn.Module):
    def __init__(self, decoder_channels, in_channels=256, is_complex=True):
        super().__init__()
        self.layers = nn.ModuleList()
        c = in_channels
        for out_c in decoder_channels:
            self.layers.append(ConvTransposeBlock(2 * c, out_c, kernel_size=(5, 2), stride=(2, 1),
                                                  padding=(2, 0), output_padding=(1, 0), causal=True,
                                                  is_complex=is_complex))
            c = out_c

    def forward(self, x, encoder_outputs):
        for layer in self.layers:
            skip = encoder_outputs.pop()
            # the reference trims one trailing frame of x (dccrn.py:116-117); the joined GEMMs
            # read the first T frames of x directly
            aligned = x.shape[-1] - skip.shape[-1] in (0, 1) and x.shape[2] == skip.shape[2]
            y = layer.forward_joined(x, skip) if aligned else None
            if y is None and aligned and x.is_cuda and x.dtype == skip.dtype:
                # no joined GEMM for this mode / width: the trim and complex_concat as one
                # HIP pass each way (se_complex_join), any storage type
                y = layer(F.complex_join(x, skip))
            if y is None:
                if x.shape[-1] > skip.shape[-1]:
                    x = x[..., :-1]
                y = layer(complex_concat([x, skip], dim=1))
            x = y
        return x


class DCCRN(nn.Module):
    """dccrn.py:123-212."""

    def __init__(self, config="dccrn-CL", window_size=400, hop_size=100, fft_size=512, lstm_channels=256,
                 linear_channels=1024, bidirectional=False, is_complex=True):
        super().__init__()
        if config in ("dccrn-C", "dccrn-R", "dccrn-E"):
            enc, masking = [32, 64, 128, 128, 256, 256], config[-1]
        else:
            enc, masking = [32, 64, 128, 256, 256, 256], "E"
        dec = enc[:-1][::-1] + [2]
        freq_channels = (fft_size // 2 // (2 ** len(enc))) * enc[-1]
        self.stft = ConvSTFT(window_size, hop_size, fft_size)
        self.istft = ConviSTFT(window_size, hop_size, fft_size)
        self.encoder = Encoder(enc, in_channels=2, is_complex=is_complex)
        mark_data_fed(self.encoder.layers[0])        # the noisy spectrum enters here
        self.decoder = Decoder(dec, in_channels=256, is_complex=is_complex)
        self.lstm = LSTMBlock(freq_channels, lstm_channels, linear_channels, num_layers=2, batch_first=True,
                              bidirectional=bidirectional, is_complex=is_complex)
        self.lstm.feature_major_out = True
        if is_complex:
            self.lstm.layers[-1].feature_major_out = True
        self.masking, self.fft_size = masking, fft_size

    def forward(self, x):
        half = self.fft_size // 2 + 1
        spec = self.stft(x)
        nr, ni = spec[:, :half], spec[:, half:]
        h, skips = self.encoder(glue.contiguous(spec.view(spec.shape[0], 2, half, -1)[:, :, 1:]))
        b, c, f, t = h.shape
        h = self.lstm(h.reshape(b, c * f, t).transpose(1, 2)).transpose(1, 2).reshape(b, c, f, t)
        dec = self.decoder(h, skips)
        est = None
        if self.masking == "E" and dec.shape[-1] - nr.shape[-1] in (0, 1):
            # the top zero row (F.pad, dccrn.py:172), the trailing-frame trim (:180-182), the mask
            # and the concat in one pass each way (se_polar_mask_fwd / _bwd, m_row0 = 1)
            est = F.polar_mask_stored(dec, nr, ni, 1, row0=1)
        if est is None:
            h = TF.pad(dec, (0, 0, 1, 0))
            mr, mi = h[:, 0], h[:, 1]
            if mr.shape[-1] > nr.shape[-1]:
                mr, mi = mr[..., :-1], mi[..., :-1]
            est = F.polar_mask(mr, mi, nr, ni, 1) if self.masking == "E" else None
            if est is None:
                re, im = self._mask_processing(nr, ni, mr, mi)
                est = torch.cat([re, im], dim=1)
        if est.dim() == 4:
            est = est.view(est.shape[0], -1, est.shape[-1])
        return est, glue.clamp(self.istft(est), -1, 1)

    def _mask_processing(self, noisy_real, noisy_imag, mask_real, mask_imag):
        """dccrn.py:187-207."""
        if self.masking == "R":
            return noisy_real * mask_real, noisy_imag * mask_imag
        if self.masking == "C":
            return (noisy_real * mask_real - noisy_imag * mask_imag,
                    noisy_real * mask_imag + noisy_imag * mask_real)
        n_mag, n_ph = self._return_mag_phase(noisy_real, noisy_imag)
        m_mag, _ = self._return_mag_phase(mask_real, mask_imag)
        m_ph = torch.atan2(mask_imag / m_mag, mask_real / m_mag)
        gain = n_mag * torch.tanh(m_mag)
        return gain * torch.cos(n_ph + m_ph), gain * torch.sin(n_ph + m_ph)

    @staticmethod
    def _return_mag_phase(real, imag):
        return torch.sqrt(real ** 2 + imag ** 2 + 1e-8), torch.atan2(imag, real)
