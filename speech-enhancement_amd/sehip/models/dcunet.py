"""DCUNet on the HIP path (drop-in for models/_1903_03107_dcunet.py and the
dcunet table of models/architectures.py:53-97)."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as TF

from ..complex_nn import (ComplexBatchNorm2d, ComplexConv2d, ComplexConvTranspose2d, ComplexLeakyReLU,
                          mark_data_fed, norm_act, real_conv2d)
from .. import functional as F
from .. import glue
from ..conv_stft import ConvSTFT, ConviSTFT

# name -> per-layer ((complex channels, real channels), kernel, stride, padding)
dcunet_architecture = {
    "dcunet10": [((32, 45), (7, 5), (2, 2), (3, 2)), ((64, 90), (7, 5), (2, 2), (3, 2)),
                 ((64, 90), (5, 3), (2, 2), (2, 1)), ((64, 90), (5, 3), (2, 2), (2, 1)),
                 ((64, 90), (5, 3), (2, 1), (2, 1))],
    "dcunet16": [((32, 45), (7, 5), (2, 2), (3, 2)), ((32, 45), (7, 5), (2, 1), (3, 2)),
                 ((64, 90), (7, 5), (2, 2), (3, 2)), ((64, 90), (5, 3), (2, 1), (2, 1)),
                 ((64, 90), (5, 3), (2, 2), (2, 1)), ((64, 90), (5, 3), (2, 1), (2, 1)),
                 ((64, 90), (5, 3), (2, 2), (2, 1)), ((64, 90), (5, 3), (2, 1), (2, 1))],
    "dcunet20": [((32, 45), (7, 1), (1, 1), (3, 0)), ((32, 45), (1, 7), (1, 1), (0, 3)),
                 ((64, 90), (7, 5), (2, 2), (3, 2)), ((64, 90), (7, 5), (2, 1), (3, 2)),
                 ((64, 90), (5, 3), (2, 2), (2, 1)), ((64, 90), (5, 3), (2, 1), (2, 1)),
                 ((64, 90), (5, 3), (2, 2), (2, 1)), ((64, 90), (5, 3), (2, 1), (2, 1)),
                 ((64, 90), (5, 3), (2, 2), (2, 1)), ((90, 180), (5, 3), (2, 1), (2, 1))],
    "dcunet20-large": [((45, 45), (7, 1), (1, 1), (3, 0)), ((45, 45), (1, 7), (1, 1), (0, 3)),
                       ((90, 90), (7, 5), (2, 2), (3, 2)), ((90, 90), (7, 5), (2, 1), (3, 2)),
                       ((90, 90), (5, 3), (2, 2), (2, 1)), ((90, 90), (5, 3), (2, 1), (2, 1)),
                       ((90, 90), (5, 3), (2, 2), (2, 1)), ((90, 90), (5, 3), (2, 1), (2, 1)),
                       ((90, 90), (5, 3), (2, 2), (2, 1)), ((128, 128), (5, 3), (2, 1), (2, 1))],
}


class _Block(nn.Module):
    def __init__(self, transposed, in_channels, out_channels, kernel_size, norm, act, is_complex, slope,
                 kwargs):
        super().__init__()
        if is_complex:
            conv = ComplexConvTranspose2d if transposed else ComplexConv2d
            norm_cls, act_cls = ComplexBatchNorm2d, ComplexLeakyReLU
        else:
            conv = nn.ConvTranspose2d if transposed else nn.Conv2d
            norm_cls, act_cls = nn.BatchNorm2d, nn.LeakyReLU
        self._attr = "conv_transposed" if transposed else "conv"
        setattr(self, self._attr, conv(in_channels, out_channels, kernel_size, bias=not norm, **kwargs))
        self.norm = norm_cls(out_channels) if norm else nn.Identity()
        self.act = act_cls(slope) if act else nn.Identity()

    def forward(self, x):
        conv = getattr(self, self._attr)
        y = real_conv2d(conv, x) if isinstance(conv, (nn.Conv2d, nn.ConvTranspose2d)) else conv(x)
        return norm_act(self.norm, self.act, y)

    def forward_joined(self, x, skip):
        """self(torch.cat([pad(x), skip])) (dcunet.py:84-94) with the pad and cat folded into the
        convT's GEMMs (se_conv2d_*_joined, join_cat; the 2-channel mask layer's forward on the
        chunked stencil); None where no joined kernel covers the layer (a real conv, or jh = C/2
        not a multiple of 32). A pass without a joined kernel for its shape materialises the cat
        for that pass only."""
        conv = getattr(self, self._attr)
        if (not isinstance(conv, ComplexConvTranspose2d) or not x.is_cuda or x.dtype != skip.dtype
                or x.shape[1] != skip.shape[1] or x.shape[2] > skip.shape[2] or x.shape[3] > skip.shape[3]
                or (x.shape[1] // 2) % 32):
            return None
        y = conv.forward_joined(x, skip, cat=True)
        return norm_act(self.norm, self.act, y)


class ConvBlock(_Block):
    """dcunet.py:12-27."""

    def __init__(self, in_channels, out_channels, kernel_size, norm=True, act=True, is_complex=True,
                 **kwargs):
        slope = kwargs.pop("negative_slope", 0.01)
        super().__init__(False, in_channels, out_channels, kernel_size, norm, act, is_complex, slope, kwargs)


class ConvTransposeBlock(_Block):
    """dcunet.py:29-43 (LeakyReLU default slope 0.01)."""

    def __init__(self, in_channels, out_channels, kernel_size, norm=True, act=True, is_complex=True,
                 **kwargs):
        super().__init__(True, in_channels, out_channels, kernel_size, norm, act, is_complex, 0.01, kwargs)


def _width(spec, is_complex):
    return spec[0][0] * 2 if is_complex else spec[0][1]


class Encoder(nn.Module):
    def __init__(self, architecture, in_channels=32, is_complex=True):
        super().__init__()
        self.layers = nn.ModuleList()
        c = in_channels
        for spec in architecture:
            out_c = _width(spec, is_complex)
            self.layers.append(ConvBlock(c, out_c, spec[1], stride=spec[2], padding=spec[3],
                                         is_complex=is_complex))
            c = out_c

    def forward(self, x):
        outs = []
        for layer in self.layers:
            x = layer(x)
            outs.append(x)
        return x, outs


class Decoder(nn.Module):
    def __init__(self, architecture, in_channels=64, mask_channels=2, is_complex=True):
        super().__init__()
        self.layers = nn.ModuleList()
        c = in_channels
        for i in range(len(architecture) - 1):
            k, s, p = architecture[-i - 1][1:]
            out_c = _width(architecture[-i - 2], is_complex)
            self.layers.append(ConvTransposeBlock(2 * c, out_c, k, stride=s, padding=p, is_complex=is_complex))
            c = out_c
        k, s, p = architecture[0][1:]
        self.layers.append(ConvTransposeBlock(2 * c, mask_channels, k, stride=s, padding=p,
                                              is_complex=is_complex, act=False))

    def forward(self, x, encoder_outputs=None):
        for layer in self.layers:
            if encoder_outputs is not None:
                skip = encoder_outputs.pop()
                # dcunet.py:89-93: x zero-padded to the skip's grid, then a plain torch.cat (not
                # complex_concat); folded into the convT's GEMMs where a joined kernel exists
                y = layer.forward_joined(x, skip)
                if y is not None:
                    x = y
                    continue
                if skip.shape != x.shape:                      # dcunet.py:89-92
                    x = TF.pad(x, (0, abs(skip.shape[3] - x.shape[3]), 0, abs(skip.shape[2] - x.shape[2])))
                x = torch.cat([x, skip], dim=1)                # plain cat, not complex_concat (:93)
            x = layer(x)
        return x


class DCUNet(nn.Module):
    """dcunet.py:98-189."""

    def __init__(self, config, window_size=512, hop_size=128, fft_size=512, normalize=False,
                 is_complex=True):
        super().__init__()
        arch = dcunet_architecture[config]
        enc_channels = _width(arch[0], is_complex)
        dec_channels = _width(arch[-1], is_complex)
        mask_channels = 2 if is_complex else 1
        self.window_size, self.hop_size, self.fft_size, self.normalize = window_size, hop_size, fft_size, normalize
        self.stft = ConvSTFT(window_size, hop_size, fft_size)
        self.istft = ConviSTFT(window_size, hop_size, fft_size)
        self.first_conv = ConvBlock(in_channels=mask_channels, out_channels=enc_channels, kernel_size=3,
                                    padding=1, is_complex=is_complex)
        mark_data_fed(self.first_conv)               # the noisy spectrum enters here
        self.encoder = Encoder(arch, enc_channels, is_complex)
        self.decoder = Decoder(arch, dec_channels, mask_channels, is_complex)

    def forward(self, x):
        half = self.fft_size // 2 + 1
        spec = self.stft(x)
        noisy = spec.view(spec.shape[0], 2, half, spec.shape[-1])
        if self.normalize:                                      # dcunet.py:127-130
            noisy = (noisy - noisy.mean(dim=[1, 2, 3], keepdim=True)) / \
                    (noisy.std(dim=[1, 2, 3], keepdim=True) + 1e-8)
        h, skips = self.encoder(self.first_conv(noisy))
        h = self.decoder(h, skips)
        dh, dw = abs(h.shape[2] - noisy.shape[2]), abs(h.shape[3] - noisy.shape[3])   # :141-146
        if dh:
            h = h[:, :, :-dh]
        if dw:
            h = h[:, :, :, :-dw]
        est = self._mask_processing(h, noisy)
        b, c, f, t = est.shape
        est = est.reshape(b, c * f, t)
        return est, glue.clamp(self.istft(est), -1, 1)

    def _mask_processing(self, x, noisy_spec, method="bounded_tanh"):
        """dcunet.py:158-184."""
        if method == "unbounded":
            return noisy_spec * x
        if method == "bounded_sigmoid":
            return noisy_spec * torch.sigmoid(x)
        fused = F.polar_mask_nograd(x[:, 0], x[:, 1], noisy_spec[:, 0], noisy_spec[:, 1], 0)
        if fused is not None:   # inference: one pass (se_polar_mask_fwd), the same values
            return fused
        m_mag, m_ph = self._return_mag_phase(x[:, 0], x[:, 1])
        n_mag, n_ph = self._return_mag_phase(noisy_spec[:, 0], noisy_spec[:, 1])
        ph = n_ph + m_ph / m_mag
        gain = n_mag * torch.tanh(m_mag)
        return torch.stack([gain * torch.cos(ph), gain * torch.sin(ph)], dim=1)

    @staticmethod
    def _return_mag_phase(real, imag, eps=1e-8):
        return torch.sqrt(real ** 2 + imag ** 2 + eps), torch.atan2(imag, real)
