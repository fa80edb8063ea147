"""Oracle model forwards: FRCRN, DCCRN, DCUNet, CARN/GCARN, CRN.

Restates the reference models under /root/reference/models (test
infrastructure only) with the reference's module names so state_dicts are
interchangeable.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .ccbam import CCBAM
from .complex_nn import (ComplexBatchNorm2d, ComplexConv2d, ComplexConvTranspose2d,
                         ComplexLeakyReLU, ComplexLinear, ComplexLSTM, complex_concat)
from .stft import ConvSTFT, ConviSTFT


def _stacked_spec(spec, nfft, drop_dc):
    half = nfft // 2 + 1
    x = torch.stack([spec[:, :half], spec[:, half:]], dim=1)
    return x[:, :, 1:] if drop_dc else x


# ----------------------------------------------------------------- FRCRN ---
class _CausalBlock(nn.Module):
    """frcrn.py:11-59 / dccrn.py:11-57: left time pad -> (T)conv -> norm -> act."""

    def __init__(self, transposed, in_ch, out_ch, kernel, padding, act, complex_, **kw):
        super().__init__()
        self.causal, self.padding = True, padding
        conv = (ComplexConvTranspose2d if transposed else ComplexConv2d) if complex_ else \
            (nn.ConvTranspose2d if transposed else nn.Conv2d)
        norm = ComplexBatchNorm2d if complex_ else nn.BatchNorm2d
        m = conv(in_ch, out_ch, kernel, padding=(padding[0], 0), bias=False, **kw)
        setattr(self, "conv_transposed" if transposed else "conv", m)
        self.norm = norm(out_ch)
        self.act = act

    def forward(self, x):
        x = F.pad(x, (self.padding[1], 0, 0, 0))
        m = self.conv_transposed if hasattr(self, "conv_transposed") else self.conv
        return self.act(self.norm(m(x)))


class _Stack(nn.Module):
    def __init__(self):
        super().__init__()
        self.layers = nn.ModuleList()

    def forward(self, x):
        skips = []
        for layer in self.layers:
            x = layer(x)
            skips.append(x)
        return x, skips


class FRCRN(nn.Module):
    """frcrn.py:104-155."""

    def __init__(self, window_size=320, hop_size=160, fft_size=640, lstm_channels=256,
                 reduction_ratio=16, is_complex=True):
        super().__init__()
        self.stft = ConvSTFT(window_size, hop_size, fft_size)
        self.istft = ConviSTFT(window_size, hop_size, fft_size)
        self.encoder = _Stack()                                       # frcrn.py:62-76
        cin = 2
        for _ in range(6):
            self.encoder.layers.append(_CausalBlock(False, cin, 128, (5, 2), (0, 1),
                                                    nn.LeakyReLU(0.2), is_complex, stride=(2, 1)))
            cin = 128
        self.decoder = nn.Module()                                    # frcrn.py:78-102
        self.decoder.skip_connection_attention_layers = nn.ModuleList(
            [CCBAM(128, reduction_ratio) for _ in range(6)])
        self.decoder.layers = nn.ModuleList(
            [_CausalBlock(True, 256, 128, (5, 2), (0, 0), nn.LeakyReLU(0.2), is_complex, stride=(2, 1))
             for _ in range(6)])
        self.lstm = ComplexLSTM(256, lstm_channels, num_layers=2, bidirectional=False, batch_first=True)
        self.final_conv = nn.Conv2d(128, 2, kernel_size=(1, 2), bias=False)
        self.fft_size = fft_size

    def forward(self, x):
        noisy = _stacked_spec(self.stft(x), self.fft_size, drop_dc=True)   # :121-127
        h, skips = self.encoder(noisy)
        b, c, f, t = h.shape                                          # :133-137
        h = self.lstm(h.reshape(b, c * f, t).transpose(1, 2)).transpose(1, 2).reshape(b, c, f, t)
        for att, layer in zip(self.decoder.skip_connection_attention_layers, self.decoder.layers):
            skip = att(skips.pop())                                   # :92-93
            if h.shape[-1] > skip.shape[-1]:
                h = h[..., :-1]
            if h.shape[-2] < skip.shape[-2]:
                h = F.pad(h, (0, 0, 0, 1))
            h = layer(complex_concat([h, skip], dim=1))
        mask = torch.tanh(F.pad(self.final_conv(h), (0, 0, 1, 0)))   # :140-144
        est = F.pad(mask * noisy, (0, 0, 1, 0))                       # :145-146
        est = torch.cat([est[:, 0], est[:, 1]], dim=1)                # :149-152
        return est, torch.clamp_(self.istft(est), -1, 1)              # :153-155


# ----------------------------------------------------------------- DCCRN ---
class _DCCRNLSTM(nn.Module):
    """dccrn.py:59-86: two one-layer ComplexLSTMs + ComplexLinear, or (is_complex=False,
    :73-75) one two-layer nn.LSTM + nn.Linear."""

    def __init__(self, in_ch, hid, lin, bidirectional, is_complex=True, **kw):
        super().__init__()
        nd = 2 if bidirectional else 1
        if is_complex:
            self.layers = nn.ModuleList([
                ComplexLSTM(in_ch, hid, num_layers=1, bidirectional=bidirectional, **kw),
                ComplexLSTM(nd * hid, hid, num_layers=1, bidirectional=bidirectional, **kw),
                ComplexLinear(nd * hid, lin)])
        else:
            self.layers = nn.ModuleList([nn.LSTM(in_ch, hid, num_layers=2, bidirectional=bidirectional, **kw),
                                         nn.Linear(nd * hid, lin)])

    def forward(self, x):
        for layer in self.layers:
            x = layer(x)
            x = x[0] if isinstance(x, tuple) else x   # nn.LSTM returns (output, (h_n, c_n))
        return x


class DCCRN(nn.Module):
    """dccrn.py:123-212."""

    def __init__(self, config="dccrn-CL", window_size=400, hop_size=100, fft_size=512,
                 lstm_channels=256, linear_channels=1024, bidirectional=False, is_complex=True):
        super().__init__()
        if config in ("dccrn-C", "dccrn-R", "dccrn-E"):
            enc, self.masking = [32, 64, 128, 128, 256, 256], config[-1]
        else:
            enc, self.masking = [32, 64, 128, 256, 256, 256], "E"
        dec = enc[:-1][::-1] + [2]
        freq_ch = (fft_size // 2 // 2 ** len(enc)) * enc[-1]         # :135-136
        self.stft = ConvSTFT(window_size, hop_size, fft_size)
        self.istft = ConviSTFT(window_size, hop_size, fft_size)
        self.encoder = _Stack()
        cin = 2
        for c in enc:
            self.encoder.layers.append(_CausalBlock(False, cin, c, (5, 2), (2, 1), nn.PReLU(),
                                                    is_complex, stride=(2, 1)))
            cin = c
        self.decoder = nn.Module()
        self.decoder.layers = nn.ModuleList()
        cin = 256
        for c in dec:
            self.decoder.layers.append(_CausalBlock(True, cin * 2, c, (5, 2), (2, 0), nn.PReLU(),
                                                    is_complex, stride=(2, 1), output_padding=(1, 0)))
            cin = c
        self.lstm = _DCCRNLSTM(freq_ch, lstm_channels, linear_channels, bidirectional, is_complex, batch_first=True)
        self.fft_size = fft_size

    def forward(self, x):
        spec = self.stft(x)
        half = self.fft_size // 2 + 1
        nr, ni = spec[:, :half], spec[:, half:]
        h, skips = self.encoder(_stacked_spec(spec, self.fft_size, drop_dc=True))
        b, c, f, t = h.shape
        h = self.lstm(h.reshape(b, c * f, t).transpose(1, 2)).transpose(1, 2).reshape(b, c, f, t)
        for layer in self.decoder.layers:                             # :113-121
            skip = skips.pop()
            if h.shape[-1] > skip.shape[-1]:
                h = h[..., :-1]
            h = layer(complex_concat([h, skip], dim=1))
        h = F.pad(h, (0, 0, 1, 0))
        mr, mi = h[:, 0], h[:, 1]
        if mr.shape[-1] > nr.shape[-1]:                               # :175-177
            mr, mi = mr[..., :-1], mi[..., :-1]
        re, im = self._mask(nr, ni, mr, mi)
        est = torch.cat([re, im], dim=1)
        return est, torch.clamp_(self.istft(est), -1, 1)

    def _mask(self, nr, ni, mr, mi):
        """dccrn.py:187-212."""
        if self.masking == "R":
            return nr * mr, ni * mi
        if self.masking == "C":
            return nr * mr - ni * mi, nr * mi + ni * mr
        n_mag, n_ph = torch.sqrt(nr ** 2 + ni ** 2 + 1e-8), torch.atan2(ni, nr)
        m_mag = torch.sqrt(mr ** 2 + mi ** 2 + 1e-8)
        m_ph = torch.atan2(mi / m_mag, mr / m_mag)
        g = n_mag * torch.tanh(m_mag)
        return g * torch.cos(n_ph + m_ph), g * torch.sin(n_ph + m_ph)


# ---------------------------------------------------------------- DCUNet ---
# architectures.py:53-97: (complex ch, real ch), kernel, stride, padding
DCUNET_ARCH = {
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
    """dcunet.py:12-43: (T)conv -> norm -> LeakyReLU, no causal pad."""

    def __init__(self, transposed, cin, cout, k, act=True, complex_=True, slope=0.01, **kw):
        super().__init__()
        conv = (ComplexConvTranspose2d if transposed else ComplexConv2d) if complex_ else \
            (nn.ConvTranspose2d if transposed else nn.Conv2d)
        setattr(self, "conv_transposed" if transposed else "conv", conv(cin, cout, k, bias=False, **kw))
        self.norm = (ComplexBatchNorm2d if complex_ else nn.BatchNorm2d)(cout)
        self.act = ComplexLeakyReLU(slope) if act else nn.Identity()

    def forward(self, x):
        m = self.conv_transposed if hasattr(self, "conv_transposed") else self.conv
        return self.act(self.norm(m(x)))


class DCUNet(nn.Module):
    """dcunet.py:98-189."""

    def __init__(self, config, window_size=512, hop_size=128, fft_size=512, normalize=False,
                 is_complex=True):
        super().__init__()
        arch = DCUNET_ARCH[config]
        ch = (lambda spec: spec[0][0] * 2) if is_complex else (lambda spec: spec[0][1])
        self.window_size, self.hop_size, self.fft_size, self.normalize = window_size, hop_size, fft_size, normalize
        self.stft = ConvSTFT(window_size, hop_size, fft_size)
        self.istft = ConviSTFT(window_size, hop_size, fft_size)
        mask_ch = 2 if is_complex else 1
        enc_ch = ch(arch[0])
        self.first_conv = _Block(False, mask_ch, enc_ch, 3, complex_=is_complex, padding=1)
        self.encoder = _Stack()
        cin = enc_ch
        for spec in arch:                                             # dcunet.py:45-64
            cout = ch(spec)
            self.encoder.layers.append(_Block(False, cin, cout, spec[1], complex_=is_complex,
                                              stride=spec[2], padding=spec[3]))
            cin = cout
        self.decoder = nn.Module()                                    # dcunet.py:66-96
        self.decoder.layers = nn.ModuleList()
        cin = ch(arch[-1])
        for i in range(len(arch) - 1):
            k, s, p = arch[-i - 1][1:]
            cout = ch(arch[-i - 2])
            self.decoder.layers.append(_Block(True, cin * 2, cout, k, complex_=is_complex,
                                              slope=0.01, stride=s, padding=p))
            cin = cout
        k, s, p = arch[0][1:]
        self.decoder.layers.append(_Block(True, cin * 2, mask_ch, k, act=False, complex_=is_complex,
                                          stride=s, padding=p))

    def forward(self, x):
        spec = self.stft(x)
        ident = _stacked_spec(spec, self.fft_size, drop_dc=False)
        h = ident
        if self.normalize:                                            # :127-130
            h = (h - h.mean(dim=[1, 2, 3], keepdim=True)) / (h.std(dim=[1, 2, 3], keepdim=True) + 1e-8)
            ident = h
        h, skips = self.encoder(self.first_conv(h))
        for layer in self.decoder.layers:                             # :84-96
            skip = skips.pop()
            if skip.shape != h.shape:
                h = F.pad(h, (0, abs(skip.shape[3] - h.shape[3]), 0, abs(skip.shape[2] - h.shape[2])))
            h = layer(torch.cat([h, skip], dim=1))
        dh, dw = abs(h.shape[2] - ident.shape[2]), abs(h.shape[3] - ident.shape[3])   # :141-146
        if dh:
            h = h[:, :, :-dh]
        if dw:
            h = h[:, :, :, :-dw]
        est = self._mask(h, ident)
        b, c, f, t = est.shape
        est = est.reshape(b, c * f, t)
        return est, torch.clamp_(self.istft(est), -1, 1)

    @staticmethod
    def _mask(h, noisy):
        """dcunet.py:158-184 (bounded_tanh; mask_phase is divided by mask_mag)."""
        mr, mi, nr, ni = h[:, 0], h[:, 1], noisy[:, 0], noisy[:, 1]
        m_mag, m_ph = torch.sqrt(mr ** 2 + mi ** 2 + 1e-8), torch.atan2(mi, mr)
        n_mag, n_ph = torch.sqrt(nr ** 2 + ni ** 2 + 1e-8), torch.atan2(ni, nr)
        ph = n_ph + m_ph / m_mag
        g = n_mag * torch.tanh(m_mag)
        return torch.stack([g * torch.cos(ph), g * torch.sin(ph)], dim=1)


# ------------------------------------------------------------------ CARN ---
class _GLU(nn.Module):
    """carn.py:9-27."""

    def __init__(self, transposed, cin, cout, k, **kw):
        super().__init__()
        conv = nn.ConvTranspose2d if transposed else nn.Conv2d
        pre = "conv_transpose" if transposed else "conv"
        setattr(self, pre + "1", conv(cin, cout, k, **kw))
        setattr(self, pre + "2", conv(cin, cout, k, **kw))
        self.pre = pre

    def forward(self, x):
        return getattr(self, self.pre + "1")(x) * torch.sigmoid(getattr(self, self.pre + "2")(x))


class _RealBlock(nn.Module):
    """carn.py:30-56."""

    def __init__(self, transposed, cin, cout, k, gate, **kw):
        super().__init__()
        if gate:
            m = _GLU(transposed, cin, cout, k, bias=False, **kw)
        else:
            m = (nn.ConvTranspose2d if transposed else nn.Conv2d)(cin, cout, k, bias=False, **kw)
        setattr(self, "conv_transposed" if transposed else "conv", m)
        self.norm = nn.BatchNorm2d(cout)
        self.act = nn.PReLU()

    def forward(self, x):
        m = self.conv_transposed if hasattr(self, "conv_transposed") else self.conv
        return self.act(self.norm(m(x)))


class _Attention(nn.Module):
    """carn.py:59-76."""

    def __init__(self, c):
        super().__init__()
        self.conv1 = nn.Conv2d(c, 2 * c, 3, padding=1, bias=False)
        self.conv2 = nn.Conv2d(c, 2 * c, 3, padding=1, bias=False)
        self.conv3 = nn.Conv2d(2 * c, c, 3, padding=1, bias=False)

    def forward(self, x_u, x_c):
        a = torch.sigmoid(self.conv1(x_u) + self.conv2(x_c))
        return torch.sigmoid(self.conv3(a)) * x_c


class CARN(nn.Module):
    """carn.py:121-172."""

    def __init__(self, window_size=320, hop_size=160, fft_size=512, lstm_channels=512, gate=False):
        super().__init__()
        self.fft_size = fft_size
        self.stft = ConvSTFT(window_size, hop_size, fft_size)
        self.istft = ConviSTFT(window_size, hop_size, fft_size)
        self.encoder = _Stack()
        cin = 2
        for c in [16, 32, 64, 96, 128, 128]:                          # carn.py:78-93
            self.encoder.layers.append(_RealBlock(False, cin, c, (3, 3), gate, stride=(2, 1), padding=(1, 1)))
            cin = c
        self.decoder = nn.Module()                                    # carn.py:95-118
        self.decoder.conv_transpose_layers = nn.ModuleList()
        self.decoder.attention_layers = nn.ModuleList()
        cin = 128
        for c in [128, 96, 64, 32, 16, 2]:
            self.decoder.attention_layers.append(_Attention(cin))
            self.decoder.conv_transpose_layers.append(
                _RealBlock(True, cin * 2, c, (1, 3), gate, stride=(2, 1), padding=(0, 1), output_padding=(1, 0)))
            cin = c
        self.lstm = nn.LSTM(input_size=lstm_channels, hidden_size=lstm_channels, num_layers=2, batch_first=True)
        self.linear = nn.Linear(fft_size, fft_size + 2)

    def forward(self, x):
        spec = self.stft(x)
        half = self.fft_size // 2 + 1
        nr, ni = spec[:, :half], spec[:, half:]
        h, skips = self.encoder(_stacked_spec(spec, self.fft_size, drop_dc=True))
        b, c, f, t = h.shape
        h = self.lstm(h.reshape(b, c * f, t).transpose(1, 2))[0].transpose(1, 2).reshape(b, c, f, t)
        for att, layer in zip(self.decoder.attention_layers, self.decoder.conv_transpose_layers):
            skip = skips.pop()
            if h.shape[2] < skip.shape[2]:
                h = F.pad(h, (0, 0, 0, 1))
            h = layer(torch.cat([att(h, skip), skip], dim=1))
        h = self.linear(h.reshape(b, c * f, t).transpose(1, 2)).transpose(1, 2).reshape(b, 2, half, t)
        mr, mi = h[:, 0], h[:, 1]
        est = torch.cat([mr * nr - mi * ni, mr * ni - mi * nr], dim=1)   # carn.py:165-166 sign quirk
        return est, torch.clamp_(self.istft(est), -1, 1)


class GCARN(CARN):
    """carn.py:174-176."""

    def __init__(self, window_size=320, hop_size=160, fft_size=512, lstm_channels=512):
        super().__init__(window_size, hop_size, fft_size, lstm_channels, gate=True)


# ------------------------------------------------------------------- CRN ---
class _CRNBlock(nn.Module):
    """crn.py:9-41: conv -> causal crop -> BN -> ELU."""

    def __init__(self, transposed, cin, cout, k, norm=True, act=True, **kw):
        super().__init__()
        self.padding = kw.get("padding", (0, 0))
        m = (nn.ConvTranspose2d if transposed else nn.Conv2d)(cin, cout, k, bias=not norm, **kw)
        setattr(self, "conv_transposed" if transposed else "conv", m)
        self.norm = nn.BatchNorm2d(cout) if norm else nn.Identity()
        self.act = nn.ELU(1) if act else nn.Identity()
        self.transposed = transposed

    def forward(self, x):
        if self.transposed:
            x = self.conv_transposed(x)[:, :, :-1]
        else:
            x = self.conv(x)[:, :, :-self.padding[0]]
        return self.act(self.norm(x))


class CRN(nn.Module):
    """crn.py:82-109."""

    def __init__(self, window_size=320, hop_size=160, fft_size=320):
        super().__init__()
        self.stft = ConvSTFT(window_size, hop_size, fft_size, return_mag_phase=True)
        self.istft = ConviSTFT(window_size, hop_size, fft_size)
        self.encoder = _Stack()
        cin = 1
        for c in [16, 32, 64, 128, 256]:
            self.encoder.layers.append(_CRNBlock(False, cin, c, (2, 3), stride=(1, 2), padding=(1, 0)))
            cin = c
        self.lstm_layers = nn.LSTM(input_size=1024, hidden_size=1024, num_layers=2, batch_first=True)
        self.decoder = nn.Module()
        self.decoder.layers = nn.ModuleList()
        cin = 512
        for i, c in enumerate([128, 64, 32, 16, 1]):                  # crn.py:60-73
            kw = dict(stride=(1, 2))
            if i == 3:
                kw["output_padding"] = (0, 1)
            if i == 4:
                kw.update(norm=False, act=False)
            self.decoder.layers.append(_CRNBlock(True, cin, c, (2, 3), **kw))
            cin = c * 2

    def forward(self, x):
        mag, phase = self.stft(x)
        h, skips = self.encoder(mag.transpose(1, 2).unsqueeze(1))
        b, c, t, f = h.shape
        h = self.lstm_layers(h.permute(0, 2, 1, 3).reshape(b, t, c * f))[0]
        h = h.reshape(b, t, c, f).permute(0, 2, 1, 3)
        for layer in self.decoder.layers:
            h = layer(torch.cat([h, skips.pop()], dim=1))
        est = F.softplus(h).squeeze(1).transpose(1, 2)
        return est, self.istft(est, phase)
