"""Oracle complex-valued layers on channel-stacked [re; im] tensors.

Restates /root/reference/models/modules/complex_nn.py (test infrastructure
only). The complex convs are kept in the reference's four-real-conv form so
the oracle is an independent check of the HIP path's fused block-weight GEMM.
"""
from __future__ import annotations

import torch
import torch.nn as nn


def split_complex(x, dim=1):
    """complex_nn.py:18-30."""
    if isinstance(x, (tuple, list)):
        return x[0], x[1]
    if torch.is_complex(x):
        return x.real, x.imag
    if isinstance(x, torch.Tensor):
        return torch.chunk(x, 2, dim=dim)
    raise ValueError("Input must be a complex tensor or a tuple of real and imaginary tensors")


def merge_real_imag(x, real, imag, dim=1):
    """complex_nn.py:32-42 — same container kind as x."""
    if isinstance(x, (tuple, list)):
        return [real, imag]
    if torch.is_complex(x):
        return torch.complex(real, imag)
    return torch.cat([real, imag], dim=dim)


def complex_concat(inputs, dim=1):
    """complex_nn.py:4-16: [x_re, e_re, ..., x_im, e_im, ...]."""
    parts = [torch.chunk(t, 2, dim=dim) for t in inputs]
    return torch.cat([p[0] for p in parts] + [p[1] for p in parts], dim=dim)


def _half(n, what):
    assert n % 2 == 0, f"{what} must be a factor of 2, current channels: {n}"
    return n // 2


class _ComplexConvBase(nn.Module):
    """complex_nn.py:44-65: four real convs, re = Wr*xr - Wi*xi, im = Wi*xr + Wr*xi."""

    def forward(self, x):
        xr, xi = split_complex(x)
        re = self.real_conv(xr) - self.imag_conv(xi)
        im = self.imag_conv(xr) + self.real_conv(xi)
        return merge_real_imag(x, re, im)


class ComplexConv2d(_ComplexConvBase):
    """complex_nn.py:67-78."""

    def __init__(self, in_channels, out_channels, kernel_size, **kwargs):
        super().__init__()
        cin, cout = _half(in_channels, "in_channels"), _half(out_channels, "out_channels")
        self.real_conv = nn.Conv2d(cin, cout, kernel_size, **kwargs)
        self.imag_conv = nn.Conv2d(cin, cout, kernel_size, **kwargs)


class ComplexConvTranspose2d(_ComplexConvBase):
    """complex_nn.py:80-91."""

    def __init__(self, in_channels, out_channels, kernel_size, **kwargs):
        super().__init__()
        cin, cout = _half(in_channels, "in_channels"), _half(out_channels, "out_channels")
        self.real_conv = nn.ConvTranspose2d(cin, cout, kernel_size, **kwargs)
        self.imag_conv = nn.ConvTranspose2d(cin, cout, kernel_size, **kwargs)


class ComplexLinear(nn.Module):
    """complex_nn.py:93-113 — separate real/imag linears, no cross terms."""

    def __init__(self, in_channels, out_channels, **kwargs):
        super().__init__()
        cin, cout = _half(in_channels, "in_channels"), _half(out_channels, "out_channels")
        self.real_linear = nn.Linear(cin, cout, **kwargs)
        self.imag_linear = nn.Linear(cin, cout, **kwargs)

    def forward(self, x):
        xr, xi = split_complex(x, dim=-1)
        return merge_real_imag(x, self.real_linear(xr), self.imag_linear(xi), dim=-1)


class ComplexLSTM(nn.Module):
    """complex_nn.py:115-145 — four LSTM applications."""

    def __init__(self, in_channels, hidden_channels, **kwargs):
        super().__init__()
        cin, hid = _half(in_channels, "in_channels"), _half(hidden_channels, "hidden_channels")
        self.real_lstm = nn.LSTM(cin, hid, **kwargs)
        self.imag_lstm = nn.LSTM(cin, hid, **kwargs)

    def forward(self, x):
        xr, xi = split_complex(x, dim=-1)
        re = self.real_lstm(xr)[0] - self.imag_lstm(xi)[0]
        im = self.imag_lstm(xr)[0] + self.real_lstm(xi)[0]
        return merge_real_imag(x, re, im, dim=-1)

    def flatten_parameters(self):
        self.real_lstm.flatten_parameters()
        self.imag_lstm.flatten_parameters()


class ComplexBatchNorm2d(nn.Module):
    """complex_nn.py:148-329: 2x2 whitening batch norm (Trabelsi et al.)."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True,
                 track_running_stats=True, complex_axis=1):
        super().__init__()
        self.num_features = num_features // 2
        self.eps, self.momentum, self.affine = eps, momentum, affine
        self.track_running_stats, self.complex_axis = track_running_stats, complex_axis
        c = self.num_features
        for n in ("Wrr", "Wri", "Wii", "Br", "Bi"):
            if affine:
                setattr(self, n, nn.Parameter(torch.empty(c)))
            else:
                self.register_parameter(n, None)
        if track_running_stats:
            self.register_buffer("RMr", torch.zeros(c))
            self.register_buffer("RMi", torch.zeros(c))
            self.register_buffer("RVrr", torch.ones(c))
            self.register_buffer("RVri", torch.zeros(c))
            self.register_buffer("RVii", torch.ones(c))
            self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))
        else:
            for n in ("RMr", "RMi", "RVrr", "RVri", "RVii", "num_batches_tracked"):
                self.register_parameter(n, None)
        self.reset_parameters()

    def reset_parameters(self):                                      # :193-210
        if self.track_running_stats:
            self.RMr.zero_(); self.RMi.zero_(); self.RVri.zero_()
            self.RVrr.fill_(1); self.RVii.fill_(1); self.num_batches_tracked.zero_()
        if self.affine:
            with torch.no_grad():
                self.Br.zero_(); self.Bi.zero_()
                self.Wrr.fill_(1); self.Wii.fill_(1)
                self.Wri.uniform_(-.9, .9)

    def forward(self, inputs):
        xr, xi = torch.chunk(inputs, 2, dim=self.complex_axis)      # :218
        factor = 0.0
        if self.training and self.track_running_stats:               # :221-226
            self.num_batches_tracked += 1
            factor = (1.0 / self.num_batches_tracked.item()) if self.momentum is None else self.momentum
        batch_stats = self.training or not self.track_running_stats  # :234
        red = [d for d in range(xr.dim()) if d != 1]
        shp = [1] * xr.dim()
        shp[1] = xr.shape[1]
        if batch_stats:                                              # :244-251
            mr, mi = xr.mean(red, keepdim=True), xi.mean(red, keepdim=True)
            if self.track_running_stats:
                self.RMr.lerp_(mr.reshape(-1), factor)
                self.RMi.lerp_(mi.reshape(-1), factor)
        else:
            mr, mi = self.RMr.view(shp), self.RMi.view(shp)
        xr, xi = xr - mr, xi - mi                                    # :255
        if batch_stats:                                              # :263-274
            vrr = (xr * xr).mean(red, keepdim=True)
            vri = (xr * xi).mean(red, keepdim=True)
            vii = (xi * xi).mean(red, keepdim=True)
            if self.track_running_stats:
                self.RVrr.lerp_(vrr.reshape(-1), factor)
                self.RVri.lerp_(vri.reshape(-1), factor)
                self.RVii.lerp_(vii.reshape(-1), factor)
        else:
            vrr, vri, vii = self.RVrr.view(shp), self.RVri.view(shp), self.RVii.view(shp)
        vrr, vii = vrr + self.eps, vii + self.eps                    # :279-281
        # inverse square root of the 2x2 covariance (:288-297)
        s = torch.sqrt(vrr * vii - vri * vri)
        t = torch.sqrt(vrr + vii + 2 * s)
        r = 1.0 / (s * t)
        urr, uii, uri = (s + vii) * r, (s + vrr) * r, -vri * r
        if self.affine:                                              # :308-315
            wrr, wri, wii = self.Wrr.view(shp), self.Wri.view(shp), self.Wii.view(shp)
            zrr, zri = wrr * urr + wri * uri, wrr * uri + wri * uii
            zir, zii = wri * urr + wii * uri, wri * uri + wii * uii
        else:
            zrr, zri, zir, zii = urr, uri, uri, uii
        yr = zrr * xr + zri * xi                                     # :317-322
        yi = zir * xr + zii * xi
        if self.affine:
            yr, yi = yr + self.Br.view(shp), yi + self.Bi.view(shp)
        return torch.cat([yr, yi], self.complex_axis)


class ComplexPReLU(nn.Module):
    """complex_nn.py:337-357."""

    def __init__(self, **kwargs):
        super().__init__()
        self.real_prelu = nn.PReLU(**kwargs)
        self.imag_prelu = nn.PReLU(**kwargs)

    def forward(self, x):
        xr, xi = split_complex(x, dim=1)
        re = self.real_prelu(xr) - self.imag_prelu(xi)
        im = self.imag_prelu(xr) + self.real_prelu(xi)
        return merge_real_imag(x, re, im, dim=1)


ComplexReLU = nn.ReLU            # complex_nn.py:359
ComplexLeakyReLU = nn.LeakyReLU  # complex_nn.py:360
