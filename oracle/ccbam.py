"""Oracle complex CBAM skip attention (FRCRN decoder).

Restates /root/reference/models/modules/ccbam.py (test infrastructure only).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .complex_nn import (ComplexBatchNorm2d, ComplexConv2d, ComplexLinear,
                         complex_concat, merge_real_imag, split_complex)


class ConvBlock(nn.Module):
    """ccbam.py:7-16: complex conv -> CBN -> ReLU."""

    def __init__(self, in_channels, out_channels, kernel_size, norm=True, act=True, **kwargs):
        super().__init__()
        self.conv = ComplexConv2d(in_channels, out_channels, kernel_size, bias=not norm, **kwargs)
        self.norm = ComplexBatchNorm2d(out_channels) if norm else nn.Identity()
        self.act = nn.ReLU() if act else nn.Identity()

    def forward(self, x):
        return self.act(self.norm(self.conv(x)))


class LinearBlock(nn.Module):
    """ccbam.py:18-26."""

    def __init__(self, in_channels, out_channels, act=True, **kwargs):
        super().__init__()
        self.linear = ComplexLinear(in_channels, out_channels, **kwargs)
        self.act = nn.ReLU() if act else nn.Identity()

    def forward(self, x):
        return self.act(self.linear(x))


class ChannelAttention(nn.Module):
    """ccbam.py:28-63: sigmoid(MLP(avgpool) + MLP(maxpool)) per channel."""

    def __init__(self, feature_map_channels, r=16):
        super().__init__()
        red = feature_map_channels // r or 2                          # :32-35
        self.avg_pool = nn.AdaptiveAvgPool2d((1, 1))
        self.max_pool = nn.AdaptiveMaxPool2d((1, 1))
        self.shared_fc_layer = nn.Sequential(
            LinearBlock(feature_map_channels, red, act=True, bias=False),
            LinearBlock(red, feature_map_channels, act=False, bias=False))

    def forward(self, x):
        b, c = x.shape[:2]
        # pooling each half and re-stacking them is a per-channel pool (:47-56)
        avg = self.avg_pool(x).flatten(1)
        mx = self.max_pool(x).flatten(1)
        att = torch.sigmoid(self.shared_fc_layer(avg) + self.shared_fc_layer(mx))
        return att.view(b, c, 1, 1)


class SpatialAttention(nn.Module):
    """ccbam.py:65-86: channel mean/max per half -> complex conv k7 -> sigmoid."""

    def __init__(self):
        super().__init__()
        self.conv = ConvBlock(in_channels=4, out_channels=2, kernel_size=7, padding=3)

    def forward(self, x):
        xr, xi = split_complex(x)
        avg = torch.cat([xr.mean(1, keepdim=True), xi.mean(1, keepdim=True)], 1)
        # torch.max(dim)[0] as at ccbam.py:79-80: the gradient goes to ONE index
        mx = torch.cat([torch.max(xr, 1, keepdim=True)[0], torch.max(xi, 1, keepdim=True)[0]], 1)
        return torch.sigmoid(self.conv(complex_concat([avg, mx], dim=1)))


class CCBAM(nn.Module):
    """ccbam.py:88-106: x*ca, then the 2-channel spatial map is ADDED to re/im."""

    def __init__(self, feature_map_channels, reduction=16):
        super().__init__()
        self.channel_attention_branch = ChannelAttention(feature_map_channels, reduction)
        self.spatial_attention_branch = SpatialAttention()

    def forward(self, x):
        x = x * self.channel_attention_branch(x)
        sa = self.spatial_attention_branch(x)
        xr, xi = split_complex(x)
        return merge_real_imag(x, xr + sa[:, 0:1], xi + sa[:, 1:2], dim=1)
