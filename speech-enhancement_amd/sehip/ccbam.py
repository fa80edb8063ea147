"""Complex CBAM skip attention (FRCRN decoder), HIP path.

Drop-in for /root/reference/models/modules/ccbam.py (same module tree and
state_dict keys). The spatial branch's ComplexConv2d(4->2, k7) + CBN + ReLU
run on the fused HIP kernels; the pooling / sigmoid glue is plain PyTorch
on the device for now (SURVEY.md §8f rank 2 fuses it).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .complex_nn import (ComplexBatchNorm2d, ComplexConv2d, ComplexLinear, complex_concat,
                         merge_real_imag, norm_act, split_complex)


class ConvBlock(nn.Module):
    """ccbam.py:7-16."""

    def __init__(self, in_channels, out_channels, kernel_size, norm=True, act=True, **kwargs):
        super().__init__()
        self.conv = ComplexConv2d(in_channels, out_channels, kernel_size, bias=not norm, **kwargs)
        self.norm = ComplexBatchNorm2d(out_channels) if norm else nn.Identity()
        self.act = nn.ReLU() if act else nn.Identity()

    def forward(self, x):
        return norm_act(self.norm, self.act, self.conv(x))


class LinearBlock(nn.Module):
    """ccbam.py:18-26."""

    def __init__(self, in_channels, out_channels, act=True, **kwargs):
        super().__init__()
        self.linear = ComplexLinear(in_channels, out_channels, **kwargs)
        self.act = nn.ReLU() if act else nn.Identity()

    def forward(self, x):
        return self.act(self.linear(x))


class ChannelAttention(nn.Module):
    """ccbam.py:28-63. The avg- and max-pooled descriptors go through the
    shared MLP as one stacked batch (same weights, one GEMM per layer)."""

    def __init__(self, feature_map_channels, r=16):
        super().__init__()
        reduction = feature_map_channels // r if feature_map_channels // r else 2
        self.avg_pool = nn.AdaptiveAvgPool2d((1, 1))
        self.max_pool = nn.AdaptiveMaxPool2d((1, 1))
        self.shared_fc_layer = nn.Sequential(
            LinearBlock(feature_map_channels, reduction, act=True, bias=False),
            LinearBlock(reduction, feature_map_channels, act=False, bias=False))

    def forward(self, x):
        b, c = x.shape[:2]
        pooled = torch.cat([x.mean(dim=(2, 3)), x.amax(dim=(2, 3))], dim=0)
        a, m = torch.chunk(self.shared_fc_layer(pooled), 2, dim=0)
        return torch.sigmoid(a + m).view(b, c, 1, 1)


class SpatialAttention(nn.Module):
    """ccbam.py:65-86."""

    def __init__(self):
        super().__init__()
        self.conv = ConvBlock(in_channels=4, out_channels=2, kernel_size=7, padding=3)

    def forward(self, x):
        re, im = split_complex(x)
        avg = torch.cat([re.mean(1, keepdim=True), im.mean(1, keepdim=True)], dim=1)
        mx = torch.cat([re.amax(1, keepdim=True), im.amax(1, keepdim=True)], dim=1)
        return torch.sigmoid(self.conv(complex_concat([avg, mx], dim=1)))


class CCBAM(nn.Module):
    """ccbam.py:88-106: channel gate (multiplicative), then the 2-channel
    spatial map ADDED to the real and the imaginary halves."""

    def __init__(self, feature_map_channels, reduction=16):
        super().__init__()
        self.channel_attention_branch = ChannelAttention(feature_map_channels, reduction)
        self.spatial_attention_branch = SpatialAttention()

    def forward(self, x):
        x = x * self.channel_attention_branch(x)
        sa = self.spatial_attention_branch(x)
        re, im = split_complex(x)
        return merge_real_imag(x, re + sa[:, 0:1], im + sa[:, 1:2], dim=1)
