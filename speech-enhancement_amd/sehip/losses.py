"""Training losses (drop-in for /root/reference/losses.py).

SI_SNR_loss on CUDA estimates (fp32, or the bf16 / fp16 tensors of a
model.to(bfloat16) / .half() run, read and written in that dtype) runs on the
HIP kernels (se_sisnr_fwd / se_sisnr_bwd, csrc/step.hip: one workgroup per
utterance, fp64 sums, one elementwise backward); si_snr_loss_aligned also
folds utils.py:105-121's mono reshape and pad / truncate of the estimate into
the kernel's reads. The other losses are plain PyTorch device ops."""
from __future__ import annotations

import torch

from . import _native as N


class _SiSnr(torch.autograd.Function):
    """est [B, le] (row stride est.stride(0)), target [B, lt]: -mean SI-SNR with
    the estimate zero-padded / truncated to lt (utils.py:111-121)."""

    @staticmethod
    def forward(ctx, est, target, zero_mean, eps):
        N.require_device(est, target, dtype=est.dtype)
        if est.stride(1) != 1:
            est = est.contiguous()
        target = target.contiguous()
        B, le = est.shape
        lt = target.shape[1]
        loss = torch.empty(1, device=est.device, dtype=est.dtype)
        save = torch.empty(int(N.lib().se_sisnr_save_bytes(B)), device=est.device, dtype=torch.uint8)
        N.check(N.lib().se_sisnr_fwd(est.data_ptr(), le, est.stride(0), target.data_ptr(), lt, B, int(zero_mean),
                                     float(eps), loss.data_ptr(), save.data_ptr(), N.dtype_code(est),
                                     N.stream_of(est)), "se_sisnr_fwd")
        ctx.save_for_backward(est, target, save)
        ctx.cfg = (int(zero_mean), float(eps))
        return loss.view(())

    @staticmethod
    def backward(ctx, gl):
        est, target, save = ctx.saved_tensors
        zero_mean, eps = ctx.cfg
        B, le = est.shape
        g = torch.empty((B, le), device=est.device, dtype=est.dtype)
        gl = gl.reshape(1)
        if gl.dtype != est.dtype:
            gl = gl.to(est.dtype)
        N.check(N.lib().se_sisnr_bwd(est.data_ptr(), le, est.stride(0), target.data_ptr(), target.shape[1], B,
                                     zero_mean, eps, save.data_ptr(), gl.data_ptr(), g.data_ptr(), le,
                                     N.dtype_code(est), N.stream_of(est)), "se_sisnr_bwd")
        return g, None, None, None


def _hip_sisnr_ok(estimate, target) -> bool:
    return (estimate.is_cuda and estimate.dtype in N.DTYPES and target.dtype == estimate.dtype
            and estimate.dim() == 2 and target.dim() == 2 and estimate.shape[0] == target.shape[0]
            and not target.requires_grad)


def si_snr_loss_aligned(estimate_wav, target_wav, zero_mean=False, eps=1e-8):
    """SI_SNR_loss(pad_or_truncate_wav(reshape_wav_to_mono(est), target), target)
    (trainer.py:107-113) with the reshape / pad / truncate folded into the kernel."""
    est = reshape_wav_to_mono(estimate_wav)
    tgt = reshape_wav_to_mono(target_wav)
    if _hip_sisnr_ok(est, tgt):
        return _SiSnr.apply(est, tgt, zero_mean, eps)
    return SI_SNR_loss(pad_or_truncate_wav(est, tgt), tgt, zero_mean, eps)


def SI_SNR_loss(estimate, target, zero_mean=False, eps=1e-8):
    """losses.py:62-84: negative mean scale-invariant SNR in dB."""
    if _hip_sisnr_ok(estimate, target) and estimate.shape[1] == target.shape[1]:
        return _SiSnr.apply(estimate, target, zero_mean, eps)
    if zero_mean:
        estimate = estimate - estimate.mean(dim=1, keepdim=True)
        target = target - target.mean(dim=1, keepdim=True)
    t_energy = target.pow(2).sum(dim=1, keepdim=True)
    proj = (estimate * target).sum(dim=1, keepdim=True) * target / t_energy
    signal = proj.pow(2).sum(dim=1) + eps
    noise = (estimate - proj).pow(2).sum(dim=1) + eps
    return -torch.mean(10 * torch.log10(signal / noise))


def SDR_loss(estimate, target, eps=1e-8):
    """losses.py:4-17: -mean 10 log10((|t|^2+eps) / (|t-e|^2+eps))."""
    t = target.pow(2).sum(dim=1) + eps
    e = (target - estimate).pow(2).sum(dim=1) + eps
    return -torch.mean(10 * torch.log10(t / e))


def reshape_wav_to_mono(wav):
    """utils.py:105-109."""
    if wav.dim() == 3:
        b, c, n = wav.shape
        wav = wav.reshape(b * c, n)
    return wav


def pad_or_truncate_wav(estimate_wav, target_wav):
    """utils.py:111-121."""
    le, lt = estimate_wav.shape[-1], target_wav.shape[-1]
    if le < lt:
        return torch.nn.functional.pad(estimate_wav, (0, lt - le))
    if le > lt:
        return estimate_wav[:, :lt]
    return estimate_wav
