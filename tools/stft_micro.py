"""ConvSTFT / ConviSTFT fwd+bwd at the FRCRN bench shape (B=64, 4 s, 320/160/640):
per-launch time over a burst of back-to-back launches and GB/s of the algorithmic
bytes (wav read once + spectrum written once). Optional argv[1]: run only the
named op (stft_fwd / istft_fwd / istft_bwd), e.g. for a PMC pass. STFT_B=n: batch n
instead of 64 (per-launch time against the batch shows whether the grid's last round
of workgroups dominates)."""
import os, sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "speech-enhancement_amd"))
from sehip.conv_stft import ConvSTFT, ConviSTFT  # noqa: E402

dev = torch.device("cuda")
B, L = int(os.environ.get("STFT_B", "64")), 64000
x = torch.randn(B, 1, L, device=dev) * 0.3
st, ist = ConvSTFT(320, 160, 640).to(dev), ConviSTFT(320, 160, 640).to(dev)
with torch.no_grad():
    spec = st(x)
nbytes = 4 * (x.numel() + spec.numel())
from sehip import functional as F  # noqa: E402
# launched straight into preallocated buffers, as bench.py's bursts (no autograd / allocation)
x2 = x[:, 0].contiguous()
wav = ist(spec)
off = ist.pad if ist.center else 0
wav_buf, gspec, gy = torch.empty_like(wav), torch.empty_like(spec), torch.randn_like(wav)
with torch.no_grad():
    only = sys.argv[1] if len(sys.argv) > 1 else None
    for name, f in (("stft_fwd", lambda: F.stft_launch(x2, spec, None, st._win, st._tw, st.window_size, st.hop_size,
                                                       st.fft_size, st.center, False)),
                    ("istft_fwd", lambda: F.istft_launch(spec, wav_buf, ist._win, ist._tw, ist.window_size,
                                                         ist.hop_size, ist.fft_size, off, wav.shape[-1])),
                    ("istft_bwd", lambda: F.istft_bwd_launch(gy, gspec, ist._win, ist._tw, ist.window_size,
                                                             ist.hop_size, ist.fft_size, off, wav.shape[-1]))):
        if only and name != only:
            continue
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 50
        print(f"{name:9s} {ms * 1e3:7.1f} us  {nbytes / ms / 1e6:7.1f} GB/s", flush=True)
