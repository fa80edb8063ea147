"""Practical fp16 / bf16 MFMA ceiling on this box: hipBLASLt (torch.matmul) on random
operands, square and at the conv GEMMs' tall-skinny shapes (M = B*H*W positions,
K = taps * Cin, N = output columns), timed back to back with HIP events. The library's
rate on random data is what the DVFS-held clock allows a tuned GEMM; the conv GEMMs'
fractions are read against it.

Usage: python tools/mfma_ceiling.py"""
import torch

dev = torch.device("cuda")
SHAPES = [  # (name, M, N, K)
    ("square 8192", 8192, 8192, 8192),
    ("square 16384", 16384, 16384, 8192),
    ("dec5 data-grad-like (M=4.07M, N=256, K=640)", 64 * 158 * 403, 256, 640),
    ("dec5 fwd-like (M=2.04M, N=128, K=1536)", 64 * 79 * 403, 128, 1536),
    ("wgrad-like (M=1280, N=256, K=4.07M)", 1280, 256, 64 * 158 * 403),
]
for dt in (torch.float16, torch.bfloat16):
    for name, M, N, K in SHAPES:
        a = torch.randn(M, K, device=dev, dtype=dt)
        b = torch.randn(K, N, device=dev, dtype=dt)
        for _ in range(3):
            c = a @ b
        torch.cuda.synchronize()
        it = max(3, min(50, int(2e13 / (2 * M * N * K))))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            c = a @ b
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        tf = 2 * M * N * K / ms / 1e9
        print(f"{str(dt)[6:]:9s} {name:48s} {ms:8.3f} ms  {tf:7.1f} TFLOP/s  = {tf / 2500:.3f} of 2.5 PF", flush=True)
        del a, b, c
