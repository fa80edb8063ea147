"""Debug probe of se_gemm's 16-bit storage path: index-encoding inputs, decoded outputs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
import torch

from sehip import functional as F

dev = torch.device("cuda")
M = N = K = 32
for dt in (torch.float32, torch.float16, torch.bfloat16):
    for am in (False, True):
        for bn in (False, True):
            Am = (torch.arange(M)[:, None] + 32 * torch.arange(K)[None, :]).float() / (1 if dt != torch.bfloat16 else 8)
            Bm = torch.eye(K, N)
            A = (Am.t() if am else Am).contiguous().to(dt).to(dev)
            B = (Bm if bn else Bm.t()).contiguous().to(dt).to(dev)
            C = torch.zeros(M, N, device=dev, dtype=dt)
            amax = lambda t: t.float().abs().max().reshape(1).clone()
            F.gemm(A, B, C, M=M, N=N, K=K, lda=M if am else K, ldb=N if bn else K, ldc=N, a_mcontig=am, b_ncontig=bn,
                   amax_a=amax(A) if dt == torch.float32 else None, amax_b=amax(B) if dt == torch.float32 else None)
            ref = (Am @ Bm).to(dt).float()
            err = (C.float().cpu() - ref).abs().max().item()
            print(f"{dt} am={am} bn={bn}: max err {err}")
            if err:
                print("  C[0:3, 0:6] =", C.float().cpu()[0:3, 0:6].tolist())
                print("  ref         =", ref[0:3, 0:6].tolist())
            ones = torch.ones(M, K, device=dev, dtype=dt)
            C2 = torch.zeros(M, N, device=dev, dtype=dt)
            F.gemm(ones, torch.ones(N, K, device=dev, dtype=dt), C2, M=M, N=N, K=K, lda=K, ldb=K, ldc=N,
                   amax_a=amax(ones) if dt == torch.float32 else None, amax_b=amax(ones) if dt == torch.float32 else None)
            print("  ones: C2 unique", torch.unique(C2.float()).tolist()[:5])
