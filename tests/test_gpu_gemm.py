"""se_gemm / se_colsum (csrc/gemm.hip): the LSTM layer GEMMs that replaced
torch.addmm / bmm on rocBLAS (the input projection and the weight / input
gradients of torch.nn.LSTM as ComplexLSTM runs it, complex_nn.py:115-145).

Oracle: the same products in fp64 with torch on the CPU. Bar: rel-L2 <= 2e-6
per product (the split-fp16 "f16x3" arithmetic of the conv GEMMs: 22-bit
operand splits, fp32 accumulation; measured ~3-6e-7), and the column sum
bit-exact against a sequential fp32 sum in the same chunk order.
The LSTM layer with these GEMMs is compared against SEHIP_LSTM_GEMM=torch
(rocBLAS) at FRCRN size; tests/test_gpu_lstm*.py compare it with nn.LSTM."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def _amax(t):
    return t.abs().max().reshape(1).float().clone()


CASES = [   # M, N, K, batches, sum_batches, a_mcontig, b_ncontig, kmask
    (130, 70, 45, 1, False, False, False, (0, 0)),     # tails in every dimension
    (257, 129, 96, 2, False, False, True, (0, 0)),
    (96, 200, 300, 3, True, False, True, (0, 0)),      # batch sum (dx of a shared input)
    (64, 48, 1000, 2, False, True, True, (7, 6)),      # weight-grad form, long K, masked rows
    (40, 256, 77, 1, False, True, False, (0, 0)),
]


@pytest.mark.parametrize("case", CASES)
def test_gemm_layouts_vs_fp64(gpu_device, case):
    from sehip import functional as F
    M, N, K, nb, sb, am, bn, km = case
    torch.manual_seed(1)
    # A(b, m, k), B(b, k, n) stored in the described layouts
    Am = torch.randn(nb, M, K, dtype=torch.float64) * torch.logspace(-2, 1, K, dtype=torch.float64)
    Bm = torch.randn(nb, K, N, dtype=torch.float64)
    if km[0]:
        mask = (torch.arange(K) % km[0] == km[1])
        Am_eff = Am.clone()
        Am_eff[:, :, mask] = 0
    else:
        Am_eff = Am
    A = (Am.transpose(1, 2) if am else Am).contiguous().float()
    B = (Bm if bn else Bm.transpose(1, 2)).contiguous().float()
    lda = M if am else K
    ldb = N if bn else K
    ref = torch.bmm(Am_eff, Bm)
    bias0 = torch.randn(nb, N)
    bias1 = torch.randn(nb, N)
    if sb:
        ref = ref.sum(0, keepdim=True)
        bias0, bias1 = bias0[:1], bias1[:1]
    ref = ref + bias0.double()[:, None, :] + bias1.double()[:, None, :]
    nbz = 1 if sb else nb
    ldc = N + 3
    C = torch.full((nbz, M, ldc), float("nan"), device=gpu_device)
    Ad, Bd = A.to(gpu_device), B.to(gpu_device)
    F.gemm(Ad, Bd, C, M=M, N=N, K=K, lda=lda, ldb=ldb, ldc=ldc, amax_a=_amax(Ad), amax_b=_amax(Bd),
           a_mcontig=am, b_ncontig=bn, batches=nb, sum_batches=sb, stride_a=M * K, stride_b=K * N,
           stride_c=M * ldc, bias0=bias0.to(gpu_device), bias1=bias1.to(gpu_device), stride_bias=N, kmask=km)
    torch.cuda.synchronize()
    assert torch.isnan(C[:, :, N:]).all()            # nothing written past N
    assert _rel(C[:, :, :N], ref) < 2e-6


def test_gemm_split_k_deterministic(gpu_device):
    """A weight-gradient-shaped product (K = 25792 rows) runs as split-K slabs added in
    split order: repeated calls are bit-identical."""
    from sehip import functional as F
    torch.manual_seed(2)
    R, G, I = 25792, 512, 128
    dg = torch.randn(R, G, device=gpu_device)
    x = torch.randn(R, I, device=gpu_device)
    outs = []
    for _ in range(2):
        C = torch.empty(G, I, device=gpu_device)
        F.gemm(dg, x, C, M=G, N=I, K=R, lda=G, ldb=I, ldc=I, amax_a=_amax(dg), amax_b=_amax(x),
               a_mcontig=True, b_ncontig=True)
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    assert _rel(outs[0], dg.double().t() @ x.double()) < 2e-6


@pytest.mark.parametrize("R", [1000, 51584, 37])
def test_colsum_exact(gpu_device, R):
    """Bit-exact against a sequential fp32 sum in the kernel's order (64 row chunks,
    each in row order, then the chunks in order); max |x| exact."""
    from sehip import _native as N
    from sehip import functional as F
    torch.manual_seed(3)
    L, G = 2, 300
    x = torch.randn(L, R, G, device=gpu_device)
    out = torch.empty(L, G, device=gpu_device)
    amax = torch.full((1,), 123.0, device=gpu_device)
    lib = N.lib()
    ws = F._workspace(lib.se_colsum_workspace_size(L, R, G), gpu_device)
    N.check(lib.se_colsum(x.data_ptr(), L, R, G, out.data_ptr(), amax.data_ptr(), ws.data_ptr(), ws.numel(),
                          N.stream_of(x)), "se_colsum")
    xc = x.cpu()
    rows = (R + 63) // 64
    parts = []
    for c0 in range(0, 64 * rows, rows):
        part = torch.zeros(L, G)
        for r in range(c0, min(R, c0 + rows)):
            part += xc[:, r]
        parts.append(part)
    ref = torch.zeros(L, G)
    for p in parts:
        ref += p
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), ref)
    assert amax.item() == xc.abs().max().item()


@pytest.mark.parametrize("rev", [0, 1, 2])
def test_lstm_layer_hip_gemm_vs_rocblas(gpu_device, monkeypatch, rev):
    """_LstmLayer with se_gemm (default) against SEHIP_LSTM_GEMM=torch (rocBLAS fp32):
    FRCRN's layer-0 form (one [B, T, 256] input shared by the real and imaginary LSTMs,
    H = 128) at B = 64 x 403 frames, with forward / reverse / mixed directions."""
    from sehip import functional as F
    torch.manual_seed(4)
    L, H, I, B, T = 2, 128, 256, 64, 403
    x = torch.randn(B, T, I, device=gpu_device) * 0.7
    w_ih = torch.randn(L, 4 * H, I, device=gpu_device) * 0.06
    w_hh = torch.randn(L, 4 * H, H, device=gpu_device) * 0.08
    b_ih = torch.randn(L, 4 * H, device=gpu_device) * 0.1
    b_hh = torch.randn(L, 4 * H, device=gpu_device) * 0.1
    gy = torch.randn(L, B, T, H, device=gpu_device)
    res = []
    for mode in ("torch", "hip"):
        monkeypatch.setenv("SEHIP_LSTM_GEMM", mode)
        ps = [t.clone().requires_grad_(True) for t in (x, w_ih, w_hh, b_ih, b_hh)]
        h = F.lstm_layer(*ps, rev_mask=rev)
        (h * gy).sum().backward()
        torch.cuda.synchronize()
        res.append([h.detach()] + [p.grad for p in ps])
    names = ("h", "dx", "dw_ih", "dw_hh", "db_ih", "db_hh")
    for n, a, b in zip(names, res[1], res[0]):
        assert _rel(a, b) < 1e-5, (n, _rel(a, b))
