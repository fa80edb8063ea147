"""The models' glue as HIP passes (sehip.glue -> csrc/glue.hip, ABI 10) against the
reference's torch forms of the same ops, on the GPU:

* contiguous / stack (se_copy_strided): bit-exact (copies and casts);
* clamp (the models' torch.clamp_(wav, -1, 1)): values and gradient bit-exact vs torch;
* ComplexLSTM re / im stacking and combination (complex_nn.py:128-142): fp32 bit-exact
  (one add or subtract), 16-bit: one rounding of the fp32 result;
* CARN's mask + cat (carn.py:161-168), attention gates (carn.py:59-76) and decoder cat
  (carn.py:112-113), GLU (carn.py:9-27): vs torch autograd of the reference op sequence
  in fp64 (fp32: rel-L2 <= 1e-6; fp16: the reference's own fp16 op sequence within 2 ulp-ish);
* long-form chunk split / overlap-add: bit-exact vs sehip.longform's torch form (CPU)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


@pytest.mark.parametrize("src_dt,dst_dt", [(torch.float32, torch.float32), (torch.bfloat16, torch.float32),
                                           (torch.float32, torch.float16), (torch.float16, torch.bfloat16)])
def test_contiguous_and_stack_bit_exact(gpu_device, src_dt, dst_dt):
    from sehip import glue
    torch.manual_seed(1)
    base = torch.randn(3, 5, 7, 11, device=gpu_device).to(src_dt)
    for view in (base.transpose(1, 3), base[:, 1:4, :, 2:9], base.permute(2, 0, 3, 1)):
        out = glue.contiguous(view, dst_dt)
        assert out.is_contiguous() and out.dtype == dst_dt
        assert torch.equal(out, view.to(dst_dt).contiguous())
    ts = [torch.randn(6, 9, device=gpu_device).to(src_dt).requires_grad_(True) for _ in range(3)]
    st = glue.stack(ts, dst_dt)
    assert torch.equal(st, torch.stack([t.to(dst_dt) for t in ts]))
    g = torch.randn_like(st)
    st.backward(g)
    for i, t in enumerate(ts):
        assert torch.equal(t.grad, g[i].to(src_dt))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_clamp_matches_torch(gpu_device, dtype):
    from sehip import glue
    torch.manual_seed(2)
    x = (torch.randn(4, 3001, device=gpu_device) * 1.2).to(dtype)
    x[0, :5] = torch.tensor([1.0, -1.0, 1.5, -1.5, 0.0], dtype=dtype)   # the boundary values pass the gradient
    a = x.clone().requires_grad_(True)
    b = x.clone().requires_grad_(True)
    ya = glue.clamp(a * 1, -1, 1)
    yb = torch.clamp_(b * 1, -1, 1)
    assert torch.equal(ya, yb)
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    assert torch.equal(a.grad, b.grad)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("feature_major", [False, True])
def test_complex_lstm_glue(gpu_device, dtype, feature_major):
    """stack_re_im + combine == the reference's split / four outputs / sub / add / merge."""
    from sehip import glue
    torch.manual_seed(3)
    B, T, I, H = 3, 17, 10, 8
    x = torch.randn(B, I * 2, T, device=gpu_device).to(dtype).transpose(1, 2).requires_grad_(True)  # a strided view
    both = glue.stack_re_im(x)
    assert both.dtype == torch.float32 and both.shape == (2 * B, T, I)
    assert torch.equal(both, torch.cat(torch.chunk(x.float(), 2, dim=-1), dim=0))
    h = torch.randn(2, 2 * B, T, H, device=gpu_device, requires_grad=True)
    out = glue.complex_lstm_combine(h, dtype, feature_major)
    r2r, i2r = h[0, :B], h[0, B:]
    r2i, i2i = h[1, :B], h[1, B:]
    ref = torch.cat([r2r - i2i, r2i + i2r], dim=-1).to(dtype)
    assert out.shape == ref.shape and torch.equal(out, ref)
    if feature_major:
        assert out.transpose(1, 2).is_contiguous()
    g = torch.randn(B, T, 2 * H, device=gpu_device).to(dtype)
    out.backward(g)
    gr, gi = g.float()[..., :H], g.float()[..., H:]
    want = torch.stack([torch.cat([gr, gi]), torch.cat([gi, -gr])])
    assert torch.equal(h.grad, want)
    gx = torch.randn(2 * B, T, I, device=gpu_device)
    both.backward(gx)
    assert torch.equal(x.grad, torch.cat([gx[:B], gx[B:]], dim=-1).to(dtype))


def _carn_ref(m, spec, half):
    mr, mi = m[:, 0], m[:, 1]
    nr, ni = spec[:, :half], spec[:, half:]
    return torch.cat([mr * nr - mi * ni, mr * ni - mi * nr], dim=1)   # carn.py:165-168


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_carn_mask_vs_reference_ops(gpu_device, dtype):
    from sehip import glue
    torch.manual_seed(4)
    B, half, T = 2, 257, 101
    m = torch.randn(B, 2, half, T, device=gpu_device).to(dtype).requires_grad_(True)
    spec = torch.randn(B, 2 * half, T, device=gpu_device).to(dtype).requires_grad_(True)
    est = glue.carn_mask(m, spec, half)
    ref16 = _carn_ref(m.detach(), spec.detach(), half)        # the reference's own op sequence in `dtype`
    if dtype == torch.float32:
        assert torch.equal(est, ref16)
    else:
        assert (est.float() - ref16.float()).abs().max().item() <= 2 * 2 ** -10 * ref16.float().abs().max().item()
    g = torch.randn_like(est)
    est.backward(g)
    m64 = m.detach().double().cpu().requires_grad_(True)
    s64 = spec.detach().double().cpu().requires_grad_(True)
    _carn_ref(m64, s64, half).backward(g.double().cpu())
    bar = 1e-6 if dtype == torch.float32 else 2 ** -10
    assert _rel(m.grad, m64.grad) < bar
    assert _rel(spec.grad, s64.grad) < bar


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_carn_attention_gates_vs_reference_ops(gpu_device, dtype):
    """add_sigmoid + gate_cat (the decoder's cat([sigmoid(conv3 s) * skip, skip])) and glu."""
    from sehip import glue
    torch.manual_seed(5)
    shape = (2, 16, 19, 33)
    a, b, c, skip = [torch.randn(shape, device=gpu_device).to(dtype).requires_grad_(True) for _ in range(4)]
    s1 = glue.add_sigmoid(a, b)
    out = glue.gate_cat(c * s1, skip)
    y = glue.glu(a, c)
    ref = [t.detach().double().cpu().requires_grad_(True) for t in (a, b, c, skip)]
    ra, rb, rc, rskip = ref
    rs1 = torch.sigmoid(ra + rb)
    rout = torch.cat([torch.sigmoid(rc * rs1) * rskip, rskip], dim=1)
    ry = ra * torch.sigmoid(rc)
    bar = 1e-6 if dtype == torch.float32 else 2 ** -10
    assert _rel(out, rout) < bar and _rel(y, ry) < bar
    g1, g2 = torch.randn_like(out), torch.randn_like(y)
    (out * g1).sum().add((y * g2).sum()).backward()
    (rout * g1.double().cpu()).sum().add((ry * g2.double().cpu()).sum()).backward()
    bar = 1e-6 if dtype == torch.float32 else 4 * 2 ** -10
    for t, r in zip((a, b, c, skip), ref):
        assert _rel(t.grad, r.grad) < bar, _rel(t.grad, r.grad)


@pytest.mark.parametrize("L,chunk,overlap,dtype", [(10007, 3000, 500, torch.float32), (1440000, 192000, 2400,
                                                   torch.float16), (6000, 3000, 0, torch.float32),
                                                   (9000, 3000, 1700, torch.float32)])
def test_chunk_split_overlap_add_vs_torch_form(gpu_device, L, chunk, overlap, dtype):
    from sehip import longform as LF
    torch.manual_seed(6)
    x = torch.randn(L).to(dtype)
    c_cpu = LF.split_chunks(x, chunk, overlap)
    c_gpu = LF.split_chunks(x.to(gpu_device), chunk, overlap)
    assert torch.equal(c_gpu.cpu(), c_cpu)
    y = torch.randn(c_cpu.shape).to(dtype)
    ref = LF.overlap_add(y.float(), L, overlap) if dtype == torch.float16 else LF.overlap_add(y, L, overlap)
    out = LF.overlap_add(y.to(gpu_device), L, overlap).cpu()
    if dtype == torch.float32:
        assert torch.equal(out, ref)
    else:   # fp16 steps of the same arithmetic
        assert (out.float() - ref).abs().max().item() <= 2 ** -9 * ref.abs().max().item()
