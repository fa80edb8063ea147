"""Fused BatchNorm2d + activation (csrc/bn.hip via norm.bn_act) against the
modules it replaces, act(norm(x)) with nn.BatchNorm2d + nn.PReLU (CARN,
models/_2104_05267_carn.py:30-56) or nn.ELU (CRN, _1809_01405_crn.py:9-45).

Oracle: the same nn modules on the CPU in fp64 (training and eval; outputs,
input / parameter gradients, running statistics). Tolerances: rel-L2 <= 1e-5
for outputs and gradients (fp32 kernels, fp64 statistics), running stats
<= 1e-5 relative."""
import copy

import pytest
import torch
import torch.nn as nn

from conftest import rel_l2

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return rel_l2(a.detach().double().cpu().numpy(), b.detach().double().cpu().numpy())


def _pair(C, act_kind):
    torch.manual_seed(C)
    norm = nn.BatchNorm2d(C)
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
        norm.bias.uniform_(-0.2, 0.2)
        norm.running_mean.uniform_(-0.1, 0.1)
        norm.running_var.uniform_(0.8, 1.2)
    if act_kind == "prelu":
        act = nn.PReLU()
    elif act_kind == "prelu_c":
        act = nn.PReLU(C, init=0.1)
    elif act_kind == "elu":
        act = nn.ELU(0.7)
    else:
        act = nn.Identity()
    return norm, act


@pytest.mark.parametrize("shape,act_kind,train,crop", [
    ((4, 16, 33, 50), "prelu", True, 0),
    ((3, 32, 9, 101), "prelu_c", True, 0),
    ((2, 64, 17, 40), "elu", True, 1),      # CRN: conv(x)[:, :, :-1, :] view
    ((4, 16, 33, 50), "prelu", False, 0),
    ((2, 24, 12, 31), "elu", False, 2),
    ((5, 8, 7, 13), "none", True, 0),
])
def test_bn_act_matches_modules(gpu_device, shape, act_kind, train, crop):
    from sehip.norm import bn_act
    norm, act = _pair(shape[1], act_kind)
    rn, ra = copy.deepcopy(norm).double(), copy.deepcopy(act).double()
    rn.train(train)
    ra.train(train)
    full = torch.randn(shape[0], shape[1], shape[2] + crop, shape[3]) * 1.3 + 0.4
    xr = full.double().requires_grad_(True)
    yr = ra(rn(xr[:, :, :shape[2]] if crop else xr))
    gy = torch.randn(shape)
    (yr * gy.double()).sum().backward()
    dn, da = norm.to(gpu_device).train(train), act.to(gpu_device).train(train)
    xd = full.to(gpu_device).requires_grad_(True)
    y = bn_act(dn, da, xd[:, :, :shape[2]] if crop else xd)
    assert _rel(y, yr) < 1e-5
    (y * gy.to(gpu_device)).sum().backward()
    assert _rel(xd.grad, xr.grad) < 1e-5
    assert _rel(dn.weight.grad, rn.weight.grad) < 1e-5
    assert _rel(dn.bias.grad, rn.bias.grad) < 1e-5
    if act_kind.startswith("prelu"):
        assert _rel(da.weight.grad, ra.weight.grad) < 1e-5
    assert _rel(dn.running_mean, rn.running_mean) < 1e-5
    assert _rel(dn.running_var, rn.running_var) < 1e-5
    assert int(dn.num_batches_tracked) == int(rn.num_batches_tracked)


def test_bn_act_fp16_eval(gpu_device):
    """model.half() inference (config 5): fp16 storage, fp32 arithmetic, fp16 out."""
    from sehip.norm import bn_act
    norm, act = _pair(16, "prelu")
    norm.eval()
    x = torch.randn(2, 16, 9, 20)
    ref = act(norm(x))
    y = bn_act(norm.to(gpu_device).half(), act.to(gpu_device).half(), x.to(gpu_device).half())
    assert y.dtype == torch.float16
    assert _rel(y.float(), ref) < 2e-3
