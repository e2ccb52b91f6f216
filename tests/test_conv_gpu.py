"""Native stem / downsample convolutions (ConvS2Fn, csrc/conv.hip) against torch fp32:
[BN(train|eval) [+ GELU] ->] nn.Conv2d(cin, cout, 3, 2, 1) forward and every gradient, on odd
image sizes and strided NCHW / channels-last inputs (DFormer.py:194-228, 295-303)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    torch.manual_seed(0)


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


TOL = {torch.float32: 1e-4, torch.bfloat16: 2e-2, torch.float16: 3e-3}


def _reference(x, conv, bn, gelu, train):
    """torch fp32: BN (batch or running statistics) -> GELU -> conv3x3 s2."""
    z = x
    run = None
    if bn is not None:
        run = (bn.running_mean.clone(), bn.running_var.clone())
        z = F.batch_norm(z, run[0], run[1], bn.weight, bn.bias, train, bn.momentum, bn.eps)
        if gelu:
            z = F.gelu(z)
    return F.conv2d(z, conv.weight, conv.bias, stride=2, padding=1), run


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,cin,cout,H,W,kind", [
    (2, 3, 16, 37, 50, "plain"),       # stem conv 1 on the raw float32 image (Cin = 3 -> Kp 32)
    (2, 1, 8, 21, 30, "plain"),        # depth stem conv 1 on the x_e[:, 0:1] view
    (2, 16, 32, 19, 25, "bn_gelu"),    # stem conv 2: BN -> GELU -> conv
    (3, 64, 128, 15, 20, "bn"),        # stage downsample: BN -> conv
    (2, 32, 64, 8, 11, "bn"),
    (2, 64, 128, 30, 40, "bn_eval"),
])
def test_conv_s2(dt, B, cin, cout, H, W, kind):
    from dformer_amd.encoder import ConvS2Fn
    conv = nn.Conv2d(cin, cout, 3, 2, 1).to(DEV)
    bn = None
    train = kind != "bn_eval"
    if kind != "plain":
        bn = nn.BatchNorm2d(cin).to(DEV)
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.5, 0.5)
            bn.running_mean.uniform_(-1, 1)
            bn.running_var.uniform_(0.5, 2)
        bn.train(train)
    gelu = kind == "bn_gelu"
    if kind == "plain" and cin == 1:
        src = torch.randn(B, 3, H, W, device=DEV)
        x = src[:, 0:1]                     # strided channel view, float32 (the depth stem input)
    elif kind == "plain":
        x = torch.randn(B, cin, H, W, device=DEV)  # contiguous NCHW float32 image
    else:
        # NCHW-logical view of NHWC rows (the previous stage's output), |mean| >> std channels
        rows = (torch.randn(B * H * W, cin, device=DEV) * 0.5 + 3.0).to(dt)
        x = rows.view(B, H, W, cin).permute(0, 3, 1, 2)
    x_ref = x.detach().float().clone().requires_grad_(True)
    x = x.detach().requires_grad_(True)  # keeps the strided view (image gradient for the plain stem conv)
    ref, run_ref = _reference(x_ref, conv, bn, gelu, train)
    y = ConvS2Fn.apply(x, conv.weight, conv.bias, bn.weight if bn is not None else None,
                       bn.bias if bn is not None else None, bn, False, gelu, dt)
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    assert y.shape == (B * Ho * Wo, cout) and y.dtype == dt
    y4 = y.view(B, Ho, Wo, cout).permute(0, 3, 1, 2).float()
    assert rel(y4, ref.detach()) < TOL[dt], rel(y4, ref.detach())
    if bn is not None:  # running statistics updated like torch (train) / untouched (eval)
        assert rel(bn.running_mean, run_ref[0]) < TOL[dt] and rel(bn.running_var, run_ref[1]) < TOL[dt]
    dy = torch.randn_like(ref)
    params = [conv.weight, conv.bias] + ([bn.weight, bn.bias] if bn is not None else [])
    g_ref = torch.autograd.grad(ref, [x_ref] + params, dy)
    ins = [x] + params
    g = torch.autograd.grad(y4, ins, dy)
    tol = TOL[dt] * (2 if dt != torch.float32 else 1)
    for a, b in zip(g, g_ref):
        assert a.shape == b.shape
        assert rel(a.float(), b) < tol, (a.shape, rel(a.float(), b))


def test_col2im_deterministic():
    """The input gradient is a fixed-order gather: two runs are bitwise equal."""
    from dformer_amd.encoder import ConvS2Fn
    B, cin, cout, H, W = 4, 64, 128, 30, 40
    conv = nn.Conv2d(cin, cout, 3, 2, 1).to(DEV)
    bn = nn.BatchNorm2d(cin).to(DEV)
    rows = torch.randn(B * H * W, cin, device=DEV).bfloat16()
    outs = []
    for _ in range(2):
        x = rows.view(B, H, W, cin).permute(0, 3, 1, 2).detach().requires_grad_(True)
        y = ConvS2Fn.apply(x, conv.weight, conv.bias, bn.weight, bn.bias, bn, False, True, torch.bfloat16)
        gx, = torch.autograd.grad(y, [x], torch.ones_like(y))
        outs.append(gx.contiguous(memory_format=torch.channels_last))
    assert torch.equal(outs[0], outs[1])
