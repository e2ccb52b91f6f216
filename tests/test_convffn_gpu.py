"""Fused ConvFFN kernels (csrc/convffn.hip) vs a plain PyTorch fp32 reference of the same op:
MLP (DFormer.py:48-67: LN -> fc1 -> DW3x3 + identity -> GELU -> fc2) inside the Block residual
with layer scale and a DropPath row scale (DFormer.py:173-179), forward and backward, at odd
image sizes, every channel width class, fp32 and bf16."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
TOL = {torch.float32: 2e-4, torch.bfloat16: 3e-2, torch.float16: 1e-2}


def rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30)).item()


def torch_ffn(x, shape, rs, p):
    B, H, W = shape
    C = x.shape[1]
    xn = F.layer_norm(x, (C,), p["ln_w"], p["ln_b"], 1e-6)
    h = xn @ p["w1"].t() + p["b1"]
    hid = h.shape[1]
    hi = h.view(B, H, W, hid).permute(0, 3, 1, 2)
    hp = F.conv2d(hi, p["wpos"], p["bpos"], padding=1, groups=hid) + hi
    g = F.gelu(hp).permute(0, 2, 3, 1).reshape(B * H * W, hid)
    f = g @ p["w2"].t() + p["b2"]
    rsx = rs.repeat_interleave(H * W)[:, None] if rs is not None else 1.0
    return x + rsx * p["ls"] * f


SHAPES = [(2, 11, 13, 32, 8), (1, 16, 20, 64, 8), (1, 17, 23, 48, 8), (2, 12, 16, 16, 8), (1, 30, 40, 64, 8),
          (2, 25, 37, 32, 4), (1, 8, 16, 64, 8), (1, 1, 1, 32, 8)]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,H,W,C,r", SHAPES)
def test_fused_convffn_matches_torch(dt, B, H, W, C, r):
    from dformer_amd import functional as Fn
    torch.manual_seed(C + H)
    hid = r * C
    gen = torch.Generator(device=DEV).manual_seed(1)
    p = {"ln_w": 1 + 0.1 * torch.randn(C, device=DEV), "ln_b": 0.1 * torch.randn(C, device=DEV),
         "w1": torch.randn(hid, C, device=DEV) / C ** 0.5, "b1": 0.1 * torch.randn(hid, device=DEV),
         "wpos": torch.randn(hid, 1, 3, 3, device=DEV) / 3, "bpos": 0.1 * torch.randn(hid, device=DEV),
         "w2": torch.randn(C, hid, device=DEV) / hid ** 0.5, "b2": 0.1 * torch.randn(C, device=DEV),
         "ls": 0.5 + 0.5 * torch.rand(C, device=DEV)}
    p = {k: v.requires_grad_() for k, v in p.items()}
    rs = torch.tensor([1.25, 0.0][:B], device=DEV) if B == 2 else None
    x = torch.randn(B * H * W, C, device=DEV, generator=gen)
    gy = torch.randn(B * H * W, C, device=DEV, generator=gen)
    xr = x.clone().requires_grad_()
    ref = torch_ffn(xr, (B, H, W), rs, p)
    ref.backward(gy)
    want = {k: v.grad.clone() for k, v in p.items()}
    for v in p.values():
        v.grad = None
    Fn.invalidate_weights()
    Fn.FUSED_FFN = True  # this test exercises the fused kernels whatever the default is
    assert Fn._ffn_fusable(x.to(dt), p["w1"])
    xd = x.to(dt).requires_grad_()
    out = Fn.ConvFFNFn.apply(xd, (B, H, W), rs, p["ln_w"], p["ln_b"], p["w1"], p["b1"], p["wpos"], p["bpos"],
                             p["w2"], p["b2"], p["ls"])
    out.backward(gy.to(dt))
    tol = TOL[dt]
    assert rel(out.float(), ref) < tol
    assert rel(xd.grad.float(), xr.grad) < tol * 2
    for k in ("w1", "b1", "wpos", "bpos", "w2", "b2", "ls", "ln_w", "ln_b"):
        assert rel(p[k].grad, want[k]) < tol * 2, k
    Fn.FUSED_FFN = Fn.os.environ.get("DFM_FUSED_FFN", "0") == "1"
