"""The fused ConvFFN (dfm_convffn_fwd / dfm_convffn_bwd, csrc/convffn.hip) against a float64 torch
restatement of DFormer's MLP inside the Block residual (models/encoders/DFormer.py:48-67, 176-179)
on the same 16-bit inputs, and against the op-level kernel chain it replaces (functional.FUSED_FFN =
False): every output and gradient of the fused path must be as close to float64 as the unfused
chain's (both round h, GELU(hpre), dhpre and dh to the 16-bit dtype at the same points)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    from dformer_amd import kernels  # noqa: F401


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def make_case(B, H, W, C, R, dt, seed, droppath):
    g = torch.Generator(device=DEV).manual_seed(seed)

    def rn(*s, sc=1.0):
        return torch.randn(*s, device=DEV, generator=g) * sc

    P = B * H * W
    p = dict(ln_w=1.0 + 0.2 * rn(C), ln_b=0.1 * rn(C), w1=rn(R, C, sc=C ** -0.5), b1=0.1 * rn(R),
             wpos=rn(R, 1, 3, 3, sc=1 / 3), bpos=0.1 * rn(R), w2=rn(C, R, sc=R ** -0.5), b2=0.1 * rn(C),
             ls=0.5 + 0.5 * torch.rand(C, device=DEV, generator=g))
    # the kernels read 16-bit weight copies: round the fp32 masters to that grid so both paths and
    # the float64 reference see the same weights
    p["w1"] = p["w1"].to(dt).float()
    p["w2"] = p["w2"].to(dt).float()
    x = rn(P, C).to(dt)
    dout = rn(P, C, sc=0.5).to(dt)
    rowscale = (torch.tensor([0.0, 1.25] * B, device=DEV)[:B] if droppath else None)
    return p, x, dout, rowscale


def ref64(p, x, shape, rowscale):
    B, H, W = shape
    P, C = x.shape
    R = p["w1"].shape[0]
    d = {k: v.double().detach().requires_grad_(True) for k, v in p.items()}
    xd = x.double().detach().requires_grad_(True)
    xn = F.layer_norm(xd, (C,), d["ln_w"], d["ln_b"], 1e-6)
    h = xn @ d["w1"].t() + d["b1"]
    hc = h.view(B, H, W, R).permute(0, 3, 1, 2)
    hp = F.conv2d(hc, d["wpos"], d["bpos"], padding=1, groups=R) + hc
    g = F.gelu(hp.permute(0, 2, 3, 1).reshape(P, R))
    f = g @ d["w2"].t() + d["b2"]
    rs = rowscale.double().repeat_interleave(H * W)[:, None] if rowscale is not None else 1.0
    out = xd + rs * d["ls"] * f
    return out, xd, d


def run_fn(p, x, dout, shape, rowscale, fused):
    from dformer_amd import functional as Fn
    # fresh parameter tensors can reuse a freed one's id() and address: drop the 16-bit weight cache
    Fn.invalidate_weights()
    prm = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    xr = x.clone().requires_grad_(True)
    old = Fn.FUSED_FFN
    Fn.FUSED_FFN = fused
    try:
        out = Fn.ConvFFNFn.apply(xr, shape, rowscale, prm["ln_w"], prm["ln_b"], prm["w1"], prm["b1"], prm["wpos"],
                                 prm["bpos"], prm["w2"], prm["b2"], prm["ls"])
        out.backward(dout)
    finally:
        Fn.FUSED_FFN = old
    torch.cuda.synchronize()
    return out.detach(), xr.grad, {k: v.grad for k, v in prm.items()}


CASES = [  # B, H, W, C, hidden: DFormer-B stages (mlp and mlp_e2), Tiny / odd planes, partial tiles
    (2, 120, 160, 64, 512), (2, 120, 160, 32, 256), (2, 60, 80, 128, 1024), (2, 60, 80, 64, 512),
    (3, 30, 40, 256, 1024), (3, 30, 40, 128, 512), (2, 11, 13, 64, 512), (1, 17, 23, 128, 512),
    (2, 7, 9, 256, 1024), (1, 33, 41, 32, 128),
]


@pytest.mark.parametrize("mode", [True, "fwd"])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CASES)
def test_convffn_fused_vs_float64_and_unfused(dt, case, mode):
    """mode True: fused forward and backward; "fwd": the fused forward storing GELU / GELU' for the
    op-level backward."""
    from dformer_amd import kernels as Kk
    B, H, W, C, R = case
    shape = (B, H, W)
    if not Kk.convffn_supported(dt, shape, C, R):
        pytest.skip(f"no fused kernel for C={C} (op-level chain)")
    p, x, dout, rowscale = make_case(B, H, W, C, R, dt, seed=C + R + H, droppath=(H % 2 == 0))
    out64, x64, d64 = ref64(p, x, shape, rowscale)
    out64.backward(dout.double())
    ref_g = {k: v.grad for k, v in d64.items()}
    fo, fdx, fg = run_fn(p, x, dout, shape, rowscale, mode)
    uo, udx, ug = run_fn(p, x, dout, shape, rowscale, False)
    rows = [("out", fo, uo, out64), ("dx", fdx, udx, x64.grad)] + [(k, fg[k], ug[k], ref_g[k]) for k in p]
    floor = 4e-3 if dt == torch.bfloat16 else 1e-3
    report = []
    for name, a, u, r in rows:
        ef, eu = rel(a, r), rel(u, r)
        report.append(f"{name} {ef:.2e}/{eu:.2e}")
        assert torch.isfinite(a).all(), name
        assert ef <= max(1.5 * eu, floor), (name, ef, eu, report)
    print(case, dt, mode, " ".join(report))


@pytest.mark.parametrize("case", [(2, 60, 80, 64, 512), (2, 40, 48, 32, 256)])
def test_convffn_fused_backward_bitwise_reproducible(case):
    B, H, W, C, R = case
    p, x, dout, rowscale = make_case(B, H, W, C, R, torch.bfloat16, seed=5, droppath=True)
    a = run_fn(p, x, dout, (B, H, W), rowscale, True)
    b = run_fn(p, x, dout, (B, H, W), rowscale, True)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    for k in p:
        assert torch.equal(a[2][k], b[2][k]), k


def test_convffn_supported_shapes():
    from dformer_amd import kernels as Kk
    assert not Kk.convffn_supported(torch.float32, (2, 8, 8), 64, 512)  # fp32 parity path stays unfused
    assert not Kk.convffn_supported(torch.bfloat16, (2, 8, 8), 48, 384)  # DFormer-Large mlp_e2 s0
    assert not Kk.convffn_supported(torch.bfloat16, (2, 8, 8), 512, 2048)
    assert Kk.convffn_supported(torch.float16, (2, 8, 8), 64, 512)
