"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op (GPU)."""
import math

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
    torch.manual_seed(0)


def K():
    from dformer_amd import kernels
    return kernels


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


TOL = {torch.float32: 2e-5, torch.bfloat16: 2e-2, torch.float16: 3e-3}
# GEMM gates: rel-to-max on identical (already rounded) 16-bit inputs with fp32 accumulation, so the
# only error left is the rounding of the 16-bit output (2^-9 relative for bf16, 2^-11 for fp16) plus
# accumulation order — about two output roundings, not percent-level drift
GTOL = {torch.float32: 2e-5, torch.bfloat16: 5e-3, torch.float16: 1.5e-3}
DTYPES = [torch.float32, torch.bfloat16, torch.float16]


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("M,N,Kd", [(300, 64, 64), (1000, 160, 96), (77, 33, 40), (4096, 512, 128), (5, 7, 16),
                                    (640, 1024, 256)])
def test_gemm_layouts(dt, M, N, Kd):
    k = K()
    x = torch.randn(M, Kd, device=DEV).to(dt)
    w = torch.randn(N, Kd, device=DEV).to(dt)
    b = torch.randn(N, device=DEV)
    y = k.linear(x, w, b)
    ref = x.float() @ w.float().t() + b
    assert rel(y.float(), ref) < GTOL[dt]
    dy = torch.randn(M, N, device=DEV).to(dt)
    dx = k.linear_dgrad(dy, w)
    assert rel(dx.float(), dy.float() @ w.float()) < GTOL[dt]
    dw = k.linear_wgrad(dy, x)
    assert dw.dtype == torch.float32
    assert rel(dw, dy.float().t() @ x.float()) < GTOL[dt]
    dw2, db = k.linear_wgrad(dy, x, bias_grad=True)
    assert rel(dw2, dy.float().t() @ x.float()) < GTOL[dt]
    assert rel(db, dy.float().sum(0)) < GTOL[dt]


@pytest.mark.parametrize("M,N,Kd", [(140000, 64, 64), (131072 + 77, 256, 128), (140001, 160, 64),
                                    (135000, 64, 512)])
def test_gemm_stream_large_m(M, N, Kd):
    """Large-M x short-K shapes take the persistent M-streaming kernel (bf16): forward with the
    full fused epilogue and dgrad with the GELU-derivative multiplier, incl. ragged M / N tails."""
    k = K()
    dt = torch.bfloat16
    x = torch.randn(M, Kd, device=DEV).to(dt)
    w = (torch.randn(N, Kd, device=DEV) / Kd ** 0.5).to(dt)
    b = torch.randn(N, device=DEV)
    res = torch.randn(M, N, device=DEV).to(dt)
    ls = torch.rand(N, device=DEV)
    pre = torch.empty(M, N, device=DEV, dtype=dt)
    y = k.linear(x, w, b, preact=pre, res=res, colscale=ls)
    f = x.float() @ w.float().t() + b
    assert rel(pre.float(), f) < GTOL[dt]
    assert rel(y.float(), res.float() + ls * f) < GTOL[dt]
    dy = torch.randn(M, N, device=DEV).to(dt)
    h = torch.randn(M, Kd, device=DEV).to(dt)
    dx = k.linear_dgrad(dy, w, gelu_grad_of=h)
    hf = h.float()
    gg = 0.5 * (1 + torch.erf(hf / math.sqrt(2))) + hf * torch.exp(-0.5 * hf * hf) / math.sqrt(2 * math.pi)
    assert rel(dx.float(), (dy.float() @ w.float()) * gg) < GTOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
def test_gemm_splitk_and_strided(dt):
    k = K()
    big = torch.randn(20000, 96, device=DEV).to(dt)
    x = big[:, 16:80]  # strided view, ld=96
    dy = torch.randn(20000, 48, device=DEV).to(dt)
    dw = k.linear_wgrad(dy, x)
    assert rel(dw, dy.float().t() @ x.float()) < GTOL[dt]
    acc = torch.randn(48, 64, device=DEV)
    ref = acc + dy.float().t() @ x.float()
    k.linear_wgrad(dy, x, out=acc, accumulate=True)
    assert rel(acc, ref) < GTOL[dt]


@pytest.mark.parametrize("M,N,Kd", [(1000, 128, 256), (777, 200, 1000), (4800, 512, 2048), (130, 40, 136),
                                    (19200, 256, 1024), (300, 64, 520)])
def test_gemm_lds_dma_paths(M, N, Kd):
    """bf16 k-loops of >= 2 whole 64-deep slices take the LDS-DMA ring kernel in all three layouts
    (forward, dgrad, wgrad with the fused bias-gradient column), incl. k tails, ragged M / N and
    split-K, with the full forward epilogue."""
    k = K()
    dt = torch.bfloat16
    x = torch.randn(M, Kd, device=DEV).to(dt)
    w = (torch.randn(N, Kd, device=DEV) / Kd ** 0.5).to(dt)
    b = torch.randn(N, device=DEV)
    res = torch.randn(M, N, device=DEV).to(dt)
    ls = torch.rand(N, device=DEV)
    pre = torch.empty(M, N, device=DEV, dtype=dt)
    y = k.linear(x, w, b, preact=pre, res=res, colscale=ls)
    f = x.float() @ w.float().t() + b
    assert rel(pre.float(), f) < GTOL[dt]
    assert rel(y.float(), res.float() + ls * f) < GTOL[dt]
    dy = torch.randn(M, Kd, device=DEV).to(dt)
    wd = (torch.randn(Kd, N, device=DEV) / Kd ** 0.5).to(dt)   # dx[M, N] = dy[M, Kd] @ wd[Kd, N]
    dx = k.linear_dgrad(dy, wd)
    assert rel(dx.float(), dy.float() @ wd.float()) < GTOL[dt]
    g = torch.randn(Kd, M, device=DEV).to(dt)     # wgrad over Kd "pixels": dW[M, N] = g^T x2
    x2 = torch.randn(Kd, N, device=DEV).to(dt)
    dw, db = k.linear_wgrad(g, x2, bias_grad=True)
    assert rel(dw, g.float().t() @ x2.float()) < GTOL[dt]
    assert rel(db, g.float().sum(0)) < GTOL[dt]
    dw2 = k.linear_wgrad(g, x2)
    assert torch.equal(dw2, dw)


@pytest.mark.parametrize("dt", DTYPES)
def test_gemm_epilogues(dt):
    k = K()
    M, N, Kd = 513, 96, 64
    x = torch.randn(M, Kd, device=DEV).to(dt)
    w = torch.randn(N, Kd, device=DEV).to(dt)
    b = torch.randn(N, device=DEV)
    pre = torch.empty(M, N, device=DEV, dtype=dt)
    y = k.linear(x, w, b, act=1, preact=pre)
    lin = x.float() @ w.float().t() + b
    assert rel(pre.float(), lin) < GTOL[dt]
    assert rel(y.float(), F.gelu(lin)) < GTOL[dt]
    mul = torch.randn(M, N, device=DEV).to(dt)
    res = torch.randn(M, N, device=DEV).to(dt)
    cs = torch.rand(N, device=DEV)
    rs = torch.rand(3, device=DEV)
    y = k.linear(x, w, b, mul=mul, res=res, colscale=cs, rowscale=rs, rows_per_scale=171)
    rsx = rs.repeat_interleave(171)[:M, None]
    assert rel(y.float(), res.float() + cs * rsx * (lin * mul.float())) < GTOL[dt]


@pytest.mark.parametrize("dt", [torch.float32])
def test_bmm_layouts(dt):
    k = K()
    a = torch.randn(3, 70, 40, device=DEV, dtype=dt)
    b = torch.randn(3, 40, 24, device=DEV, dtype=dt)
    assert rel(k.bmm(a, b), a @ b) < GTOL[dt]
    at = a.transpose(1, 2).contiguous()
    assert rel(k.bmm(at, b, a_t=True), a @ b) < GTOL[dt]
    bt = b.transpose(1, 2).contiguous()
    assert rel(k.bmm(a, bt, b_t=True), a @ b) < GTOL[dt]
    assert rel(k.bmm(at, bt, a_t=True, b_t=True), a @ b) < GTOL[dt]
    # odd N (not a multiple of the vector width): NMF at 530x730 (N = 67*92)
    x = torch.rand(2, 64, 6164, device=DEV)
    c = torch.rand(2, 6164, 32, device=DEV)
    assert rel(k.bmm(x, c), x @ c) < GTOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("C", [16, 32, 64, 96, 288, 576])
def test_layernorm(dt, C):
    k = K()
    x = (torch.randn(1037, C, device=DEV) * 2 + 0.5).to(dt)
    g = torch.rand(C, device=DEV) + 0.5
    b = torch.randn(C, device=DEV)
    y, mean, rstd = k.layernorm(x, g, b, 1e-6)
    xr = x.float().requires_grad_()
    gr, br = g.clone().requires_grad_(), b.clone().requires_grad_()
    ref = F.layer_norm(xr, (C,), gr, br, 1e-6)
    assert rel(y.float(), ref) < TOL[dt]
    dy = torch.randn(1037, C, device=DEV).to(dt)
    ref.backward(dy.float())
    dx, dg, db = k.layernorm_bwd(x, dy, g, mean, rstd)
    assert rel(dx.float(), xr.grad) < TOL[dt] * 2
    assert rel(dg, gr.grad) < TOL[dt] * 2
    assert rel(db, br.grad) < TOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("C", [32, 128, 512, 1024])
def test_layernorm_views_accumulate(dt, C):
    """Column-slice views (row stride > C), the fused residual-gradient add and accumulate=True."""
    k = K()
    rows = 777
    xb = (torch.randn(rows, C + 16, device=DEV) * 2 + 0.5).to(dt)
    x = xb[:, 8:8 + C]
    g = torch.rand(C, device=DEV) + 0.5
    b = torch.randn(C, device=DEV)
    yb = torch.zeros(rows, C + 8, device=DEV).to(dt)
    _, mean, rstd = k.layernorm(x, g, b, 1e-6, out=yb[:, 8:])
    xr = x.float().requires_grad_()
    ref = F.layer_norm(xr, (C,), g, b, 1e-6)
    assert rel(yb[:, 8:].float(), ref) < TOL[dt]
    dy = torch.randn(rows, C, device=DEV).to(dt)
    dres = torch.randn(rows, C, device=DEV).to(dt)
    base = torch.randn(rows, C + 8, device=DEV).to(dt)
    dx = base.clone()
    ref.backward(dy.float())
    k.layernorm_bwd(x, dy, g, mean, rstd, dx=dx[:, :C], accumulate=True, dres=dres)
    want = xr.grad + dres.float() + base[:, :C].float()
    assert rel(dx[:, :C].float(), want) < TOL[dt] * 2
    assert torch.equal(dx[:, C:], base[:, C:])


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("ks,ident", [(7, False), (3, True)])
# (1, 9, 10, 520) / (1, 33, 34, 520): channel vectors not a multiple of the 64-lane slice of the
# row-streaming kernels (partial last slice), the latter also on the streaming 3x3 forward's planes
# (planes below the 7-row window, whole 128-channel slices)
@pytest.mark.parametrize("B,H,W,C", [(2, 11, 13, 48), (1, 30, 40, 64), (2, 5, 7, 16), (1, 33, 41, 40),
                                     (1, 9, 10, 520), (1, 33, 34, 520), (2, 11, 13, 128), (1, 3, 2, 256),
                                     (2, 30, 40, 256), (1, 15, 20, 512), (1, 1, 1, 128)])
def test_dwconv(dt, ks, ident, B, H, W, C):
    k = K()
    x = torch.randn(B, H, W, C, device=DEV).to(dt)
    w = torch.randn(C, 1, ks, ks, device=DEV) / ks
    bias = torch.randn(C, device=DEV)
    xr = x.float().permute(0, 3, 1, 2).contiguous().requires_grad_()
    wr, br = w.clone().requires_grad_(), bias.clone().requires_grad_()
    ref = F.conv2d(xr, wr, br, padding=ks // 2, groups=C)
    if ident:
        ref = ref + xr
    y = k.dwconv(x.view(-1, C), (B, H, W), w, bias, ks, ident)
    assert rel(y.float().view(B, H, W, C).permute(0, 3, 1, 2), ref) < TOL[dt]
    dy = torch.randn(B, H, W, C, device=DEV).to(dt)
    ref.backward(dy.float().permute(0, 3, 1, 2))
    dx = k.dwconv_bwd_data(dy.view(-1, C), (B, H, W), w, ks, ident)
    assert rel(dx.float().view(B, H, W, C).permute(0, 3, 1, 2), xr.grad) < TOL[dt]
    dw, db = k.dwconv_bwd_weight(x.view(-1, C), dy.view(-1, C), (B, H, W), ks)
    assert rel(dw, wr.grad) < TOL[dt] * 2
    assert rel(db, br.grad) < TOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("flip", [False, True])
@pytest.mark.parametrize("B,H,W,C", [(2, 19, 37, 128), (1, 60, 80, 128), (3, 8, 5, 256), (2, 7, 7, 384)])
def test_dwconv7_strided_accumulate(dt, flip, B, H, W, C):
    """7x7 on column-slice views at 128-lane channel multiples: forward with and without bias, and the
    input gradient (flipped taps) accumulated into a strided destination."""
    k = K()
    g = torch.Generator(device=DEV).manual_seed(B * H * W + C + flip)
    xb = torch.randn(B * H * W, C + 16, device=DEV, generator=g).to(dt)
    x = xb[:, 8:8 + C]
    w = torch.randn(C, 1, 7, 7, device=DEV, generator=g) / 7
    bias = torch.randn(C, device=DEV, generator=g)
    xr = x.float().reshape(B, H, W, C).permute(0, 3, 1, 2)
    base = torch.randn(B * H * W, C + 8, device=DEV, generator=g).to(dt)
    out = base.clone()
    if flip:
        k.dwconv_bwd_data(x, (B, H, W), w, 7, False, dx=out[:, 8:], accumulate=True)
        ref = F.conv_transpose2d(xr, w, padding=3, groups=C) + base[:, 8:].float().reshape(B, H, W, C).permute(0, 3, 1, 2)
    else:
        k.dwconv(x, (B, H, W), w, None, 7, False, out=out[:, 8:])
        ref = F.conv2d(xr, w, None, padding=3, groups=C)
    assert rel(out[:, 8:].float().reshape(B, H, W, C).permute(0, 3, 1, 2), ref) < TOL[dt]
    assert torch.equal(out[:, :8], base[:, :8])
    if not flip:
        y = k.dwconv(x, (B, H, W), w, bias, 7, False)
        assert rel(y.float().reshape(B, H, W, C).permute(0, 3, 1, 2), F.conv2d(xr, w, bias, padding=3, groups=C)) < TOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("ks", [3, 7])
@pytest.mark.parametrize("B,H,W,C", [(2, 19, 37, 80), (1, 9, 70, 32), (3, 33, 5, 24), (2, 37, 29, 24)])
def test_dwconv_strided_gelu_accumulate(dt, ks, B, H, W, C):
    """Column-slice views (row stride > C), the fused GELU second output and accumulate=True."""
    k = K()
    xb = torch.randn(B * H * W, C + 16, device=DEV).to(dt)
    x = xb[:, 8:8 + C]
    w = torch.randn(C, 1, ks, ks, device=DEV) / ks
    bias = torch.randn(C, device=DEV)
    xr = x.float().reshape(B, H, W, C).permute(0, 3, 1, 2)
    ref = F.conv2d(xr, w, bias, padding=ks // 2, groups=C) + xr
    yb = torch.zeros(B * H * W, C + 8, device=DEV).to(dt)
    gb = torch.zeros(B * H * W, C + 24, device=DEV).to(dt)
    k.dwconv(x, (B, H, W), w, bias, ks, True, out=yb[:, :C], gelu_out=gb[:, 16:16 + C])
    y = yb[:, :C].float().reshape(B, H, W, C).permute(0, 3, 1, 2)
    assert rel(y, ref) < TOL[dt]
    g = gb[:, 16:16 + C].float().reshape(B, H, W, C).permute(0, 3, 1, 2)
    assert rel(g, F.gelu(y)) < TOL[dt]
    dy = torch.randn(B * H * W, C, device=DEV).to(dt)
    base = torch.randn(B * H * W, C, device=DEV).to(dt)
    dx = base.clone()
    k.dwconv_bwd_data(dy, (B, H, W), w, ks, False, dx=dx, accumulate=True)
    dyr = dy.float().reshape(B, H, W, C).permute(0, 3, 1, 2)
    refdx = F.conv_transpose2d(dyr, w, padding=ks // 2, groups=C) + base.float().reshape(B, H, W, C).permute(0, 3, 1, 2)
    assert rel(dx.float().reshape(B, H, W, C).permute(0, 3, 1, 2), refdx) < TOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("ident,acc", [(True, False), (False, True)])
# planes of every stage geometry incl. odd sizes, partial 64-lane channel slices (520) and strided views
# (C % 128 == 0 or C >= 384: the row-scatter kernel, one channel pair per lane; otherwise the 8-byte-lane
# gather kernel)
@pytest.mark.parametrize("B,H,W,C", [(2, 11, 13, 48), (1, 30, 40, 64), (2, 5, 7, 16), (1, 33, 41, 40),
                                     (1, 9, 10, 520), (2, 120, 160, 32), (3, 15, 20, 256), (2, 30, 40, 128),
                                     (1, 23, 37, 256), (2, 7, 5, 384), (1, 2, 3, 128), (1, 60, 80, 512),
                                     (2, 34, 46, 576), (1, 5, 6, 392)])
def test_dwconv_fused_bwd(dt, ident, acc, B, H, W, C):
    """dfm_dwconv_bwd (3x3 input + weight gradient in one pass) vs torch fp32, and vs the separate
    kernels: the weight / bias gradients bit for bit where both use the same partial geometry and
    summation order (the 8-byte-lane kernel), to fp32 summation order otherwise (the row-scatter one)."""
    k = K()
    xb = torch.randn(B * H * W, C + 8, device=DEV).to(dt)
    x = xb[:, :C]
    w = torch.randn(C, 1, 3, 3, device=DEV) / 3
    xr = x.float().reshape(B, H, W, C).permute(0, 3, 1, 2).contiguous().requires_grad_()
    wr, br = w.clone().requires_grad_(), torch.zeros(C, device=DEV, requires_grad=True)
    ref = F.conv2d(xr, wr, br, padding=1, groups=C)
    if ident:
        ref = ref + xr
    dyb = torch.randn(B * H * W, C + 16, device=DEV).to(dt)
    dy = dyb[:, 16:]
    ref.backward(dy.float().reshape(B, H, W, C).permute(0, 3, 1, 2))
    base = torch.randn(B * H * W, C, device=DEV).to(dt)
    dx = base.clone() if acc else None
    dx, dw, db = k.dwconv_bwd(x, dy, (B, H, W), w, 3, add_identity=ident, dx=dx, accumulate=acc)
    want = xr.grad + (base.float().reshape(B, H, W, C).permute(0, 3, 1, 2) if acc else 0)
    assert rel(dx.float().reshape(B, H, W, C).permute(0, 3, 1, 2), want) < TOL[dt]
    assert rel(dw, wr.grad) < TOL[dt] * 2
    assert rel(db, br.grad) < TOL[dt]
    dw2, db2 = k.dwconv_bwd_weight(x, dy, (B, H, W), 3)
    if C % 128 and C < 384:  # the gather kernel: the separate kernel's partial geometry and order
        assert torch.equal(dw, dw2) and torch.equal(db, db2)
    else:  # the row-scatter kernel (520: a partial last 64-lane slice)
        assert rel(dw, dw2) < 1e-5 and rel(db, db2) < 1e-5


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("acc", [False, True])
# every DFormer-B stage geometry (C and C/2), tile-ragged planes, a partial channel slab (C = 40: 5 bf16 /
# 10 fp32 vectors) and strided views
@pytest.mark.parametrize("B,H,W,C", [(1, 120, 160, 64), (2, 60, 80, 128), (2, 30, 40, 256), (3, 15, 20, 512),
                                     (2, 11, 13, 48), (1, 17, 23, 40), (2, 5, 7, 32)])
def test_dwconv7_fused_bwd(dt, acc, B, H, W, C):
    """dfm_dwconv_bwd with k = 7 (one pass over dy: input gradient + weight / bias gradient) vs torch fp32,
    and vs the separate kernels: the weight / bias gradients bit for bit (same tiles, lanes and order)."""
    k = K()
    g = torch.Generator(device=DEV).manual_seed(B * H * W + C)
    xb = torch.randn(B * H * W, C + 8, device=DEV, generator=g).to(dt)
    x = xb[:, 8:]
    w = torch.randn(C, 1, 7, 7, device=DEV, generator=g) / 7
    xr = x.float().reshape(B, H, W, C).permute(0, 3, 1, 2).contiguous().requires_grad_()
    wr, br = w.clone().requires_grad_(), torch.zeros(C, device=DEV, requires_grad=True)
    ref = F.conv2d(xr, wr, br, padding=3, groups=C)
    dyb = torch.randn(B * H * W, C + 16, device=DEV, generator=g).to(dt)
    dy = dyb[:, 16:]
    ref.backward(dy.float().reshape(B, H, W, C).permute(0, 3, 1, 2))
    base = torch.randn(B * H * W, C, device=DEV, generator=g).to(dt)
    dx = base.clone() if acc else None
    dx, dw, db = k.dwconv_bwd(x, dy, (B, H, W), w, 7, dx=dx, accumulate=acc)
    want = xr.grad + (base.float().reshape(B, H, W, C).permute(0, 3, 1, 2) if acc else 0)
    assert rel(dx.float().reshape(B, H, W, C).permute(0, 3, 1, 2), want) < TOL[dt]
    assert rel(dw, wr.grad) < TOL[dt] * 2
    assert rel(db, br.grad) < TOL[dt]
    dw2, db2 = k.dwconv_bwd_weight(x, dy, (B, H, W), 7)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)
    dx2 = k.dwconv_bwd_data(dy, (B, H, W), w, 7, dx=base.clone() if acc else None, accumulate=acc)
    assert rel(dx.float(), dx2.float()) <= {torch.float32: 1e-6, torch.bfloat16: 2.0 ** -7, torch.float16: 2.0 ** -10}[dt]


@pytest.mark.parametrize("dt", DTYPES)
# degenerate planes for the streaming 3x3 kernels' clamped-address loads (out-of-image taps read the
# unit's own first row / column and are zeroed at first use): one pixel, one row, one column, widths
# below the 4-column strip, a partial last strip and row chunk
@pytest.mark.parametrize("B,H,W,C", [(1, 1, 1, 8), (2, 1, 5, 16), (1, 3, 2, 24), (2, 9, 1, 8), (1, 2, 9, 48),
                                     (3, 6, 6, 32), (1, 1, 1, 128), (2, 1, 5, 128), (2, 9, 1, 256), (1, 4, 3, 128)])
def test_dwconv3_stream_edges(dt, B, H, W, C):
    k = K()
    x = torch.randn(B * H * W, C, device=DEV).to(dt)
    w = torch.randn(C, 1, 3, 3, device=DEV) / 3
    bias = torch.randn(C, device=DEV)
    xr = x.float().view(B, H, W, C).permute(0, 3, 1, 2).contiguous().requires_grad_()
    wr, br = w.clone().requires_grad_(), bias.clone().requires_grad_()
    ref = F.conv2d(xr, wr, br, padding=1, groups=C) + xr
    y = k.dwconv(x, (B, H, W), w, bias, 3, True)
    assert rel(y.float().view(B, H, W, C).permute(0, 3, 1, 2), ref) < TOL[dt]
    dy = torch.randn(B * H * W, C, device=DEV).to(dt)
    ref.backward(dy.float().view(B, H, W, C).permute(0, 3, 1, 2))
    dx, dw, db = k.dwconv_bwd(x, dy, (B, H, W), w, 3, add_identity=True)
    assert rel(dx.float().view(B, H, W, C).permute(0, 3, 1, 2), xr.grad) < TOL[dt]
    assert rel(dw, wr.grad) < TOL[dt] * 2
    assert rel(db, br.grad) < TOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("B,H,W,C", [(2, 19, 37, 80), (2, 120, 160, 32), (1, 30, 40, 64)])
def test_dwconv_gelu_grad_out(dt, B, H, W, C):
    """Flag 2: y receives GELU'(pre) while gelu_out receives GELU(pre) (tile and streaming kernels)."""
    k = K()
    x = torch.randn(B * H * W, C, device=DEV).to(dt)
    w = torch.randn(C, 1, 3, 3, device=DEV) / 3
    bias = torch.randn(C, device=DEV)
    pre = k.dwconv(x, (B, H, W), w, bias, 3, True)
    g1 = torch.empty_like(x)
    g2 = torch.empty_like(x)
    gp = k.dwconv(x, (B, H, W), w, bias, 3, True, gelu_out=g1, out_gelu_grad=True)
    k.dwconv(x, (B, H, W), w, bias, 3, True, gelu_out=g2)
    assert torch.equal(g1, g2)
    p = pre.float().requires_grad_()
    F.gelu(p).sum().backward()
    assert rel(gp.float(), p.grad) < TOL[dt] * 2


@pytest.mark.parametrize("dt", DTYPES)
def test_gemm_act3_gelu_grad_preact(dt):
    """GEMM act 3: GELU on the columns from act_col0 (as act 1) and preact = GELU'(pre-activation)."""
    k = K()
    M, N, Kd, c0 = 700, 96, 64, 40
    x = torch.randn(M, Kd, device=DEV).to(dt)
    w = torch.randn(N, Kd, device=DEV).to(dt) / 8
    b = torch.randn(N, device=DEV)
    pre1 = torch.empty(M, N - c0, device=DEV, dtype=dt)
    pre3 = torch.empty(M, N - c0, device=DEV, dtype=dt)
    y1 = k.linear(x, w, b, act=1, preact=pre1, act_col0=c0)
    y3 = k.linear(x, w, b, act=3, preact=pre3, act_col0=c0)
    # the same GELU; contraction may differ in the last bit of the output: one ulp at the maximum
    ulp = {torch.float32: 1e-6, torch.bfloat16: 2.0 ** -7, torch.float16: 2.0 ** -10}[dt]
    assert rel(y3.float(), y1.float()) <= ulp
    p = pre1.float().requires_grad_()
    F.gelu(p).sum().backward()
    assert rel(pre3.float(), p.grad) < GTOL[dt] * 2


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("H,W", [(15, 20), (8, 10), (5, 7), (60, 80), (17, 23)])
def test_pool7(dt, H, W):
    k = K()
    B, C = 2, 40
    x = torch.randn(B, H, W, C, device=DEV).to(dt)
    xr = x.float().permute(0, 3, 1, 2).contiguous().requires_grad_()
    ref = F.adaptive_avg_pool2d(xr, 7)
    y = k.pool7(x.view(-1, C), (B, H, W))
    assert rel(y.float().view(B, 7, 7, C).permute(0, 3, 1, 2), ref) < TOL[dt]
    dy = torch.randn(B, 7, 7, C, device=DEV).to(dt)
    ref.backward(dy.float().permute(0, 3, 1, 2))
    dx = k.pool7_bwd(dy.view(-1, C), (B, H, W))
    assert rel(dx.float().view(B, H, W, C).permute(0, 3, 1, 2), xr.grad) < TOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("hi,ho", [((7, 7), (15, 20)), ((7, 7), (5, 7)), ((30, 40), (60, 80)), ((15, 20), (60, 80)),
                                   ((60, 80), (480, 640)), ((34, 46), (133, 183))])
def test_bilinear(dt, hi, ho):
    k = K()
    B, C = 2, 24
    x = torch.randn(B, *hi, C, device=DEV).to(dt)
    xr = x.float().permute(0, 3, 1, 2).contiguous().requires_grad_()
    ref = F.interpolate(xr, ho, mode="bilinear", align_corners=False)
    y = k.bilinear(x.view(-1, C), hi, ho, B)
    assert rel(y.float().view(B, *ho, C).permute(0, 3, 1, 2), ref) < TOL[dt]
    dy = torch.randn(B, *ho, C, device=DEV).to(dt)
    ref.backward(dy.float().permute(0, 3, 1, 2))
    dx = k.bilinear_bwd(dy.view(-1, C), hi, ho, B)
    assert rel(dx.float().view(B, *hi, C).permute(0, 3, 1, 2), xr.grad) < TOL[dt] * 2


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("hi,ho,C", [((12, 16), (24, 32), 64), ((6, 8), (24, 32), 128), ((7, 7), (60, 80), 64),
                                     ((30, 40), (60, 80), 512)])
def test_bilinear_strided(dt, hi, ho, C):
    """Column-slice views on both sides (the decoders' resize+concat and its backward)."""
    k = K()
    B = 2
    xb = torch.randn(B * hi[0] * hi[1], C + 24, device=DEV).to(dt)
    x = xb[:, 16:16 + C]
    yb = torch.zeros(B * ho[0] * ho[1], C + 40, device=DEV).to(dt)
    k.bilinear(x, hi, ho, B, out=yb[:, 32:32 + C])
    xr = x.float().reshape(B, *hi, C).permute(0, 3, 1, 2).contiguous().requires_grad_()
    ref = F.interpolate(xr, ho, mode="bilinear", align_corners=False)
    assert rel(yb[:, 32:32 + C].float().view(B, *ho, C).permute(0, 3, 1, 2), ref) < TOL[dt]
    dyb = torch.randn(B * ho[0] * ho[1], C + 8, device=DEV).to(dt)
    dy = dyb[:, 8:]
    ref.backward(dy.float().reshape(B, *ho, C).permute(0, 3, 1, 2))
    dx = k.bilinear_bwd(dy, hi, ho, B)
    assert rel(dx.float().view(B, *hi, C).permute(0, 3, 1, 2), xr.grad) < TOL[dt] * 2


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("B,heads,N,dh",[(2, 2, 300, 32), (1, 4, 1200, 32), (2, 1, 37, 16), (1, 2, 150, 48),
                                         (2, 4, 99, 36), (2, 4, 1564, 36), (2, 8, 391, 36)])
def test_pooled_attention(dt, B, heads, N, dh):
    """MFMA pooled attention (bf16 / fp16; fp32 on the scalar kernels) vs torch fp32 on the same rounded
    inputs. The kernel's own error sources are P and dS rounded to the 16-bit MFMA operand type and the
    16-bit outputs (bf16: 2^-9 relative, i.e. ~1.1e-3 in norm from the output rounding alone), so the
    gates sit a few roundings above that instead of at the generic elementwise tolerance."""
    tol = {torch.float32: 2e-5, torch.bfloat16: 6e-3, torch.float16: 1.5e-3}[dt]
    k = K()
    C2 = heads * dh
    q = torch.randn(B * 49, C2, device=DEV).to(dt)
    kv = torch.randn(B * N, 2 * C2, device=DEV).to(dt)
    scale = dh ** -0.5
    o, lse = k.pooled_attn(q, kv[:, :C2], kv[:, C2:], B, heads, N, dh, scale)
    qr = q.float().view(B, 49, heads, dh).permute(0, 2, 1, 3).requires_grad_()
    kr = kv.float()[:, :C2].reshape(B, N, heads, dh).permute(0, 2, 1, 3).contiguous().requires_grad_()
    vr = kv.float()[:, C2:].reshape(B, N, heads, dh).permute(0, 2, 1, 3).contiguous().requires_grad_()
    ref = ((qr * scale) @ kr.transpose(-2, -1)).softmax(-1) @ vr
    assert rel(o.float().view(B, 49, heads, dh).permute(0, 2, 1, 3), ref) < tol
    do = torch.randn(B * 49, C2, device=DEV).to(dt)
    ref.backward(do.float().view(B, 49, heads, dh).permute(0, 2, 1, 3))
    dq = torch.empty_like(q)
    dkv = torch.empty_like(kv)
    k.pooled_attn_bwd(q, kv[:, :C2], kv[:, C2:], o, do, lse, B, heads, N, dh, scale, dq, dkv[:, :C2], dkv[:, C2:])
    assert rel(dq.float().view(B, 49, heads, dh).permute(0, 2, 1, 3), qr.grad) < tol * 2
    assert rel(dkv[:, :C2].float().reshape(B, N, heads, dh).permute(0, 2, 1, 3), kr.grad) < tol * 2
    assert rel(dkv[:, C2:].float().reshape(B, N, heads, dh).permute(0, 2, 1, 3), vr.grad) < tol * 2


@pytest.mark.parametrize("dt", DTYPES)
def test_colsum_and_elementwise(dt):
    k = K()
    x = torch.randn(5000, 72, device=DEV).to(dt)
    m = torch.randn(5000, 72, device=DEV).to(dt)
    rs = torch.rand(4, device=DEV)
    s = k.colsum(x, mul=m, rowscale=rs, rows_per_scale=1250)
    ref = (x.float() * m.float() * rs.repeat_interleave(1250)[:, None]).sum(0)
    assert rel(s, ref) < TOL[dt]
    pre = torch.randn(5000, 72, device=DEV).to(dt)
    g = k.gelu_bwd(x, pre)
    pr = pre.float().requires_grad_()
    F.gelu(pr).backward(x.float())
    assert rel(g.float(), pr.grad) < TOL[dt]
    cs = torch.rand(72, device=DEV)
    y = k.scale_mul(x, mul=m, colscale=cs)
    assert rel(y.float(), x.float() * m.float() * cs) < TOL[dt]
    # strided views + accumulate (vector path) and an odd width (scalar path)
    acc = torch.randn(5000, 80, device=DEV).to(dt)
    want = acc[:, 8:].float() + x.float() * m.float() * cs * rs.repeat_interleave(1250)[:, None]
    k.scale_mul(x, mul=m, colscale=cs, rowscale=rs, rows_per_scale=1250, out=acc[:, 8:], accumulate=True)
    assert rel(acc[:, 8:].float(), want) < TOL[dt]
    xo, po = x[:, :71], pre.detach()[:, :71]
    pr2 = po.detach().float().clone().requires_grad_()
    F.gelu(pr2).backward(xo.float())
    assert rel(k.gelu_bwd(xo, po).float(), pr2.grad) < TOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
def test_batchnorm(dt):
    k = K()
    x = (torch.randn(3000, 64, device=DEV) * 3 + 1).to(dt)
    g = torch.rand(64, device=DEV) + 0.5
    b = torch.randn(64, device=DEV)
    rm, rv = torch.zeros(64, device=DEV), torch.ones(64, device=DEV)
    st = k.bn_stats(x)
    mean, rstd = k.bn_finalize(st, 3000, 1e-3, 0.1, rm, rv)
    y = k.bn_apply(x, mean, rstd, g, b, act=2)
    xr = x.float().requires_grad_()
    gr, br = g.clone().requires_grad_(), b.clone().requires_grad_()
    rm2, rv2 = torch.zeros(64, device=DEV), torch.ones(64, device=DEV)
    ref = F.relu(F.batch_norm(xr, rm2, rv2, gr, br, True, 0.1, 1e-3))
    assert rel(y.float(), ref) < TOL[dt]
    assert rel(rm, rm2) < 1e-4 and rel(rv, rv2) < 1e-4
    dy = torch.randn(3000, 64, device=DEV).to(dt)
    ref.backward(dy.float())
    dyr = k.relu_bwd(dy, y)
    st2 = k.bn_bwd_stats(x, dyr, mean, rstd)
    dx = k.bn_bwd_apply(x, dyr, mean, rstd, g, st2, 3000)
    assert rel(dx.float(), xr.grad) < TOL[dt] * 2
    assert rel(st2[1] , gr.grad) < TOL[dt] * 2
    assert rel(st2[0], br.grad) < TOL[dt] * 2


@pytest.mark.parametrize("C", [16, 32, 512])
def test_batchnorm_shifted_stats_large_offset(C):
    """|mean| >> std over ~1M rows (the cancellation regime of one-pass E[x^2]-E[x]^2): the
    shifted statistics must still give torch's fp32 batch_norm mean / variance / output."""
    k = K()
    rows = (1 << 20) if C <= 32 else (1 << 17)
    mu = torch.linspace(-300, 300, C, device=DEV)
    x = torch.randn(rows, C, device=DEV) * 0.5 + mu
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    mean, rstd = k.bn_finalize(k.bn_stats(x), rows, 1e-5, 0.1, rm, rv)
    xd = x.double()
    assert rel(mean, xd.mean(0)) < 1e-6
    assert rel(1.0 / rstd.double() ** 2 - 1e-5, xd.var(0, unbiased=False)) < 1e-3
    g, b = torch.ones(C, device=DEV), torch.zeros(C, device=DEV)
    y = k.bn_apply(x, mean, rstd, g, b)
    ref = (xd - xd.mean(0)) / torch.sqrt(xd.var(0, unbiased=False) + 1e-5)
    assert rel(y.double(), ref) < 1e-3


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("rows", [1, 63, 64, 65, 192, 193, 255, 256, 257, 511, 4801, 76801, 131073, 300001])
def test_column_reductions_block_tails(dt, rows):
    """colsum (with multiplier and per-image row scale), BN statistics and BN backward statistics at row
    counts that split into several blocks with partial tails (any block count / rows-per-block geometry the
    build was compiled with, dfm_build_tag), on a strided view: each against float64 on the same
    operands, bounded by the fp32 summation error relative to sum|terms| (conditioning-free)."""
    k = K()
    g = torch.Generator(device=DEV).manual_seed(rows)
    for C in (16, 20, 48, 72, 512):
        base = (torch.randn(rows, C + 8, device=DEV, generator=g) * 3 + 1).to(dt)
        x = base[:, 8:]  # a strided view; C = 20 takes the scalar kernel (16-bit), the others the vector one
        y = torch.randn(rows, C, device=DEV, generator=g).to(dt)
        rps = max(1, rows // 3)
        rs = torch.rand((rows + rps - 1) // rps, device=DEV, generator=g)
        xd, yd = x.double(), y.double()
        bound = 1e-6 * max(1.0, math.sqrt(rows))

        def chk(got, terms):
            err = ((got.double() - terms.sum(0)).abs() / terms.abs().sum(0).clamp_min(1e-30)).max().item()
            assert err < bound, (C, err, bound)

        chk(k.colsum(x, mul=y, rowscale=rs, rows_per_scale=rps), xd * yd * rs.double().repeat_interleave(rps)[:rows, None])
        st = k.bn_stats(x)
        sh = xd - xd[0]
        chk(st[0], sh)
        chk(st[1], sh * sh)
        assert torch.equal(st[2], x[0].float())
        mean = torch.randn(C, device=DEV, generator=g)
        rstd = torch.rand(C, device=DEV, generator=g) + 0.5
        s2 = k.bn_bwd_stats(x, y, mean, rstd)
        chk(s2[0], yd)
        chk(s2[1], yd * (xd - mean.double()) * rstd.double())


def test_nmf_update_softmax():
    k = K()
    a, num, den = (torch.rand(4, 100, 64, device=DEV) for _ in range(3))
    out = k.nmf_update(a, num, den)
    assert rel(out, a * num / (den + 1e-6)) < 1e-6
    ar, nr, dr = (t.clone().requires_grad_() for t in (a, num, den))
    o2 = ar * nr / (dr + 1e-6)
    g = torch.randn_like(o2)
    o2.backward(g)
    ga, gn, gd = k.nmf_update_bwd(g, a, num, den, out)
    assert rel(ga, ar.grad) < 1e-5 and rel(gn, nr.grad) < 1e-5 and rel(gd, dr.grad) < 1e-5
    x = torch.randn(500, 64, device=DEV)
    y = k.softmax_rows(x)
    assert rel(y, x.softmax(-1)) < 1e-5
    xr = x.clone().requires_grad_()
    gy = torch.randn(500, 64, device=DEV)
    xr.softmax(-1).backward(gy)
    assert rel(k.softmax_rows_bwd(y, gy), xr.grad) < 1e-5


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("B,h,w,H,W,ncls", [(2, 60, 80, 480, 640, 40), (1, 17, 23, 67, 92, 37), (2, 8, 12, 64, 96, 40), (1, 30, 40, 37, 50, 19), (1, 13, 11, 100, 90, 16),
                                                (1, 24, 20, 96, 80, 40), (2, 10, 14, 20, 28, 64), (1, 7, 9, 56, 72, 3),
                                                (1, 133, 183, 530, 730, 40), (1, 5, 4, 300, 290, 8),
                                                (2, 133, 183, 530, 730, 37)])
def test_seg_loss(dt, B, h, w, H, W, ncls):
    k = K()
    lg = torch.randn(B, h, w, ncls, device=DEV).to(dt)
    lab = torch.randint(0, ncls, (B, H, W), device=DEV)
    lab[torch.rand(B, H, W, device=DEV) < 0.1] = 255
    out = k.seg_loss_fwd(lg.view(-1, ncls), B, h, w, ncls, lab)
    lr = lg.float().permute(0, 3, 1, 2).contiguous().requires_grad_()
    up = F.interpolate(lr, (H, W), mode="bilinear", align_corners=False)
    ce = F.cross_entropy(up, lab, reduction="none", ignore_index=255)
    loss = ce[lab != 255].mean()
    assert abs((out[0] / out[1]).item() - loss.item()) < 1e-4 * abs(loss.item())
    loss.backward()
    dl = k.seg_loss_bwd(lg.view(-1, ncls), B, h, w, ncls, lab, out)
    assert rel(dl.view(B, h, w, ncls).permute(0, 3, 1, 2), lr.grad) < 1e-3


@pytest.mark.parametrize("B,h,w,H,W", [(2, 15, 20, 120, 160), (2, 30, 40, 120, 160), (2, 60, 80, 120, 160),
                                       (2, 133, 183, 530, 730), (1, 30, 40, 37, 50), (1, 9, 11, 100, 90)])
def test_seg_loss_bwd_deterministic(B, h, w, H, W):
    """every upsampling factor is bitwise reproducible run to run: integer factors (tile partials)
    and config 5's 133x183 -> 530x730 (separable x-pass / y-pass), builder.py:203,230"""
    k = K()
    ncls = 40
    lg = torch.randn(B, h, w, ncls, device=DEV).to(torch.bfloat16)
    lab = torch.randint(0, ncls, (B, H, W), device=DEV)
    lab[:, :5] = 255
    out = k.seg_loss_fwd(lg.view(-1, ncls), B, h, w, ncls, lab)
    d1 = k.seg_loss_bwd(lg.view(-1, ncls), B, h, w, ncls, lab, out)
    d2 = k.seg_loss_bwd(lg.view(-1, ncls), B, h, w, ncls, lab, out)
    assert torch.equal(d1, d2)


def test_adamw_matches_torch():
    k = K()
    p = torch.randn(10000, device=DEV)
    g = torch.randn(10000, device=DEV)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    pr = p.clone().requires_grad_()
    opt = torch.optim.AdamW([pr], lr=6e-5, betas=(0.9, 0.999), weight_decay=0.01)
    copy = torch.empty(10000, device=DEV, dtype=torch.bfloat16)
    for step in range(1, 4):
        pr.grad = g * step
        opt.step()
        k.adamw(p, g * step, m, v, 6e-5, 0.9, 0.999, 1e-8, 0.01, step, 1.0, copy)
    assert rel(p, pr.detach()) < 1e-6
    assert rel(copy.float(), p) < 1e-2


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("C", [32, 64, 256, 576])
def test_residual_bwd_and_ln_dres(dt, C):
    k = K()
    rows, B = 4000, 4
    dout = torch.randn(rows, C, device=DEV).to(dt)
    f = torch.randn(rows, C, device=DEV).to(dt)
    ls = torch.rand(C, device=DEV)
    rs = torch.rand(B, device=DEV)
    df, dls = k.residual_bwd(dout, f, ls, rs, rows // B)
    rsx = rs.repeat_interleave(rows // B)[:, None]
    assert rel(df.float(), dout.float() * ls * rsx) < TOL[dt]
    assert rel(dls, (dout.float() * f.float() * rsx).sum(0)) < TOL[dt]
    x = torch.randn(rows, C, device=DEV).to(dt)
    g, b = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    _, mean, rstd = k.layernorm(x, g, b)
    dx_a, _, _ = k.layernorm_bwd(x, f, g, mean, rstd, dres=dout)
    dx_b, _, _ = k.layernorm_bwd(x, f, g, mean, rstd)
    assert rel(dx_a.float(), dx_b.float() + dout.float()) < TOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
def test_dgrad_gelu_grad_epilogue(dt):
    k = K()
    dy = torch.randn(3000, 64, device=DEV).to(dt)
    w = torch.randn(64, 512, device=DEV).to(dt)
    pre = torch.randn(3000, 512, device=DEV).to(dt)
    out = k.linear_dgrad(dy, w, gelu_grad_of=pre)
    pr = pre.float().requires_grad_()
    torch.nn.functional.gelu(pr).backward(dy.float() @ w.float())
    assert rel(out.float(), pr.grad) < TOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("C", [64, 96, 36])
def test_dual_mul(dt, C):
    """(src*m1, src*m2) in one pass, on column slices of wider buffers (vector path) and C % 8 != 0."""
    k = K()
    rows = 1000
    buf = torch.randn(rows, 3 * C + 8, device=DEV).to(dt)
    src, m1, m2 = buf[:, :C], buf[:, C:2 * C], buf[:, 2 * C:3 * C]
    outb = torch.empty(rows, 2 * C + 8, device=DEV, dtype=dt)
    o1, o2 = k.dual_mul(src, m1, m2, out1=outb[:, :C], out2=outb[:, C + 8:2 * C + 8])
    assert rel(o1.float(), src.float() * m1.float()) < TOL[dt]
    assert rel(o2.float(), src.float() * m2.float()) < TOL[dt]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("fwd", [True, False])
def test_gemm_group_kcontig_mixed_members(dt, fwd):
    """dfm_gemm_group over k-contiguous-A problems (a Block phase's grouped forward / input-gradient
    launch): the ring-kernel members (aligned, K >= 128) run as ONE gemm_glds_group_kernel launch, the
    rest (K < 128, a misaligned A view, a bias-gradient column) on their single-GEMM route. Ragged M,
    N % 64 != 0 and the Block's epilogues (act 3 from act_col0 with GELU' saved, mul + preact, residual +
    colscale + rowscale, beta = 1; for input gradients the GELU'-multiplier and accumulate), each against
    torch fp32 and against the same problem launched alone."""
    k = K()
    M = 1999
    g = torch.Generator(device=DEV).manual_seed(7 + int(fwd))

    def rn(*s, scale=1.0):
        return (torch.randn(*s, device=DEV, generator=g) * scale).to(dt)

    probs = []  # (thunk(collect, out_dict) -> None, reference dict)
    if fwd:
        def p_act3(c, o):
            x, w, b = P["x1"], P["w1"], P["b1"]
            o["y"] = torch.empty(M, 200, device=DEV, dtype=dt)
            o["pre"] = torch.empty(M, 64, device=DEV, dtype=dt)
            k.linear(x, w, b, act=3, preact=o["pre"], act_col0=136, out=o["y"], collect=c)

        def r_act3():
            lin = P["x1"].float() @ P["w1"].float().t() + P["b1"]
            p = lin[:, 136:].clone().requires_grad_()
            F.gelu(p).sum().backward()
            return {"y": torch.cat([lin[:, :136], F.gelu(lin[:, 136:])], 1), "pre": p.grad}

        def p_mul(c, o):
            o["y"] = torch.empty(M, 136, device=DEV, dtype=dt)
            o["pre"] = torch.empty(M, 136, device=DEV, dtype=dt)
            k.linear(P["x2"], P["w2"], P["b2"], mul=P["m2"], preact=o["pre"], out=o["y"], collect=c)

        def r_mul():
            lin = P["x2"].float() @ P["w2"].float().t() + P["b2"]
            return {"y": lin * P["m2"].float(), "pre": lin}

        def p_res(c, o):
            o["y"] = torch.empty(M, 96, device=DEV, dtype=dt)
            k.linear(P["x3"], P["w3"], P["b3"], res=P["r3"], colscale=P["ls"], rowscale=P["rs"], rows_per_scale=700,
                     out=o["y"], collect=c)

        def r_res():
            lin = P["x3"].float() @ P["w3"].float().t() + P["b3"]
            return {"y": P["r3"].float() + P["ls"] * P["rs"].repeat_interleave(700)[:M, None] * lin}

        def p_short(c, o):  # K = 64 < 128: not a ring member
            o["y"] = torch.empty(M, 72, device=DEV, dtype=dt)
            k.linear(P["x4"], P["w4"], P["b4"], out=o["y"], collect=c)

        def r_short():
            return {"y": P["x4"].float() @ P["w4"].float().t() + P["b4"]}

        def p_misal(c, o):  # an A view 2 bytes off 16-byte alignment: not a ring member
            o["y"] = torch.empty(M, 80, device=DEV, dtype=dt)
            k.linear(P["x5"][:, 1:193], P["w5"], None, out=o["y"], collect=c)

        def r_misal():
            return {"y": P["x5"][:, 1:193].float() @ P["w5"].float().t()}

        def p_beta(c, o):  # beta = 1 onto a pre-filled output
            o["y"] = P["y6"].clone()
            k.linear(P["x6"], P["w6"], P["b6"], out=o["y"], beta=1.0, collect=c)

        def r_beta():
            return {"y": P["y6"].float() + P["x6"].float() @ P["w6"].float().t() + P["b6"]}

        def p_colsum(c, o):  # bias-gradient column (sum over k of each A row): not a ring member
            o["y"] = torch.empty(M, 88, device=DEV, dtype=dt)
            o["cs"] = torch.empty(M, device=DEV, dtype=torch.float32)
            x, w = P["x7"], P["w7"]
            k.gemm(x, w, M=M, N=88, K=256, a_kcontig=True, b_kcontig=True, lda=k.ld(x), ldb=k.ld(w), out=o["y"],
                   ldc=88, colsum=o["cs"], collect=c)

        def r_colsum():
            return {"y": P["x7"].float() @ P["w7"].float().t(), "cs": P["x7"].float().sum(1)}

        P = dict(x1=rn(M, 256), w1=rn(200, 256, scale=0.06), b1=torch.randn(200, device=DEV, generator=g),
                 x2=rn(M, 192), w2=rn(136, 192, scale=0.07), b2=torch.randn(136, device=DEV, generator=g),
                 m2=rn(M, 136), x3=rn(M, 320), w3=rn(96, 320, scale=0.05), b3=torch.randn(96, device=DEV, generator=g),
                 r3=rn(M, 96), ls=torch.rand(96, device=DEV, generator=g), rs=torch.rand(3, device=DEV, generator=g),
                 x4=rn(M, 64), w4=rn(72, 64, scale=0.1), b4=torch.randn(72, device=DEV, generator=g),
                 x5=rn(M, 200), w5=rn(80, 192, scale=0.07), x6=rn(M, 128), w6=rn(104, 128, scale=0.08),
                 b6=torch.randn(104, device=DEV, generator=g), y6=rn(M, 104), x7=rn(M, 256), w7=rn(88, 256, scale=0.06))
        probs = [(p_act3, r_act3), (p_mul, r_mul), (p_res, r_res), (p_short, r_short), (p_misal, r_misal),
                 (p_beta, r_beta), (p_colsum, r_colsum)]
    else:
        def p_plain(c, o):
            o["y"] = torch.empty(M, 200, device=DEV, dtype=dt)
            k.linear_dgrad(P["d1"], P["w1"], out=o["y"], collect=c)

        def r_plain():
            return {"y": P["d1"].float() @ P["w1"].float()}

        def p_gg(c, o):  # times GELU'(h)
            o["y"] = torch.empty(M, 136, device=DEV, dtype=dt)
            k.linear_dgrad(P["d2"], P["w2"], out=o["y"], gelu_grad_of=P["h2"], collect=c)

        def r_gg():
            hf = P["h2"].float()
            gg = 0.5 * (1 + torch.erf(hf / math.sqrt(2))) + hf * torch.exp(-0.5 * hf * hf) / math.sqrt(2 * math.pi)
            return {"y": (P["d2"].float() @ P["w2"].float()) * gg}

        def p_acc(c, o):
            o["y"] = P["y3"].clone()
            k.linear_dgrad(P["d3"], P["w3"], out=o["y"], accumulate=True, collect=c)

        def r_acc():
            return {"y": P["y3"].float() + P["d3"].float() @ P["w3"].float()}

        def p_short(c, o):  # K = 64: not a ring member
            o["y"] = torch.empty(M, 72, device=DEV, dtype=dt)
            k.linear_dgrad(P["d4"], P["w4"], out=o["y"], collect=c)

        def r_short():
            return {"y": P["d4"].float() @ P["w4"].float()}

        P = dict(d1=rn(M, 256), w1=rn(256, 200, scale=0.06), d2=rn(M, 192), w2=rn(192, 136, scale=0.07),
                 h2=rn(M, 136), d3=rn(M, 320), w3=rn(320, 96, scale=0.05), y3=rn(M, 96), d4=rn(M, 64),
                 w4=rn(64, 72, scale=0.1))
        probs = [(p_plain, r_plain), (p_gg, r_gg), (p_acc, r_acc), (p_short, r_short)]
    grouped = [dict() for _ in probs]
    k.gemm_many([lambda c, f=f, o=o: f(c, o) for (f, _), o in zip(probs, grouped)])
    single = [dict() for _ in probs]
    for (f, _), o in zip(probs, single):
        k.gemm_many([lambda c, f=f, o=o: f(c, o)])
    torch.cuda.synchronize()
    ulp = {torch.bfloat16: 2.0 ** -7, torch.float16: 2.0 ** -10}[dt]
    for i, ((f, ref), og, os_) in enumerate(zip(probs, grouped, single)):
        want = ref()
        for key, w in want.items():
            assert rel(og[key].float(), w) < GTOL[dt] * (2 if key == "pre" else 1), (i, f.__name__, key)
            assert rel(og[key].float(), os_[key].float()) <= ulp, (i, f.__name__, key)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("M,N,Kd,ldo", [(19200, 256, 384, 640), (1999, 136, 192, 136), (300, 40, 96, 48),
                                        (4800, 128, 1536, 128), (307200, 64, 96, 64)])
def test_dgrad_second_output_epilogue(dt, M, N, Kd, ldo):
    """Input-gradient GEMM with the second epilogue output (the backward of an elementwise product riding
    on the GEMM that produces its incoming gradient): out = (dy W) * mul, out2 = (dy W) * mul2, on the
    ring / register-staged / split-K routes, a strided output view, ragged N and the scalar tail."""
    k = K()
    g = torch.Generator(device=DEV).manual_seed(M + N)
    dy = (torch.randn(M, Kd, device=DEV, generator=g)).to(dt)
    wfull = (torch.randn(Kd, N + 24, device=DEV, generator=g) / Kd ** 0.5).to(dt)
    w = wfull[:, 8:8 + N]  # a column block of a wider weight (ldb = N + 24)
    m1 = torch.randn(M, N, device=DEV, generator=g).to(dt)
    m2 = torch.randn(M, N, device=DEV, generator=g).to(dt)
    outb = torch.zeros(M, ldo, device=DEV, dtype=dt)
    out = outb[:, :N]
    out2 = torch.empty(M, N, device=DEV, dtype=dt)
    k.linear_dgrad(dy, w, out=out, mul=m1, mul2=m2, out2=out2)
    base = dy.float() @ w.float()
    assert rel(out.float(), base * m1.float()) < GTOL[dt]
    assert rel(out2.float(), base * m2.float()) < GTOL[dt]
    # identical to the plain GEMM followed by the two products on the same (rounded) accumulator
    plain = k.linear_dgrad(dy, w)
    if dt == torch.float32:
        assert rel(out2.float(), plain.float() * m2.float()) < 1e-6


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("rows", [19200, 777, 4800])
def test_wgrad_group(dt, rows):
    """dfm_gemm_group: the weight gradients queued inside kernels.wgrad_group() (different M / N, bias
    gradient columns, an accumulating problem, strided operand views) against torch fp32 and against
    the same GEMMs launched one by one."""
    k = K()
    shapes = [(256, 256, True), (640, 256, True), (128, 128, False), (384, 512, True), (64, 96, True),
              (1024, 256, True), (256, 1024, False), (128, 384, True), (32, 48, True)]
    dys, xs, refs = [], [], []
    for n_out, n_in, bias in shapes:
        dyb = torch.randn(rows, n_out + 8, device=DEV).to(dt)
        dys.append(dyb[:, 8:])
        xs.append(torch.randn(rows, n_in, device=DEV).to(dt))
    base = torch.randn(128, 128, device=DEV)
    outs = []
    with k.wgrad_group():
        for i, (n_out, n_in, bias) in enumerate(shapes):
            if i == 2:  # accumulate into an existing gradient
                o = base.clone()
                k.linear_wgrad(dys[i], xs[i], out=o, accumulate=True)
                outs.append((o, None))
            else:
                outs.append(k.linear_wgrad(dys[i], xs[i], bias_grad=bias) if bias else (k.linear_wgrad(dys[i], xs[i]), None))
    for i, (n_out, n_in, bias) in enumerate(shapes):
        ref = dys[i].float().t() @ xs[i].float()
        if i == 2:
            ref = ref + base
        dw, db = outs[i]
        assert rel(dw, ref) < TOL[dt] * 2, (i, rel(dw, ref))
        if bias:
            assert rel(db, dys[i].float().sum(0)) < TOL[dt], i
        single = k.linear_wgrad(dys[i], xs[i], bias_grad=bias)
        sw = single[0] if bias else single
        if i != 2:
            assert rel(dw, sw) < (1e-5 if dt == torch.float32 else TOL[dt]), i


@pytest.mark.parametrize("dt", DTYPES)
def test_gemm_nmf_backward_input_gradient_descriptor(dt):
    """The exact descriptor of the NMF backward's input gradient (decoders.py NMF2DFn.backward:
    gx = Pc Qc^T, M = N_pix 4800, N = D 512, K = T*R 896, batch 16, both operands k-contiguous), the
    call a round-3 profiling run faulted next to (hipErrorIllegalAddress): through dfm_gemm vs torch
    fp32, synchronised, plus a re-run into a poisoned output (every element rewritten)."""
    k = K()
    B, N, D, KR = 16, 4800, 512, 896
    pc = torch.randn(B, N, KR, device=DEV).to(dt)
    qc = torch.randn(B, D, KR, device=DEV).to(dt)
    gx = k.bmm(pc, qc, b_t=True)
    torch.cuda.synchronize()
    ref = torch.bmm(pc.float(), qc.float().transpose(1, 2))
    assert gx.shape == (B, N, D) and gx.dtype == dt
    assert rel(gx.float(), ref) < GTOL[dt]
    out = torch.full_like(gx, float("nan"))
    k.bmm(pc, qc, b_t=True, out=out)
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all()
    assert torch.equal(out, gx)  # deterministic


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
# (the last three: the tall short-K kernel, its K padded to a multiple of 32 — DFormer-Large's C = 48 —,
# ragged M, strided A)
@pytest.mark.parametrize("M,N,Kd,ldx", [(19200, 256, 256, 256), (4800 + 37, 200, 1024, 1032), (130, 64, 64, 64),
                                        (307200 // 16, 512, 64, 64), (777, 1152, 128, 136), (70000, 384, 48, 56),
                                        (65536 + 77, 192, 80, 80), (66000, 160, 112, 120)])
def test_gemm_fused_epilogues_step_shapes(dt, M, N, Kd, ldx):
    """Forward and input-gradient GEMMs at step-like shapes (whichever kernel the routing picks) with
    every fused epilogue the Block uses: bias + GELU with GELU' stored from a column offset (act 3),
    the multiplier, the residual with column / row scales, beta accumulation, the GELU'-multiplier
    of an input gradient; ragged M, N % 64 != 0, strided A, one-slice (K = 64) tiles."""
    k = K()
    tol = GTOL[dt]
    xb = torch.randn(M, ldx, device=DEV).to(dt)
    x = xb[:, :Kd]
    w = (torch.randn(N, Kd, device=DEV) / Kd ** 0.5).to(dt)
    b = torch.randn(N, device=DEV)
    lin = x.float() @ w.float().t() + b
    # act 3 from column c0: GELU(v) out, GELU'(v) in preact[:, :N - c0]
    c0 = (N // 2) // 8 * 8
    pre = torch.empty(M, N - c0, device=DEV, dtype=dt)
    y = k.linear(x, w, b, act=3, preact=pre, act_col0=c0)
    v = lin[:, c0:]
    cdf = 0.5 * (1 + torch.erf(v / math.sqrt(2)))
    pdf = torch.exp(-0.5 * v * v) / math.sqrt(2 * math.pi)
    assert rel(y[:, :c0].float(), lin[:, :c0]) < tol
    assert rel(y[:, c0:].float(), v * cdf) < tol
    assert rel(pre.float(), cdf + v * pdf) < 2 * tol
    # multiplier with preact (the conv-modulation q * a)
    mul = torch.randn(M, N, device=DEV).to(dt)
    pre2 = torch.empty(M, N, device=DEV, dtype=dt)
    y = k.linear(x, w, b, mul=mul, preact=pre2)
    assert rel(pre2.float(), lin) < tol
    assert rel(y.float(), lin * mul.float()) < tol
    # residual + layer scale + per-image row scale (Block residual / DropPath epilogue)
    res = torch.randn(M, N, device=DEV).to(dt)
    cs = torch.rand(N, device=DEV)
    rps = max(1, M // 5)
    rs = torch.rand((M + rps - 1) // rps, device=DEV)
    y = k.linear(x, w, b, res=res, colscale=cs, rowscale=rs, rows_per_scale=rps)
    rsx = rs.repeat_interleave(rps)[:M, None]
    assert rel(y.float(), res.float() + cs * rsx * lin) < tol
    # beta accumulate into the output
    acc = torch.randn(M, N, device=DEV).to(dt)
    want = acc.float() + lin
    k.linear(x, w, b, out=acc, beta=1.0)
    assert rel(acc.float(), want) < tol
    # input gradient: dx[M, N] = dy[M, Kd] @ wd[Kd, N], plain / GELU'-multiplier / accumulate
    dy = xb[:, :Kd]
    wd = (torch.randn(Kd, N, device=DEV) / Kd ** 0.5).to(dt)
    ref = dy.float() @ wd.float()
    assert rel(k.linear_dgrad(dy, wd).float(), ref) < tol
    h = torch.randn(M, N, device=DEV).to(dt)
    hf = h.float()
    gg = 0.5 * (1 + torch.erf(hf / math.sqrt(2))) + hf * torch.exp(-0.5 * hf * hf) / math.sqrt(2 * math.pi)
    assert rel(k.linear_dgrad(dy, wd, gelu_grad_of=h).float(), ref * gg) < tol
    assert rel(k.linear_dgrad(dy, wd, mul=h).float(), ref * hf) < tol
    dx = torch.randn(M, N, device=DEV).to(dt)
    want = dx.float() + ref
    k.linear_dgrad(dy, wd, out=dx, accumulate=True)
    assert rel(dx.float(), want) < tol


def test_pack_slices():
    """dfm_pack_slices: n sources of mixed dtypes side by side into one [rows, n*cols] tensor (the NMF
    backward's rank-R factors), exactly torch.cat of the converted sources."""
    k = K()
    srcs = [torch.randn(3, 50, 64, device=DEV).to(dt) for dt in (torch.float32, torch.bfloat16, torch.float32,
                                                                    torch.float16, torch.float32)]
    for odt in (torch.bfloat16, torch.float32, torch.float16):
        out = torch.empty(3, 50, 5 * 64, device=DEV, dtype=odt)
        k.pack_slices(srcs, out)
        assert torch.equal(out, torch.cat([s.to(odt) for s in srcs], -1))
    # the element-wise path: 12-column slices (not a multiple of 8)
    odd = [torch.randn(40, 12, device=DEV).to(dt) for dt in (torch.float32, torch.bfloat16, torch.float16)]
    out = torch.empty(40, 36, device=DEV, dtype=torch.bfloat16)
    k.pack_slices(odd, out)
    assert torch.equal(out, torch.cat([s.to(torch.bfloat16) for s in odd], -1))


@pytest.mark.parametrize("dt", DTYPES)
def test_deferred_reductions_bit_identical(dt):
    """Inside wgrad_group the reduction second stages (LN dgamma/dbeta, layer-scale dscale, DW3x3
    fused and DW7x7 weight gradients) are deferred to one dfm_partial_sum_group launch: the results
    must equal the immediate two-launch path bit for bit, including a DW7 weight gradient issued on a
    side stream and joined before the flush (the attention backward's depth branch)."""
    Kk = K()
    B, H, W, C = 2, 30, 40, 96
    P = B * H * W
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(P, C, device=DEV, generator=g).to(dt)
    dy = torch.randn(P, C, device=DEV, generator=g).to(dt)
    f = torch.randn(P, C, device=DEV, generator=g).to(dt)
    gam = torch.rand(C, device=DEV, generator=g) + 0.5
    bet = torch.randn(C, device=DEV, generator=g)
    ls = torch.rand(C, device=DEV, generator=g)
    rs = torch.rand(B, device=DEV, generator=g)
    w3 = torch.randn(C, 1, 3, 3, device=DEV, generator=g) / 3
    xn, mu, rstd = Kk.layernorm(x, gam, bet)

    def run():
        out = {}
        out["ln"] = Kk.layernorm_bwd(x, dy, gam, mu, rstd, dres=f)
        out["res"] = Kk.residual_bwd(dy, f, ls, rs, H * W)
        out["dw3"] = Kk.dwconv_bwd(x, dy, (B, H, W), w3, 3, add_identity=True)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            out["dw7"] = Kk.dwconv_bwd_weight(x, dy, (B, H, W), 7)
        torch.cuda.current_stream().wait_stream(side)
        return out

    ref = run()
    with Kk.wgrad_group():
        got = run()
    torch.cuda.synchronize()
    for k in ref:
        for a, b in zip(got[k], ref[k]):
            assert torch.equal(a, b), k


@pytest.mark.parametrize("dt", DTYPES)
def test_group_scale(dt):
    """dfm_group_scale: per-group (per-image) channel scale in one launch, in place and strided."""
    Kk = K()
    B, rows, C = 4, 300, 96
    x = torch.randn(B * rows, C, device=DEV).to(dt)
    sc = torch.rand(B, C, device=DEV)
    ref = (x.float().view(B, rows, C) * sc[:, None, :]).view(B * rows, C)
    got = Kk.group_scale(x, sc, rows)
    assert rel(got.float(), ref) <= TOL[dt] / 4
    wide = torch.randn(B * rows, C + 32, device=DEV).to(dt)
    v = wide[:, 16:16 + C]
    exp = (v.float().view(B, rows, C) * sc[:, None, :]).view(B * rows, C)
    Kk.group_scale(v, sc, rows, out=v)
    assert rel(v.float(), exp) <= TOL[dt] / 4


@pytest.mark.parametrize("rows", [4800, 77, 512])
def test_nmf_update_mm_fused(rows):
    """dfm_nmf_update_mm / _bwd_mm (rank 64, the den products fused) vs torch fp32 compositions of
    the same update (ham_head.py:120-141) and of its backward with the folded Gram gradient terms."""
    Kk = K()
    Bb, R, eps = 3, 64, 1e-6
    g0 = torch.Generator(device=DEV).manual_seed(9)
    a = torch.rand(Bb, rows, R, device=DEV, generator=g0) + 0.1
    num = torch.rand(Bb, rows, R, device=DEV, generator=g0)
    Bm = torch.rand(Bb, 96, R, device=DEV, generator=g0)
    M = Bm.transpose(1, 2) @ Bm
    out, den, o16 = Kk.nmf_update_mm(a, num, M, eps, bf16_copy=True)
    den_ref = a @ M
    out_ref = a * num / (den_ref + eps)
    assert rel(den, den_ref) < 1e-5 and rel(out, out_ref) < 1e-5
    assert torch.equal(o16, out.to(torch.bfloat16))
    g = torch.randn(Bb, rows, R, device=DEV, generator=g0)
    A2 = torch.rand(Bb, rows, R, device=DEV, generator=g0)
    S = torch.randn(Bb, R, R, device=DEV, generator=g0)
    ga, gnum, gden, g16 = Kk.nmf_update_bwd_mm(g, a, num, den, out, A2=A2, S=S, Mg=M, eps=eps, bf16_copy=True)
    ge = g + A2 @ (S + S.transpose(1, 2))
    r = 1.0 / (den + eps)
    gden_ref = -ge * out * r
    assert rel(gnum, ge * a * r) < 1e-5 and rel(gden, gden_ref) < 1e-5
    assert rel(ga, ge * num * r + gden_ref @ M) < 1e-5
    assert torch.equal(g16, gnum.to(torch.bfloat16))
    ga2, gnum2, gden2 = Kk.nmf_update_bwd_mm(g, a, num, den, out, eps=eps)  # no folded terms
    assert rel(ga2, g * num * r) < 1e-5 and rel(gden2, -g * out * r) < 1e-5


@pytest.mark.parametrize("dt,Bb,N,D,steps", [(torch.float32, 2, 300, 512, 6), (torch.bfloat16, 2, 300, 512, 7),
                                              (torch.bfloat16, 16, 4800, 512, 6), (torch.float16, 3, 77, 96, 2),
                                              (torch.float32, 1, 64, 64, 0)])
def test_nmf_entry_points(dt, Bb, N, D, steps):
    """dfm_nmf_fwd / dfm_nmf_bwd (the NMF2D forward and its gradient as two calls, ham_head.py:60-145)
    give the same bits as NMF2DFn's launch-by-launch path (entry=False) for y and gx, the inference
    form (nothing saved) the same y, and the fp32 result stays within rounding of a torch fp32
    restatement of the update loop and its autograd gradient."""
    from dformer_amd.decoders import NMF2DFn
    Kk = K()
    g0 = torch.Generator(device=DEV).manual_seed(11)
    x = torch.rand(Bb, N, D, device=DEV, generator=g0).to(dt)
    bases = torch.rand(Bb, D, 64, device=DEV, generator=g0)
    bases = bases / bases.norm(dim=1, keepdim=True)
    gy = (torch.randn(Bb, N, D, device=DEV, generator=g0) * 0.1).to(dt)
    outs = []
    for entry in (True, False):
        xr = x.clone().requires_grad_(True)
        y = NMF2DFn.apply(xr, bases.clone(), steps, 1e-6, entry)
        y.backward(gy)
        outs.append((y.detach(), xr.grad))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    with torch.no_grad():
        assert torch.equal(Kk.nmf_fwd(x, bases, steps, 1e-6), outs[0][0])
    if dt == torch.float32:  # torch fp32 restatement of the update loop and its gradient
        xf = x.clone().requires_grad_(True)
        Bt = bases.clone()
        C = torch.softmax(xf @ Bt, dim=-1)
        for _ in range(steps):
            C = C * (xf @ Bt) / (C @ (Bt.transpose(1, 2) @ Bt) + 1e-6)
            Bt = Bt * (xf.transpose(1, 2) @ C) / (Bt @ (C.transpose(1, 2) @ C) + 1e-6)
        C = C * (xf @ Bt) / (C @ (Bt.transpose(1, 2) @ Bt) + 1e-6)
        yr = C @ Bt.transpose(1, 2)
        yr.backward(gy)
        assert rel(outs[0][0], yr) < 1e-4 and rel(outs[0][1], xf.grad) < 1e-3


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("B,h,w,H,W,ncls", [(2, 60, 80, 480, 640, 40), (2, 8, 12, 64, 96, 40), (1, 30, 40, 120, 160, 37),
                                            (2, 7, 9, 28, 36, 64)])
def test_seg_loss_fwd_grad_fused(dt, B, h, w, H, W, ncls):
    """dfm_seg_loss_fwd_grad + dfm_seg_loss_bwd_gather (the training loss with its gradient partials
    from the same pass, factors 8 / 4) vs torch fp32 F.interpolate + cross_entropy(ignore 255) and
    its autograd gradient, with a loss scale; bitwise reproducible."""
    k = K()
    lg = torch.randn(B, h, w, ncls, device=DEV).to(dt)
    lab = torch.randint(0, ncls, (B, H, W), device=DEV)
    lab[torch.rand(B, H, W, device=DEV) < 0.1] = 255
    out, part = k.seg_loss_fwd_grad(lg.view(-1, ncls), B, h, w, ncls, lab)
    lr = lg.float().permute(0, 3, 1, 2).contiguous().requires_grad_()
    up = F.interpolate(lr, (H, W), mode="bilinear", align_corners=False)
    ce = F.cross_entropy(up, lab, reduction="none", ignore_index=255)
    loss = ce[lab != 255].mean()
    assert abs((out[0] / out[1]).item() - loss.item()) < 1e-4 * abs(loss.item())
    (loss * 3.0).backward()
    gs = torch.full((1,), 3.0, device=DEV)
    dl = k.seg_loss_bwd_gather(part, B, h, w, ncls, out, gs, torch.float32)
    assert rel(dl.view(B, h, w, ncls).permute(0, 3, 1, 2), lr.grad) < 1e-3
    out2, part2 = k.seg_loss_fwd_grad(lg.view(-1, ncls), B, h, w, ncls, lab)
    dl2 = k.seg_loss_bwd_gather(part2, B, h, w, ncls, out2, gs, torch.float32)
    assert torch.equal(out, out2) and torch.equal(dl, dl2)
    dl16 = k.seg_loss_bwd_gather(part, B, h, w, ncls, out, gs, dt)  # written in the logits dtype directly
    assert rel(dl16.float(), dl) < (1e-6 if dt == torch.float32 else 4e-3)
