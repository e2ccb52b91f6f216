"""One encoder Block forward + backward through the C ABI alone (dfm_block_fwd / dfm_block_bwd over ctypes,
include/dformer_hip.h), against the reference's fp32 goldens (DFormer.py:147-181, 1e-3 like
tests/test_block_gpu.py) and, in bf16, against the Python autograd path built from the same kernels.
torch only allocates device memory here: no dformer_amd Python op runs on the C-ABI side."""
import ctypes

import numpy as np
import pytest
import torch

import gen
from goldens import check_param_grads, load, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")


def _meta(name):
    from test_block_gpu import make_block
    return make_block(name, "cpu")


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def run_capi(name, dtype, stack_qcl=False, fused_ffn=0, droppath=None):
    """dfm_block_fwd / _bwd on the golden's inputs; returns (y, ye, dx, dxe, {param name: grad})."""
    from dformer_amd import _lib
    g, blk, (B, H, W, C, stage, last, dp) = _meta(name)
    code = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16, torch.float16: _lib.F16}[dtype]
    sd = {k: v.detach().float().cuda() for k, v in blk.state_dict().items()}
    window = blk.attn.window
    hidden = sd["mlp.fc1.weight"].shape[0]
    d = _lib.BlockDesc(B, H, W, C, blk.attn.num_head, window, hidden, int(last), fused_ffn, 1e-6)
    keep = []  # device buffers referenced by pointer only

    def dev(t):
        keep.append(t)
        return t.data_ptr()

    params = (ctypes.c_void_p * len(_lib.BLOCK_PARAM_NAMES))()
    grads = (ctypes.c_void_p * len(_lib.BLOCK_PARAM_NAMES))()
    gbuf = {}
    stacked = None
    if stack_qcl:  # q | q_cut | l weights and biases contiguous: one GEMM forward
        names = ("attn.q", "attn.q_cut", "attn.l")
        stacked = (torch.cat([sd[n + ".weight"] for n in names]).to(dtype).contiguous(),
                   torch.cat([sd[n + ".bias"] for n in names]).contiguous())
        keep.extend(stacked)
    for i, n in enumerate(_lib.BLOCK_PARAM_NAMES):
        if n not in sd:
            continue
        t = sd[n]
        if n in _lib.BLOCK_GEMM_WEIGHTS:
            t = t.to(dtype)
        params[i] = dev(t.contiguous())
        gbuf[n] = torch.full_like(sd[n], float("nan"))  # every gradient must be written
        grads[i] = dev(gbuf[n])
    if stacked is not None:
        w, b = stacked
        rows = [0, C, C + C // 2]
        for j, n in enumerate(("attn.q", "attn.q_cut", "attn.l")):
            params[_lib.BLOCK_PARAM_NAMES.index(n + ".weight")] = w.data_ptr() + rows[j] * C * w.element_size()
            params[_lib.BLOCK_PARAM_NAMES.index(n + ".bias")] = b.data_ptr() + rows[j] * 4
    rs = None
    if droppath is not None:
        rs = (ctypes.c_void_p * 4)(*[dev(torch.tensor(m, dtype=torch.float32, device="cuda")) for m in droppath])
    x = torch.from_numpy(gen.normal(name + "/x", (B, H, W, C))).to("cuda", dtype).contiguous()
    xe = torch.from_numpy(gen.normal(name + "/xe", (B, H, W, C // 2))).to("cuda", dtype).contiguous()
    y = torch.empty_like(x)
    ye = torch.empty_like(xe)
    with_ye = "y_e" in g  # every Block with an x_e output; a drop_depth Block's e_back output (*_ye goldens)
    nsv = _lib.lib.dfm_block_saved_size(code, d)
    nws = _lib.lib.dfm_block_workspace_size(code, d)
    assert nsv > 0 and nws > 0
    saved = torch.empty(nsv, dtype=torch.uint8, device="cuda")
    ws = torch.empty(nws, dtype=torch.uint8, device="cuda")
    st = _lib.lib.dfm_block_fwd(code, d, params, rs, x.data_ptr(), xe.data_ptr(), y.data_ptr(),
                                ye.data_ptr() if with_ye else None, saved.data_ptr(), nsv, ws.data_ptr(), nws, _stream())
    assert st == 0, _lib.lib.dfm_last_error()
    gy = torch.from_numpy(gen.normal(name + "/gy", y.shape)).to("cuda", dtype).contiguous()
    gye = torch.from_numpy(gen.normal(name + "/gye", ye.shape)).to("cuda", dtype).contiguous() if with_ye else None
    dx, dxe = torch.empty_like(x), torch.empty_like(xe)
    st = _lib.lib.dfm_block_bwd(code, d, params, rs, x.data_ptr(), xe.data_ptr(), saved.data_ptr(), nsv, gy.data_ptr(),
                                None if gye is None else gye.data_ptr(), dx.data_ptr(), dxe.data_ptr(), grads,
                                ws.data_ptr(), nws, _stream())
    assert st == 0, _lib.lib.dfm_last_error()
    torch.cuda.synchronize()
    return g, not with_ye, y, (ye if with_ye else None), dx, dxe, gbuf


CASES = [("block_base_s0", False), ("block_base_s2", False), ("block_base_s2", True), ("block_base_s3_last", False),
         ("block_tiny_s1", True), ("block_tiny_s3_last_ye", False)]


@pytest.mark.parametrize("name,stack", CASES)
def test_block_capi_fp32_vs_reference_goldens(name, stack):
    g, last, y, ye, dx, dxe, grads = run_capi(name, torch.float32, stack_qcl=stack)
    tol = 1e-3
    assert rel_err(y.cpu(), g["y"]) < tol
    assert rel_err(dx.cpu(), g["gx"]) < tol
    if not last:
        assert rel_err(ye.cpu(), g["y_e"]) < tol
        assert rel_err(dxe.cpu(), g["gxe"]) < tol
    for n, t in grads.items():
        assert torch.isfinite(t).all(), n
    check_param_grads(g, {k: v.cpu() for k, v in grads.items()}, tol)


def test_block_capi_droppath_vs_reference_golden():
    """Per-sample DropPath scales (keep mask / keep prob) through the rowscale array, mmcv's call order."""
    g, blk, (B, H, W, C, stage, last, dp) = _meta("block_droppath_base_s1")
    keep = 1.0 - dp
    masks = [[m / keep for m in ms] for ms in ([1.0, 0.0], [0.0, 1.0], [1.0, 1.0], [0.0, 1.0])]
    g, last, y, ye, dx, dxe, grads = run_capi("block_droppath_base_s1", torch.float32, droppath=masks)
    tol = 1e-3
    assert rel_err(y.cpu(), g["y"]) < tol and rel_err(ye.cpu(), g["y_e"]) < tol
    assert rel_err(dx.cpu(), g["gx"]) < tol and rel_err(dxe.cpu(), g["gxe"]) < tol
    check_param_grads(g, {k: v.cpu() for k, v in grads.items()}, tol)


@pytest.mark.parametrize("name", ["block_base_s0", "block_base_s2", "block_base_s3_last"])
@pytest.mark.parametrize("fused", [0, 1])
def test_block_capi_bf16_vs_autograd_path(name, fused):
    """bf16 through the C ABI (op-level or fused ConvFFNs) against the Python autograd Block on the same
    kernels: the two differ only in GEMM grouping / split-K summation order, so they agree far inside
    the bf16 golden gates (tests/test_block_gpu.py)."""
    from test_block_gpu import run_block
    g, last, y, ye, dx, dxe, grads = run_capi(name, torch.bfloat16, stack_qcl=True, fused_ffn=fused)
    _, blk, x_ref, xe_ref, y_ref, ye_ref, _ = run_block(name, torch.bfloat16)
    pairs = [("y", y, y_ref), ("dx", dx, x_ref.grad)]
    if not last:
        pairs += [("ye", ye, ye_ref), ("dxe", dxe, xe_ref.grad)]
    pairs += [(n, grads[n], p.grad) for n, p in blk.named_parameters() if p.grad is not None]
    bad = {}
    for n, a, b in pairs:
        e = rel_err(a.detach().float().cpu(), b.detach().float().cpu())
        if not np.isfinite(e) or e > 2e-2:
            bad[n] = e
    assert not bad, bad


@pytest.mark.parametrize("name", ["block_base_s0", "block_base_s2", "block_base_s3_last", "block_base_s0_120x160"])
@pytest.mark.parametrize("fused", [0, 1])
def test_block_capi_bf16_vs_reference_goldens(name, fused):
    """bf16 through the C ABI alone, op-level or fused ConvFFNs, against the REFERENCE golden at the same
    per-tensor gates as the autograd Block (4x the reference's own bf16 error, tests/test_block_gpu.py)."""
    from test_block_gpu import bf16_envelope_check
    g, last, y, ye, dx, dxe, grads = run_capi(name, torch.bfloat16, stack_qcl=True, fused_ffn=fused)
    for n, t in grads.items():
        assert torch.isfinite(t).all(), n
    bf16_envelope_check(name, f"capi-fused{fused}", g, y, ye, dx, dxe, grads, last)


@pytest.mark.parametrize("which", ["params", "grads"])
def test_block_capi_rejects_null_entries(which):
    """A NULL params / grads entry for a parameter the Block has (a bias, a bias gradient) is DFM_ERR_ARG
    before any launch; entries the Block does not have (kv without a window) may stay NULL."""
    from dformer_amd import _lib
    g, blk, (B, H, W, C, stage, last, dp) = _meta("block_base_s0")  # window 0: no kv / short_cut_linear
    sd = {k: v.detach().float().cuda() for k, v in blk.state_dict().items()}
    d = _lib.BlockDesc(B, H, W, C, blk.attn.num_head, blk.attn.window, sd["mlp.fc1.weight"].shape[0], 0, 0, 1e-6)
    params = (ctypes.c_void_p * len(_lib.BLOCK_PARAM_NAMES))()
    grads = (ctypes.c_void_p * len(_lib.BLOCK_PARAM_NAMES))()
    keep = []
    for i, n in enumerate(_lib.BLOCK_PARAM_NAMES):
        if n in sd:
            keep += [sd[n].contiguous(), torch.zeros_like(sd[n])]
            params[i], grads[i] = keep[-2].data_ptr(), keep[-1].data_ptr()
    victim = _lib.BLOCK_PARAM_NAMES.index("attn.q.bias")
    (params if which == "params" else grads)[victim] = None
    x = torch.zeros(B * H * W, C, device="cuda")
    xe = torch.zeros(B * H * W, C // 2, device="cuda")
    nsv, nws = _lib.lib.dfm_block_saved_size(_lib.F32, d), _lib.lib.dfm_block_workspace_size(_lib.F32, d)
    saved = torch.zeros(nsv, dtype=torch.uint8, device="cuda")
    ws = torch.zeros(nws, dtype=torch.uint8, device="cuda")
    y, ye = torch.empty_like(x), torch.empty_like(xe)
    if which == "params":
        st = _lib.lib.dfm_block_fwd(_lib.F32, d, params, None, x.data_ptr(), xe.data_ptr(), y.data_ptr(),
                                    ye.data_ptr(), saved.data_ptr(), nsv, ws.data_ptr(), nws, _stream())
    else:
        st = _lib.lib.dfm_block_bwd(_lib.F32, d, params, None, x.data_ptr(), xe.data_ptr(), saved.data_ptr(), nsv,
                                    y.data_ptr(), ye.data_ptr(), x.data_ptr(), xe.data_ptr(), grads, ws.data_ptr(),
                                    nws, _stream())
    assert st != 0
    assert f"entry {victim} is NULL".encode() in _lib.lib.dfm_last_error()
