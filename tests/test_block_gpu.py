"""Parity of the HIP encoder Block against the reference goldens (fp32, 1e-3) and the oracle (bf16)."""
import numpy as np
import pytest
import torch

import dformer_ref as R
import gen
from goldens import MODELS, RATIOS, check_param_grads, load, rel_err

BLOCKS = ["block_tiny_s0", "block_tiny_s1", "block_tiny_s3_last", "block_base_s0", "block_base_s1",
          "block_base_s2", "block_base_s3", "block_base_s3_last", "block_large_s1", "block_large_s2",
          "block_droppath_base_s1"]


def make_block(name, device="cpu"):
    from dformer_amd.encoder import Block
    g = load(name)
    B, H, W, C, stage, last, dp = [int(v) for v in g["meta"]]
    model = "base" if "droppath" in name else name.split("_")[1]
    m = MODELS[model]
    depth = m["depths"][stage]
    j = depth - 1 if last else 0
    blk = Block(index=0, dim=C, num_head=m["heads"][stage], mlp_ratio=RATIOS[stage], block_index=depth - j,
                window=0 if stage == 0 else 7, dropout_layer=dict(type="DropPath", drop_prob=dp / 1e6),
                drop_depth=bool(last))
    sd = blk.state_dict()
    vals = gen.state_dict_values([(k, v.shape) for k, v in sd.items()])
    blk.load_state_dict({k: torch.from_numpy(np.asarray(v)).float() for k, v in vals.items()})
    return g, blk.to(device), (B, H, W, C, stage, bool(last), dp / 1e6)


@pytest.mark.parametrize("name", BLOCKS)
def test_block_state_dict_matches_reference_layout(name):
    g, blk, (B, H, W, C, stage, last, dp) = make_block(name)
    shapes = R.block_shapes(C, RATIOS[stage], 0 if stage == 0 else 7, last)
    sd = {k: tuple(v.shape) for k, v in blk.state_dict().items()}
    assert sd == shapes
    names = {k.split("/", 1)[1] for k in g if k.startswith("grad")}
    assert names <= set(sd)


def run_block(name, dtype):
    from dformer_amd.functional import invalidate_weights
    g, blk, (B, H, W, C, stage, last, dp) = make_block(name, "cuda")
    invalidate_weights()
    blk.train()
    if dp:
        blk.drop_path_masks = [torch.tensor(m) for m in ([1.0, 0.0], [0.0, 1.0], [1.0, 1.0], [0.0, 1.0])]
    x = torch.from_numpy(gen.normal(name + "/x", (B, H, W, C))).to("cuda", dtype).requires_grad_()
    xe = torch.from_numpy(gen.normal(name + "/xe", (B, H, W, C // 2))).to("cuda", dtype).requires_grad_()
    y, ye = blk(x, xe)
    gy = torch.from_numpy(gen.normal(name + "/gy", y.shape)).to("cuda", dtype)
    if last:
        y.backward(gy)
    else:
        gye = torch.from_numpy(gen.normal(name + "/gye", ye.shape)).to("cuda", dtype)
        torch.autograd.backward([y, ye], [gy, gye])
    torch.cuda.synchronize()
    return g, blk, x, xe, y, ye, last


@pytest.mark.gpu
@pytest.mark.parametrize("name", BLOCKS)
def test_block_fp32_vs_reference_goldens(name):
    g, blk, x, xe, y, ye, last = run_block(name, torch.float32)
    tol = 1e-3
    assert rel_err(y.cpu(), g["y"]) < tol
    assert rel_err(x.grad.cpu(), g["gx"]) < tol
    if not last:
        assert rel_err(ye.cpu(), g["y_e"]) < tol
        assert rel_err(xe.grad.cpu(), g["gxe"]) < tol
    grads = {k: p.grad.cpu() for k, p in blk.named_parameters() if p.grad is not None}
    check_param_grads(g, grads, tol)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["block_tiny_s1", "block_base_s0", "block_base_s1", "block_base_s2",
                                  "block_base_s3", "block_large_s2"])
def test_block_bf16_vs_reference_goldens(name):
    """bf16 gate is per Block on rel-to-max: forward 1e-2; input grads 2e-2."""
    g, blk, x, xe, y, ye, last = run_block(name, torch.bfloat16)
    assert rel_err(y.float().cpu(), g["y"]) < 1e-2
    assert rel_err(ye.float().cpu(), g["y_e"]) < 1e-2
    assert rel_err(x.grad.float().cpu(), g["gx"]) < 2e-2
    assert rel_err(xe.grad.float().cpu(), g["gxe"]) < 2e-2
