"""Helpers shared by the tests: golden loading, seeded parameter dicts, comparisons."""
import os

import numpy as np
import torch

import gen  # oracle/gen.py (tests may use the oracle as the checker)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MODELS = {
    "tiny": dict(dims=[32, 64, 128, 256], heads=[1, 2, 4, 8], depths=[3, 3, 5, 2]),
    "base": dict(dims=[64, 128, 256, 512], heads=[1, 2, 4, 8], depths=[3, 3, 12, 2]),
    "large": dict(dims=[96, 192, 288, 576], heads=[1, 2, 4, 8], depths=[3, 3, 12, 2]),
}
RATIOS = [8, 8, 4, 4]


def input_seed(g):
    """The rgb / depth input seed of an end-to-end golden (meta[4] when make_goldens searched for an
    off-kink draw, else gen.rgb_depth's default)."""
    m = np.asarray(g["meta"])
    return int(m[4]) if m.size > 4 else 8964


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def params(shapes, dtype=torch.float64, requires_grad=True, seed=1234):
    vals = gen.state_dict_values(shapes.items(), seed)
    out = {}
    for k, v in vals.items():
        t = torch.from_numpy(np.asarray(v))
        if t.is_floating_point():
            t = t.to(dtype)
            if requires_grad and "running" not in k:
                t.requires_grad_(True)
        out[k] = t
    return out


def rel_err(a, b):
    """max|a-b| / max|b| (relative-to-max)."""
    a = torch.as_tensor(np.asarray(a) if not torch.is_tensor(a) else a).double().cpu()
    b = torch.as_tensor(np.asarray(b) if not torch.is_tensor(b) else b).double().cpu()
    assert a.shape == b.shape, (a.shape, b.shape)
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def fp_rel_err(fp_a, fp_b, atol=1e-9):
    """Compare two gen.fingerprint vectors: sum, abs-sum, l2 relative; the strided samples as a
    relative L2 error ||a_s - b_s|| / ||b_s||.

    The samples are NOT compared rel-to-max: a gradient's 1k strided samples can miss its largest
    entries by orders of magnitude (the image gradient of e2e_tiny_small peaks far above every
    sample), so max|da_s| / max|b_s| magnified an fp32 summation-order difference of 2e-6 of the
    tensor's own max into 1e-3..4e-3 (tools/fp32_audit.py measures the full tensors against the
    fp64 oracle). `atol` floors every denominator so mathematically-zero gradients (e.g. a conv bias
    feeding a train-mode BatchNorm) compare as equal noise instead of as 100 % relative error."""
    fa, fb = np.asarray(fp_a, np.float64), np.asarray(fp_b, np.float64)
    e_s = abs(fa[0] - fb[0]) / max(fb[1], atol)
    e_a = abs(fa[1] - fb[1]) / max(fb[1], atol)
    e_l = abs(fa[2] - fb[2]) / max(fb[2], atol)
    e_samp = np.linalg.norm(fa[3:] - fb[3:]) / max(np.linalg.norm(fb[3:]), atol)
    return max(e_s, e_a, e_l, e_samp)


def check_param_grads(gold, grads, tol, atol=1e-9):
    """grads: {name: tensor}. Compares every grad/ and gradfp/ entry in the golden.

    `atol` floors the relative-error denominator: some parameters have mathematically zero
    gradients (a bias feeding a train-mode BatchNorm, directly or through linear maps) whose
    golden values are pure fp64 rounding noise."""
    worst = 0.0
    seen = 0
    for k, v in gold.items():
        if k.startswith("grad/"):
            n = k[5:]
            a = torch.as_tensor(np.asarray(grads[n].detach().cpu())).double()
            b = torch.as_tensor(np.asarray(v)).double()
            if b.abs().max().item() < 1e-12:  # mathematically zero gradient: fp64 noise in the golden
                assert a.abs().max().item() < 1e-3, f"{n}: expected a (numerically) zero gradient"
                continue
            e = ((a - b).abs().max() / max(b.abs().max().item(), atol)).item()
        elif k.startswith("gradfp/"):
            n = k[7:]
            g = grads[n]
            e = fp_rel_err(gen.fingerprint(g.detach().double().cpu().numpy(), 256), v, atol=atol)
        else:
            continue
        seen += 1
        assert e < tol, f"{n}: rel err {e:.3e} >= {tol}"
        worst = max(worst, e)
    assert seen > 0
    return worst
