"""Pin the CPU oracle (oracle/dformer_ref.py) against the reference's golden vectors.

CPU-only. The goldens were produced by running the read-only reference in float64
(oracle/make_goldens.py); the oracle restatement must reproduce them to ~1e-6.
"""
import numpy as np
import pytest
import torch

import dformer_ref as R
import gen
from goldens import MODELS, RATIOS, check_param_grads, fp_rel_err, load, params, rel_err, input_seed

TOL = 1e-6  # float64 restatement vs float64 reference (goldens stored in float32)

BLOCKS = ["block_tiny_s0", "block_tiny_s1", "block_tiny_s3_last", "block_base_s0", "block_base_s1",
          "block_base_s2", "block_base_s3", "block_base_s3_last", "block_large_s1", "block_large_s2",
          "block_droppath_base_s1", "block_tiny_s3_last_ye", "block_base_s0_120x160"]


def run_block(name, dtype=torch.float64):
    g = load(name)
    B, H, W, C, stage, last, dp = [int(v) for v in g["meta"]]
    model = name.split("_")[1] if "droppath" not in name else "base"
    heads = MODELS[model]["heads"][stage]
    window = 0 if stage == 0 else 7
    p = params(R.block_shapes(C, RATIOS[stage], window, bool(last)), dtype)
    x = torch.from_numpy(gen.normal(name + "/x", (B, H, W, C))).to(dtype).requires_grad_()
    xe = torch.from_numpy(gen.normal(name + "/xe", (B, H, W, C // 2))).to(dtype).requires_grad_()
    masks = None
    drop = dp / 1e6
    if drop:
        masks = [torch.tensor(m) for m in ([1.0, 0.0], [0.0, 1.0], [1.0, 1.0], [0.0, 1.0])]
    y, ye = R.block(p, "", x, xe, heads, window, bool(last), drop, masks)
    loss = (y * torch.from_numpy(gen.normal(name + "/gy", y.shape)).to(dtype)).sum()
    with_ye = "y_e" in g  # every Block with x_e output, and a drop_depth Block's e_back output (*_ye)
    if with_ye:
        loss = loss + (ye * torch.from_numpy(gen.normal(name + "/gye", ye.shape)).to(dtype)).sum()
    loss.backward()
    return g, p, x, xe, y, ye, not with_ye


@pytest.mark.parametrize("name", BLOCKS)
def test_block_golden(name):
    g, p, x, xe, y, ye, last = run_block(name)
    assert rel_err(y, g["y"]) < TOL
    assert rel_err(x.grad, g["gx"]) < TOL
    if not last:
        assert rel_err(ye, g["y_e"]) < TOL
        assert rel_err(xe.grad, g["gxe"]) < TOL
    check_param_grads(g, {k: v.grad for k, v in p.items() if v.grad is not None}, TOL)
    # every reference parameter with a gradient exists in the restated layout
    names = {k.split("/", 1)[1] for k in g if k.startswith("grad")}
    assert names <= set(p), names - set(p)


@pytest.mark.parametrize("name", ["nmf_train", "nmf_eval"])
def test_nmf_golden(name):
    g = load(name)
    B, C, H, W, train = [int(v) for v in g["meta"]]
    bases = torch.from_numpy(gen.nmf_bases(B, C, 64, name=name + "/bases"))
    x = torch.from_numpy(gen.uniform(name + "/x", (B, C, H, W))).requires_grad_()
    y = R.nmf2d(x, bases, bool(train))
    (y * torch.from_numpy(gen.normal(name + "/gy", y.shape))).sum().backward()
    assert rel_err(y, g["y"]) < TOL
    assert rel_err(x.grad, g["gx"]) < 1e-5


def test_ham_head_golden():
    name = "ham_tiny"
    g = load(name)
    B, H, W, ncls, train, seed, *in_ch = [int(v) for v in g["meta"]]
    tag = f"{name}#{seed}"  # the input draw whose ReLU inputs stay off the kink (make_goldens.golden_ham)
    p = params(R.ham_shapes(in_ch, ncls, pre=""))
    feats = [torch.from_numpy(gen.normal(tag + f"/f{i}", (B, c, H >> i, W >> i))).requires_grad_()
             for i, c in enumerate(in_ch)]
    bases = torch.from_numpy(gen.nmf_bases(B, 512, 64, name=tag + "/bases"))
    bufs = {k: v.clone() for k, v in p.items() if "running" in k}
    y = R.ham_head(p, "", feats, bases, bool(train), buffers=bufs)
    (y * torch.from_numpy(gen.normal(tag + "/gy", y.shape))).sum().backward()
    assert float(g["margin"]) > 1e-5
    assert rel_err(y, g["y"]) < TOL
    for i, f in enumerate(feats):
        assert rel_err(f.grad, g[f"gf{i + 1}"]) < 1e-5
    check_param_grads(g, {k: v.grad for k, v in p.items() if v.grad is not None}, 1e-5)
    for k, v in g.items():
        if k.startswith("buf/"):
            assert rel_err(bufs[k[4:]], v) < TOL


def test_mlp_decoder_golden():
    name = "mlpdec_small"
    g = load(name)
    B, H, W, ncls, embed, *in_ch = [int(v) for v in g["meta"]]
    p = params(R.mlpdec_shapes(in_ch, ncls, embed, pre=""))
    sizes = [(H, W)]
    for _ in range(3):
        sizes.append(((sizes[-1][0] - 1) // 2 + 1, (sizes[-1][1] - 1) // 2 + 1))
    feats = [torch.from_numpy(gen.normal(name + f"/f{i}", (B, c, *sizes[i]))).requires_grad_()
             for i, c in enumerate(in_ch)]
    bufs = {k: v.clone() for k, v in p.items() if "running" in k}
    y = R.mlp_decoder(p, "", feats, True, buffers=bufs)
    (y * torch.from_numpy(gen.normal(name + "/gy", y.shape))).sum().backward()
    assert rel_err(y, g["y"]) < TOL
    for i, f in enumerate(feats):
        assert rel_err(f.grad, g[f"gf{i}"]) < 1e-5
    check_param_grads(g, {k: v.grad for k, v in p.items() if v.grad is not None}, 1e-5)


E2E = [("e2e_tiny_small", "DFormer-Tiny", "ham", 40), ("e2e_base_small", "DFormer-Base", "ham", 40),
       ("e2e_large_mlp_small", "DFormer-Large", "MLPDecoder", 37)]


@pytest.mark.parametrize("name,arch,dec,ncls", E2E)
def test_e2e_golden(name, arch, dec, ncls):
    g = load(name)
    B, H, W, _ = [int(v) for v in g["meta"][:4]]
    p = params(R.segmentor_shapes(arch, dec, ncls))
    rgb_np, dep_np = gen.rgb_depth(B, H, W, seed=input_seed(g))
    rgb = torch.from_numpy(rgb_np).requires_grad_()
    dep = torch.from_numpy(dep_np).requires_grad_()
    lab = torch.from_numpy(gen.labels(B, H, W, ncls))
    bases = torch.from_numpy(gen.nmf_bases(B, 512, 64, name=name + "/bases")) if dec == "ham" else None
    bufs = {k: v.clone() for k, v in p.items() if "running" in k}
    feats, low, loss = R.segmentor_forward(p, arch, dec, rgb, dep, bases, True, lab, buffers=bufs)
    loss.backward()
    for i, f in enumerate(feats):
        assert rel_err(f, g[f"feat{i}"]) < 1e-6
    assert rel_err(low, g["low"]) < 1e-6
    assert abs(loss.item() - float(g["loss"])) < 1e-9 * max(1.0, abs(float(g["loss"])))
    assert fp_rel_err(gen.fingerprint(rgb.grad.numpy()), g["grgb_fp"]) < 1e-5
    assert fp_rel_err(gen.fingerprint(dep.grad.numpy()), g["gdep_fp"]) < 1e-5
    seen = 0
    for k, v in g.items():
        if k.startswith("gfp/"):
            n = k[4:]
            assert fp_rel_err(gen.fingerprint(p[n].grad.numpy(), 16), v) < 1e-5, n
            seen += 1
    assert seen > 100
    # parameters that never receive a gradient in the reference: stem_e_fc1/2 (DFormer.py:202-203)
    assert not any("stem_e_fc" in k for k in g)


@pytest.mark.slow
def test_e2e_tiny_full_resolution_forward():
    """BASELINE config 1: Tiny forward at 2x3x480x640 (fingerprints)."""
    name = "e2e_tiny_full_fwd"
    g = load(name)
    B, H, W, ncls = [int(v) for v in g["meta"][:4]]
    p = params(R.segmentor_shapes("DFormer-Tiny"), requires_grad=False)
    rgb, dep = (torch.from_numpy(a) for a in gen.rgb_depth(B, H, W, seed=input_seed(g)))
    bases = torch.from_numpy(gen.nmf_bases(B, 512, 64, name=name + "/bases"))
    bufs = {k: v.clone() for k, v in p.items() if "running" in k}
    with torch.no_grad():
        feats, low = R.segmentor_forward(p, "DFormer-Tiny", "ham", rgb, dep, bases, True, buffers=bufs)
    assert fp_rel_err(gen.fingerprint(low.numpy()), g["low_fp"]) < 1e-6
    for i, f in enumerate(feats):
        assert fp_rel_err(gen.fingerprint(f.numpy()), g[f"feat{i}_fp"]) < 1e-6


def test_optimizer_groups_golden():
    """group_weight quirk: layer_scale_* and the custom LayerNorm params are in no group."""
    g = load("groups_base")
    excluded = set(g["excluded"].tolist())
    shapes = R.segmentor_shapes("DFormer-Base")
    assert all(("layer_scale" in n) or (".norm" in n and "bn" not in n) for n in excluded)
    n_excl = sum(int(np.prod(shapes[n])) for n in excluded)
    assert n_excl == int(g["counts"][0]) == 41024
    assert len(excluded) == 236


@pytest.mark.parametrize("name,arch,dec,ncls,embed", [("msf_tiny_ham", "DFormer-Tiny", "ham", 40, 512),
                                                      ("msf_tiny_mlp", "DFormer-Tiny", "MLPDecoder", 37, 64)])
def test_msf_golden(name, arch, dec, ncls, embed):
    """The oracle's evaluate_msf restatement (msf_scores, confusion) against the reference's own
    evaluate_msf run (utils/val_mm.py:325-472; oracle/make_goldens.py golden_msf)."""
    g = load(name)
    B, H, W, _, flip = [int(v) for v in g["meta"]]
    scales = [float(s) for s in g["scales"]]
    p = params(R.segmentor_shapes(arch, dec, ncls, embed), requires_grad=False)
    bufs = {k: v.clone() for k, v in p.items() if "running" in k}
    bases = torch.from_numpy(gen.nmf_bases(B, 512, 64, name=name + "/bases")) if dec == "ham" else None
    hist = 0
    for i in range(2):
        rgb, dep = (torch.from_numpy(a) for a in gen.rgb_depth(B, H, W, seed=8964 + i))
        lab = torch.from_numpy(gen.labels(B, H, W, ncls, seed=8964 + i))
        with torch.no_grad():
            sc = R.msf_scores(p, arch, dec, rgb, dep, ncls, scales, bool(flip), bases, buffers=bufs)
        assert rel_err(sc, g[f"scores{i}"]) < 1e-6
        hist = hist + R.confusion(sc, lab, ncls)
    assert np.array_equal(hist.numpy(), g["hist"])
