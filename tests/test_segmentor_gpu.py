"""End-to-end parity of the HIP segmentor (encoder + decoder + fused loss) with the reference
goldens, plus decoder-module goldens (NMF2D, LightHamHead, MLPDecoder) and a DDP-style step."""
import numpy as np
import pytest
import torch

import dformer_ref as R
import gen
from goldens import check_param_grads, fp_rel_err, load, params, rel_err, input_seed


class Cfg(dict):
    __getattr__ = dict.__getitem__


def build(arch, dec, ncls, device="cpu"):
    from dformer_amd.segmentor import EncoderDecoder
    cfg = Cfg(backbone=arch, decoder=dec, decoder_embed_dim=512, num_classes=ncls, drop_path_rate=0.0,
              bn_eps=1e-3, bn_momentum=0.1, background=255)
    model = EncoderDecoder(cfg=cfg, syncbn=False)
    model.decode_head.dropout_ratio = 0.0
    sd = model.state_dict()
    vals = gen.state_dict_values([(k, v.shape) for k, v in sd.items()])
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)).to(sd[k].dtype) for k, v in vals.items()})
    return model.to(device)


E2E = [("e2e_tiny_small", "DFormer-Tiny", "ham", 40), ("e2e_base_small", "DFormer-Base", "ham", 40),
       ("e2e_large_mlp_small", "DFormer-Large", "MLPDecoder", 37)]


@pytest.mark.parametrize("name,arch,dec,ncls", E2E)
def test_segmentor_state_dict_matches_reference(name, arch, dec, ncls):
    model = build(arch, dec, ncls)
    shapes = R.segmentor_shapes(arch, dec, ncls)
    sd = {k: tuple(v.shape) for k, v in model.state_dict().items() if not k.endswith("num_batches_tracked")}
    assert sd == shapes
    g = load(name)
    names = {k[4:] for k in g if k.startswith("gfp/")}
    assert names <= set(sd)


@pytest.mark.gpu
@pytest.mark.parametrize("name,arch,dec,ncls", E2E)
def test_segmentor_fp32_vs_reference(name, arch, dec, ncls):
    g = load(name)
    B, H, W, _ = [int(v) for v in g["meta"][:4]]
    model = build(arch, dec, ncls, "cuda")
    model.train()
    if dec == "ham":
        model.decode_head.hamburger.ham.injected_bases = torch.from_numpy(
            gen.nmf_bases(B, 512, 64, name=name + "/bases")).float()
    rgb_np, dep_np = gen.rgb_depth(B, H, W, seed=input_seed(g))
    rgb = torch.from_numpy(rgb_np).float().cuda().requires_grad_()
    dep = torch.from_numpy(dep_np).float().cuda().requires_grad_()
    lab = torch.from_numpy(gen.labels(B, H, W, ncls)).cuda()
    feats = model.encoder_backbone(rgb, dep)[0]
    low = model.decode_head(feats)
    from dformer_amd.decoders import SegLossFn, _nhwc_rows
    rows, (b, h, w) = _nhwc_rows(low)
    loss = SegLossFn.apply(rows.contiguous(), b, h, w, lab, 255)
    loss.backward()
    torch.cuda.synchronize()
    env = load("fp32env_" + name)
    for i, f in enumerate(feats):
        assert rel_err(f.float().cpu(), g[f"feat{i}"]) < 1e-4, i
    assert rel_err(low.float().cpu(), g["low"]) < 1e-4
    assert abs(loss.item() - float(g["loss"])) < 1e-5 * abs(float(g["loss"]))
    e_rgb = fp_rel_err(gen.fingerprint(rgb.grad.cpu().double().numpy()), g["grgb_fp"])
    assert e_rgb < fp32_gate(env["env/grgb"]), (e_rgb, float(env["env/grgb"]))
    bad = []
    for k, v in g.items():
        if k.startswith("gfp/"):
            p = dict(model.named_parameters())[k[4:]]
            e = fp_rel_err(gen.fingerprint(p.grad.cpu().double().numpy(), 16), v, atol=1e-4)
            if e > fp32_gate(env["env/" + k]):
                bad.append((k, e, float(env["env/" + k])))
    assert not bad, bad[:10]


# fp32 end-to-end gates, from the reference's OWN float32 error on each golden (tests/golden/
# fp32env_*.npz: the reference run in float32 vs its float64 golden, oracle/make_goldens.py
# golden_bf16_env(dtype=None)): 10 x that envelope, floored at 1e-4 — ten times tighter than
# SURVEY §8c's 1e-3 fp32 gate wherever the envelope allows (it allows it everywhere but for the
# mathematically-zero gradients of conv biases ahead of a train-mode BatchNorm, whose fingerprints
# are rounding noise in the reference too). tools/fp32_audit.py / test_segmentor_fp32_vs_oracle_full
# check the full tensors against the fp64 oracle.
FP32_ENV_X = 10.0
FP32_FLOOR = 1e-4


def fp32_gate(env):
    return max(FP32_FLOOR, FP32_ENV_X * float(env))


@pytest.mark.gpu
def test_segmentor_fp32_vs_oracle_full():
    """Full tensors (not fingerprints) of the fp32 HIP path against the fp64 oracle restatement on
    e2e_tiny_small: the encoder features and their gradients, the logits and their gradient, the
    image / depth gradients and every parameter gradient, each rel-to-max <= 1e-4 (measured on
    MI355X: <= 8.3e-6; the reference's own fp32 error on this case is 1-2e-6)."""
    errs = fp32_audit("e2e_tiny_small", "DFormer-Tiny", "ham", 40)
    bad = {k: v for k, v in errs.items() if v > 1e-4}
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1])[:10]


def fp32_audit(name, arch, dec, ncls):
    """{quantity: rel-to-max error} of the fp32 HIP path vs the fp64 oracle on a golden case."""
    g = load(name)
    B, H, W, _ = [int(v) for v in g["meta"][:4]]
    rgb_np, dep_np = gen.rgb_depth(B, H, W, seed=input_seed(g))
    lab_np = gen.labels(B, H, W, ncls)
    bases = gen.nmf_bases(B, 512, 64, name=name + "/bases") if dec == "ham" else None
    model = build(arch, dec, ncls, "cuda")
    model.train()
    if dec == "ham":
        model.decode_head.hamburger.ham.injected_bases = torch.from_numpy(bases).float()
    rgb = torch.from_numpy(rgb_np).float().cuda().requires_grad_()
    dep = torch.from_numpy(dep_np).float().cuda().requires_grad_()
    feats = model.encoder_backbone(rgb, dep)[0]
    for f in feats:
        f.retain_grad()
    low = model.decode_head(feats)
    low.retain_grad()
    from dformer_amd.decoders import SegLossFn, _nhwc_rows
    rows, (b, h, w) = _nhwc_rows(low)
    loss = SegLossFn.apply(rows.contiguous(), b, h, w, torch.from_numpy(lab_np).cuda(), 255)
    loss.backward()
    torch.cuda.synchronize()
    p = params(R.segmentor_shapes(arch, dec, ncls), torch.float64)
    rgb64 = torch.from_numpy(rgb_np).double().requires_grad_()
    dep64 = torch.from_numpy(dep_np).double().requires_grad_()
    rfeats, rlow, rloss = R.segmentor_forward(p, arch, dec, rgb64, dep64,
                                              torch.from_numpy(bases).double() if bases is not None else None,
                                              True, torch.from_numpy(lab_np).long())
    for f in rfeats:
        f.retain_grad()
    rlow.retain_grad()
    rloss.backward()

    def e(a, b_):
        return rel_err(a.detach().float().cpu().double(), b_.detach())

    out = {"loss": abs(loss.item() - rloss.item()) / abs(rloss.item()), "low": e(low, rlow),
           "low.grad": e(low.grad, rlow.grad), "rgb.grad": e(rgb.grad, rgb64.grad),
           "depth.grad": e(dep.grad, dep64.grad)}
    for i, (f, rf) in enumerate(zip(feats, rfeats)):
        out[f"feat{i}"] = e(f, rf)
        out[f"feat{i}.grad"] = e(f.grad, rf.grad)
    named = dict(model.named_parameters())
    for k, v in p.items():
        if k in named and v.grad is not None and named[k].grad is not None and v.grad.abs().max() > 1e-12:
            out["grad/" + k] = e(named[k].grad, v.grad)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("train", [True, False])
def test_nmf2d_vs_reference(train):
    from dformer_amd.decoders import NMF2D
    name = "nmf_train" if train else "nmf_eval"
    g = load(name)
    B, C, H, W, _ = [int(v) for v in g["meta"]]
    nmf = NMF2D()
    nmf.train(train)
    nmf.injected_bases = torch.from_numpy(gen.nmf_bases(B, C, 64, name=name + "/bases")).float()
    x = torch.from_numpy(gen.uniform(name + "/x", (B, C, H, W))).float().cuda()
    xr = x.permute(0, 2, 3, 1).contiguous().view(B * H * W, C).requires_grad_()
    y = nmf.fused(xr, B, H * W)
    gy = torch.from_numpy(gen.normal(name + "/gy", (B, C, H, W))).float().cuda()
    y.backward(gy.permute(0, 2, 3, 1).reshape(B * H * W, C))
    yy = y.detach().view(B, H, W, C).permute(0, 3, 1, 2).cpu()
    assert rel_err(yy, g["y"]) < 1e-4
    gx = xr.grad.view(B, H, W, C).permute(0, 3, 1, 2).cpu()
    assert rel_err(gx, g["gx"]) < 1e-3


@pytest.mark.gpu
def test_ham_head_vs_reference():
    """LightHamHead fwd + bwd vs the reference (fp64 golden) at 1e-3. The golden's inputs were drawn
    (oracle/make_goldens.py golden_ham) so that every ReLU input is >= 1e-5 x max away from the
    kink: the fp32 HIP path then takes the same activation pattern as fp64 everywhere."""
    from dformer_amd.decoders import LightHamHead
    name = "ham_tiny"
    g = load(name)
    B, H, W, ncls, train, seed, *in_ch = [int(v) for v in g["meta"]]
    tag = f"{name}#{seed}"
    head = LightHamHead(in_channels=in_ch, num_classes=ncls, channels=512, norm_cfg=dict(type="BN"))
    head.dropout_ratio = 0.0
    sd = head.state_dict()
    vals = gen.state_dict_values([(k, v.shape) for k, v in sd.items()])
    head.load_state_dict({k: torch.from_numpy(np.asarray(v)).to(sd[k].dtype) for k, v in vals.items()})
    head = head.cuda().train()
    from dformer_amd.functional import invalidate_weights
    invalidate_weights()
    head.hamburger.ham.injected_bases = torch.from_numpy(gen.nmf_bases(B, 512, 64, name=tag + "/bases")).float()
    feats = [torch.from_numpy(gen.normal(tag + f"/f{i}", (B, c, H >> i, W >> i))).float().cuda()
             for i, c in enumerate(in_ch)]
    leaves = [f.permute(0, 2, 3, 1).contiguous().requires_grad_() for f in feats]
    y = head([None] + [t.permute(0, 3, 1, 2) for t in leaves])
    gy = torch.from_numpy(gen.normal(tag + "/gy", tuple(y.shape))).float().cuda()
    y.backward(gy)
    assert rel_err(y.detach().cpu(), g["y"]) < 1e-3
    for i, t in enumerate(leaves):
        assert rel_err(t.grad.permute(0, 3, 1, 2).cpu(), g[f"gf{i + 1}"]) < 1e-3, i
    grads = {k: p.grad.cpu() for k, p in head.named_parameters() if p.grad is not None}
    check_param_grads(g, grads, 1e-3, atol=1e-6)
    for k, v in g.items():
        if k.startswith("buf/"):
            assert rel_err(dict(head.named_buffers())[k[4:]].cpu(), v) < 1e-4


@pytest.mark.gpu
def test_mlp_decoder_vs_reference():
    from dformer_amd.decoders import DecoderHead
    from dformer_amd.functional import invalidate_weights
    name = "mlpdec_small"
    g = load(name)
    B, H, W, ncls, embed, *in_ch = [int(v) for v in g["meta"]]
    head = DecoderHead(in_channels=in_ch, num_classes=ncls, embed_dim=embed)
    head.dropout_ratio = 0.0
    sd = head.state_dict()
    vals = gen.state_dict_values([(k, v.shape) for k, v in sd.items()])
    head.load_state_dict({k: torch.from_numpy(np.asarray(v)).to(sd[k].dtype) for k, v in vals.items()})
    head = head.cuda().train()
    invalidate_weights()
    sizes = [(H, W)]
    for _ in range(3):
        sizes.append(((sizes[-1][0] - 1) // 2 + 1, (sizes[-1][1] - 1) // 2 + 1))
    leaves = [torch.from_numpy(gen.normal(name + f"/f{i}", (B, c, *sizes[i]))).float().cuda()
              .permute(0, 2, 3, 1).contiguous().requires_grad_() for i, c in enumerate(in_ch)]
    y = head([t.permute(0, 3, 1, 2) for t in leaves])
    gy = torch.from_numpy(gen.normal(name + "/gy", tuple(y.shape))).float().cuda()
    y.backward(gy)
    assert rel_err(y.detach().cpu(), g["y"]) < 1e-3
    for i, t in enumerate(leaves):
        assert rel_err(t.grad.permute(0, 3, 1, 2).cpu(), g[f"gf{i}"]) < 1e-3
    grads = {k: p.grad.cpu() for k, p in head.named_parameters() if p.grad is not None}
    check_param_grads(g, grads, 2e-3, atol=1e-6)


@pytest.mark.gpu
def test_train_step_bf16_runs_and_decreases_loss():
    """Tiny bf16 training steps through FusedAdamW: finite loss that drops on a fixed batch."""
    from dformer_amd.train import FusedAdamW, train_step
    torch.manual_seed(0)
    model = build("DFormer-Tiny", "ham", 40, "cuda").set_compute_dtype(torch.bfloat16)
    model.return_logits = False
    model.train()
    opt = FusedAdamW(model, lr=1e-3, compute_dtype=torch.bfloat16)
    rgb = torch.randn(2, 3, 96, 128, device="cuda")
    dep = torch.randn(2, 1, 96, 128, device="cuda")
    lab = torch.randint(0, 40, (2, 96, 128), device="cuda")
    losses = [train_step(model, opt, rgb, dep, lab).item() for _ in range(8)]
    assert all(np.isfinite(losses)), losses
    assert losses[-1] < losses[0], losses


@pytest.mark.gpu
def test_tiny_full_480x640_fp32_vs_reference():
    """BASELINE config 1 shape on the HIP path: DFormer-Tiny + ham forward at 2x3x480x640 (+ depth),
    fp32, against the reference's fp64 fingerprints (sum, abs-sum, l2, 64 strided samples) of the
    four encoder maps, the 1/8 logits and the full-resolution upsampled logits, gate 1e-3."""
    name = "e2e_tiny_full_fwd"
    g = load(name)
    B, H, W, ncls = [int(v) for v in g["meta"][:4]]
    model = build("DFormer-Tiny", "ham", ncls, "cuda").train()
    model.decode_head.hamburger.ham.injected_bases = torch.from_numpy(
        gen.nmf_bases(B, 512, 64, name=name + "/bases")).float()
    rgb_np, dep_np = gen.rgb_depth(B, H, W, seed=input_seed(g))
    rgb = torch.from_numpy(rgb_np).float().cuda()
    dep = torch.from_numpy(dep_np).float().cuda()
    with torch.no_grad():
        feats = model.encoder_backbone(rgb, dep)[0]
        low = model.decode_head(feats)
        out = model._upsample(low, (H, W))
    torch.cuda.synchronize()
    errs = {f"feat{i}": fp_rel_err(gen.fingerprint(f.double().cpu().numpy()), g[f"feat{i}_fp"])
            for i, f in enumerate(feats)}
    errs["low"] = fp_rel_err(gen.fingerprint(low.double().cpu().numpy()), g["low_fp"])
    errs["out"] = fp_rel_err(gen.fingerprint(out.double().cpu().numpy()), g["out_fp"])
    assert max(errs.values()) < 1e-3, errs


# bf16 end-to-end gates, relative to the reference's OWN bf16 autocast error on the same golden
# (tests/golden/bf16env_*.npz, oracle/make_goldens.py golden_bf16_env; SURVEY §8c: the reference's
# autocast misses a flat 1e-2 logits gate by itself — 1.0-2.1e-2 on these goldens and 2.2e-2 on the
# SURVEY's Tiny probe — and lands at a median 2-7e-2 on the parameter-gradient fingerprints).
# bf16 end-to-end error is chaotic in the accumulation order: on MI355X the same model run with the
# fused ConvFFN vs the split-K GEMM path moves the logits error by 0.7-1.4x and single-parameter
# gradient errors by up to 2x, both paths pinned at 1e-3 in fp32. The gates are therefore the
# reference's own envelope with that spread as margin:
SURVEY_BF16_LOGITS = 2.2e-2
BF16_LOW = 1.5      # logits rel-to-max <= 1.5 x max(reference autocast on this golden, SURVEY's 2.2e-2)
BF16_LOSS = 1e-3    # |loss - golden| / golden  (the reference's own is ~1e-5)
BF16_GRAD_Q = 1.5   # the distribution over parameters of the gradient-fingerprint error: its median,
                    # 90th percentile and max each <= 1.5 x the reference autocast's (single
                    # parameters are too noisy to gate one by one: the reference's own max is 2.4-6.6)


@pytest.mark.gpu
@pytest.mark.parametrize("name,arch,dec,ncls", E2E)
def test_segmentor_bf16_vs_reference_envelope(name, arch, dec, ncls):
    g = load(name)
    env = load("bf16env_" + name)
    B, H, W, _ = [int(v) for v in g["meta"][:4]]
    model = build(arch, dec, ncls, "cuda").set_compute_dtype(torch.bfloat16)
    model.train()
    if dec == "ham":
        model.decode_head.hamburger.ham.injected_bases = torch.from_numpy(
            gen.nmf_bases(B, 512, 64, name=name + "/bases")).float()
    rgb_np, dep_np = gen.rgb_depth(B, H, W, seed=input_seed(g))
    rgb = torch.from_numpy(rgb_np).float().cuda().requires_grad_()
    dep = torch.from_numpy(dep_np).float().cuda().requires_grad_()
    lab = torch.from_numpy(gen.labels(B, H, W, ncls)).cuda()
    feats = model.encoder_backbone(rgb, dep)[0]
    low = model.decode_head(feats)
    from dformer_amd.decoders import SegLossFn, _nhwc_rows
    rows, (b, h, w) = _nhwc_rows(low)
    loss = SegLossFn.apply(rows.contiguous(), b, h, w, lab, 255)
    loss.backward()
    torch.cuda.synchronize()
    e_low = rel_err(low.float().cpu(), g["low"])
    assert e_low <= BF16_LOW * max(float(env["env/low"]), SURVEY_BF16_LOGITS), (e_low, float(env["env/low"]))
    assert abs(loss.item() - float(g["loss"])) <= BF16_LOSS * abs(float(g["loss"]))
    params = dict(model.named_parameters())
    ours, refs = [], []
    for k, v in g.items():
        if not k.startswith("gfp/"):
            continue
        ours.append(fp_rel_err(gen.fingerprint(params[k[4:]].grad.double().cpu().numpy(), 16), v, atol=1e-4))
        refs.append(float(env["env/" + k]))
    for q in (50, 90, 100):
        a, r = np.percentile(ours, q), np.percentile(refs, q)
        assert a <= BF16_GRAD_Q * r, (q, a, r)


@pytest.mark.gpu
def test_syncbn_two_half_batches_equal_full_batch():
    """SyncBN statistics as the DP path forms them: the library's shifted (sum, sumsq, shift) of two
    half-batches, merged on the device (K.bn_merge), finalize to the full batch's mean / var; a single
    shard merges to itself bit for bit (what a one-rank SyncBN group relies on)."""
    from dformer_amd import kernels as K
    torch.manual_seed(0)
    x = (torch.randn(60000, 128, device="cuda") * 0.7 + torch.linspace(-20, 40, 128, device="cuda"))
    halves = [x[:26000], x[26000:]]
    parts = torch.stack([K.bn_stats(h) for h in halves])
    st = K.bn_merge(parts, torch.tensor([26000.0, 34000.0], device="cuda"))
    assert torch.equal(K.bn_merge(parts[:1], torch.tensor([26000.0], device="cuda")), parts[0])
    rm, rv = torch.zeros(128, device="cuda"), torch.ones(128, device="cuda")
    mean, rstd = K.bn_finalize(st, 60000, 1e-5, 0.1, rm, rv)
    full_mean, full_rstd = K.bn_finalize(K.bn_stats(x), 60000, 1e-5, 0.1)
    xd = x.double()
    assert rel_err(mean.cpu(), xd.mean(0).cpu()) < 1e-6
    assert rel_err(mean.cpu(), full_mean.cpu()) < 1e-6
    assert rel_err(rstd.cpu(), full_rstd.cpu()) < 1e-4
    assert rel_err((1 / rstd.double() ** 2 - 1e-5).cpu(), xd.var(0, unbiased=False).cpu()) < 1e-4
    assert rel_err(rv.cpu(), (0.9 + 0.1 * xd.var(0, unbiased=True)).cpu()) < 1e-4
