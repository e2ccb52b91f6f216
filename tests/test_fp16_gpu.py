"""fp16 compute path (BASELINE config 5: DFormer-Large + MLPDecoder trained under the reference's
torch.autocast(float16) + GradScaler, utils/train.py:288-289, 323-337) on the HIP kernels:
fp16 storage, fp32 accumulation / LN / BN / softmax statistics, dynamic loss scaling.

Gates: per Block vs the fp64 reference goldens at Large's stage geometries (incl. the 530x730
run's 34x46 stage-2 and 17x23 stage-3 planes); end to end vs the reference's OWN fp16 autocast
error on the same golden (tests/golden/f16env_*.npz, oracle/make_goldens.py golden_bf16_env with
dtype=float16); the training step with the loss scaler."""
import numpy as np
import pytest
import torch

import gen
from goldens import fp_rel_err, load, rel_err, input_seed
from test_block_gpu import run_block
from test_segmentor_gpu import build

pytestmark = pytest.mark.gpu

# fp16 has 3 more mantissa bits than bf16: the per-Block gate is 8x tighter than bf16's 1e-2 / 2e-2
F16_BLOCK_FWD = 2e-3
F16_BLOCK_BWD = 4e-3


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")


@pytest.mark.parametrize("name", ["block_large_s1", "block_large_s2", "block_large_s2_34x46", "block_large_s3_17x23",
                                  "block_base_s0", "block_base_s2", "block_tiny_s3_last"])
def test_block_fp16_vs_reference_goldens(name):
    g, blk, x, xe, y, ye, last = run_block(name, torch.float16)
    assert y.dtype == torch.float16
    e = {"y": rel_err(y.float().cpu(), g["y"]), "gx": rel_err(x.grad.float().cpu(), g["gx"])}
    if not last:
        e["y_e"] = rel_err(ye.float().cpu(), g["y_e"])
        e["gxe"] = rel_err(xe.grad.float().cpu(), g["gxe"])
    assert e["y"] < F16_BLOCK_FWD and e.get("y_e", 0) < F16_BLOCK_FWD, e
    assert e["gx"] < F16_BLOCK_BWD and e.get("gxe", 0) < F16_BLOCK_BWD, e


F16_LOW = 1.5     # logits rel-to-max <= 1.5 x max(reference fp16 autocast on this golden, 2e-3)
F16_LOSS = 1e-3
F16_GRAD_Q = 1.5  # median / p90 / max of the parameter-gradient fingerprint errors vs the reference's


def test_segmentor_fp16_large_mlp_vs_reference_envelope():
    name, arch, dec, ncls = "e2e_large_mlp_small", "DFormer-Large", "MLPDecoder", 37
    g = load(name)
    env = load("f16env_" + name)
    B, H, W, _ = [int(v) for v in g["meta"][:4]]
    model = build(arch, dec, ncls, "cuda").set_compute_dtype(torch.float16)
    model.train()
    rgb_np, dep_np = gen.rgb_depth(B, H, W, seed=input_seed(g))
    rgb = torch.from_numpy(rgb_np).float().cuda().requires_grad_()
    dep = torch.from_numpy(dep_np).float().cuda().requires_grad_()
    lab = torch.from_numpy(gen.labels(B, H, W, ncls)).cuda()
    feats = model.encoder_backbone(rgb, dep)[0]
    assert feats[2].dtype == torch.float16
    low = model.decode_head(feats)
    from dformer_amd.decoders import SegLossFn, _nhwc_rows
    rows, (b, h, w) = _nhwc_rows(low)
    loss = SegLossFn.apply(rows.contiguous(), b, h, w, lab, 255)
    loss.backward()
    torch.cuda.synchronize()
    e_low = rel_err(low.float().cpu(), g["low"])
    assert e_low <= F16_LOW * max(float(env["env/low"]), 2e-3), (e_low, float(env["env/low"]))
    assert abs(loss.item() - float(g["loss"])) <= F16_LOSS * abs(float(g["loss"]))
    params = dict(model.named_parameters())
    ours, refs = [], []
    for k, v in g.items():
        if not k.startswith("gfp/"):
            continue
        ours.append(fp_rel_err(gen.fingerprint(params[k[4:]].grad.double().cpu().numpy(), 16), v, atol=1e-4))
        refs.append(float(env["env/" + k]))
    for q in (50, 90, 100):
        a, r = np.percentile(ours, q), np.percentile(refs, q)
        assert a <= F16_GRAD_Q * max(r, 1e-3), (q, a, r)


class Cfg(dict):
    __getattr__ = dict.__getitem__


def _tiny_fp16_trainer(dpr=0.1):
    from dformer_amd.segmentor import EncoderDecoder
    from dformer_amd.train import FusedAdamW
    torch.manual_seed(0)
    cfg = Cfg(backbone="DFormer-Tiny", decoder="MLPDecoder", decoder_embed_dim=64, num_classes=13,
              drop_path_rate=dpr, bn_eps=1e-3, bn_momentum=0.1, background=255)
    model = EncoderDecoder(cfg=cfg).cuda().set_compute_dtype(torch.float16)
    model.return_logits = False
    model.train()
    opt = FusedAdamW(model, lr=2e-4, weight_decay=0.01, compute_dtype=torch.float16)
    rgb = torch.randn(2, 3, 96, 128, device="cuda")
    dep = torch.randn(2, 1, 96, 128, device="cuda")
    lab = torch.randint(0, 13, (2, 96, 128), device="cuda")
    return model, opt, rgb, dep, lab


def test_fp16_train_step_with_loss_scaler():
    from dformer_amd.train import train_step
    model, opt, rgb, dep, lab = _tiny_fp16_trainer()
    assert opt.scaler is not None and opt.scaler.scale == 2.0 ** 16
    assert opt.groups[0].shadow.dtype == torch.float16
    losses = [float(train_step(model, opt, rgb, dep, lab)) for _ in range(10)]
    assert all(np.isfinite(losses)), losses
    assert opt.step_count + opt.scaler.skipped == 10
    assert losses[-1] < losses[0], losses


def test_loss_scaler_skips_overflowing_step():
    """An inf gradient skips the update (parameters, moments and step count untouched) and halves
    the scale, like GradScaler.step / update."""
    from dformer_amd.train import train_step
    model, opt, rgb, dep, lab = _tiny_fp16_trainer()
    train_step(model, opt, rgb, dep, lab)
    steps, scale = opt.step_count, opt.scaler.scale
    flat0 = [g.flat.clone() for g in opt.groups]
    m0 = [g.m.clone() for g in opt.groups]
    loss, _ = model(rgb, dep, lab)
    loss.backward(torch.full_like(loss, opt.scaler.scale))
    opt.groups[0].grad[123] = float("inf")
    opt.step()
    assert opt.step_count == steps and opt.scaler.scale == scale / 2
    for g, f, m in zip(opt.groups, flat0, m0):
        assert torch.equal(g.flat, f) and torch.equal(g.m, m)
    train_step(model, opt, rgb, dep, lab)
    assert opt.step_count == steps + 1


def test_fp16_graphed_step_matches_eager():
    """The fp16 loss scaler is decided on the device, so the fp16 step captures into a HIP graph:
    graphed and eager steps agree bit for bit, including a step skipped on overflow (the scale halves
    and the applied-step count holds, GradScaler semantics, utils/train.py:323-338)."""
    from dformer_amd.train import GraphedTrainStep, train_step
    det, bm = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        ma, oa, rgb, dep, lab = _tiny_fp16_trainer(dpr=0.0)  # no RNG: identical math eager / graphed
        mb, ob, _, _, _ = _tiny_fp16_trainer(dpr=0.0)
        for m in (ma, mb):
            m.decode_head.dropout_ratio = 0.0
        la = [train_step(ma, oa, rgb, dep, lab).item() for _ in range(5)]
        g = GraphedTrainStep(mb, ob, rgb, dep, lab, warmup=2)
        lb = [g().item() for _ in range(3)]
        assert la[2:] == lb, (la, lb)
        assert oa.step_count == ob.step_count and oa.scaler.scale == ob.scaler.scale
        for ga, gb in zip(oa.groups, ob.groups):
            assert torch.equal(ga.flat, gb.flat) and torch.equal(ga.m, gb.m) and torch.equal(ga.v, gb.v)
        # an overflow inside a replay: the scale is forced so large that the fp16 backward overflows
        steps, scale = ob.step_count, ob.scaler.scale
        flat0 = [gr.flat.clone() for gr in ob.groups]
        ob.scaler.state[0] = 2.0 ** 127
        g()
        torch.cuda.synchronize()
        assert ob.step_count == steps and ob.scaler.scale == 2.0 ** 126 and ob.scaler.skipped >= 1
        for f, gr in zip(flat0, ob.groups):
            assert torch.equal(f, gr.flat)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det, bm


def test_loss_scale_update_kernel_schedule():
    """dfm_loss_scale_update follows GradScaler.update: x0.5 on overflow, x2 after 2000 clean steps,
    applied steps counted only when clean, the flag cleared every call."""
    from dformer_amd import kernels as K
    amp = torch.tensor([65536.0, 0.0, 0.0, 0.0], device="cuda")
    flag = torch.ones(1, device="cuda", dtype=torch.int32)
    K.loss_scale_update(amp, flag, 2.0, 0.5, 2000)
    assert amp.tolist() == [32768.0, 0.0, 0.0, 1.0] and flag.item() == 0
    for _ in range(1999):
        K.loss_scale_update(amp, flag, 2.0, 0.5, 2000)
    assert amp.tolist() == [32768.0, 1999.0, 1999.0, 1.0]
    K.loss_scale_update(amp, flag, 2.0, 0.5, 2000)
    assert amp.tolist() == [65536.0, 0.0, 2000.0, 1.0]
