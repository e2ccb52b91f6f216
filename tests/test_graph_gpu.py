"""The HIP-graph training step (train.GraphedTrainStep) replays exactly what the eager step does."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    # the library convolutions of the stem / downsample layers (MIOpen) pick deterministic
    # algorithms: every kernel of the step is then run-to-run reproducible and the graphed and
    # eager steps must agree bit for bit
    det, bm = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    yield
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det, bm


def _build(decoder):
    import bench
    from dformer_amd.segmentor import EncoderDecoder
    cfg = bench.make_cfg("DFormer-Tiny", decoder)
    cfg["drop_path_rate"] = 0.0
    torch.manual_seed(3)
    model = EncoderDecoder(cfg=cfg)
    model.decode_head.dropout_ratio = 0.0  # no RNG: eager and graphed runs see identical math
    return cfg, model


@pytest.mark.parametrize("decoder", ["ham", "MLPDecoder"])
def test_graphed_steps_match_eager(decoder):
    import bench
    from dformer_amd.train import FusedAdamW, GraphedTrainStep, train_step
    dev = torch.device("cuda", 0)
    cfg, ma = _build(decoder)   # same seed -> identical initial weights
    _, mb = _build(decoder)
    ma = ma.to(dev).set_compute_dtype(torch.bfloat16)
    mb = mb.to(dev).set_compute_dtype(torch.bfloat16)
    if decoder == "ham":  # NMF draws random bases every forward: pin them so both runs see the same
        g = torch.Generator(device=dev)
        g.manual_seed(11)
        bases = torch.rand(2, 512, 64, device=dev, generator=g)
        bases = bases / bases.norm(dim=1, keepdim=True)
        for m in (ma, mb):
            m.decode_head.hamburger.ham.injected_bases = bases
    for m in (ma, mb):
        m.return_logits = False
        m.train()
    oa = FusedAdamW(ma, lr=1e-3, weight_decay=cfg.weight_decay, compute_dtype=torch.bfloat16)
    ob = FusedAdamW(mb, lr=1e-3, weight_decay=cfg.weight_decay, compute_dtype=torch.bfloat16)
    rgb, dep, lab = bench.synthetic_batch(2, 240, 320, cfg.num_classes, dev, 5)
    # eager: 2 steps (the graph helper's warm-up) + 3 steps; graphed: warm-up 2 + capture + 3 replays
    la = [train_step(ma, oa, rgb, dep, lab).item() for _ in range(5)]
    g = GraphedTrainStep(mb, ob, rgb, dep, lab, warmup=2)
    lb = [g().item() for _ in range(3)]
    assert ob.step_count == oa.step_count == 5
    assert la[2:] == lb, (la, lb)
    for ga, gb in zip(oa.groups, ob.groups):
        assert torch.equal(ga.flat, gb.flat) and torch.equal(ga.m, gb.m) and torch.equal(ga.v, gb.v)
    # a new batch copied into the static inputs is what the next replay trains on
    rgb2, dep2, lab2 = bench.synthetic_batch(2, 240, 320, cfg.num_classes, dev, 6)
    la2 = train_step(ma, oa, rgb2, dep2, lab2).item()
    rgb.copy_(rgb2)
    dep.copy_(dep2)
    lab.copy_(lab2)
    lb2 = g().item()
    assert la2 == lb2, (la2, lb2)
    # lr and step are read on the device: a replay at lr = 0 leaves the weights untouched
    before = [gr.flat.clone() for gr in ob.groups]
    g(lr=0.0)
    torch.cuda.synchronize()
    for b0, gr in zip(before, ob.groups):
        assert torch.equal(b0, gr.flat)
