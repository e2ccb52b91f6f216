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
    # every kernel of the step is a libdformer_hip kernel with fixed-order reductions (no vendor
    # convolutions since round 3), so the step is run-to-run reproducible and the graphed and eager
    # steps must agree bit for bit; the cudnn flags are pinned anyway for any torch op
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


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_forced_collectives_one_rank_nccl():
    """The world > 1 code on the GPU with one rank: a 1-rank RCCL group and decoders.FORCE_COLLECTIVES
    send every SyncBN statistic through all_gather_into_tensor + the device merge, every BN backward
    statistic, gradient bucket and the loss through all_reduce. A Tiny + ham step run that way eagerly
    and as a captured GraphedTrainStep must agree bit for bit, and both with the plain world-1 path
    (a one-rank sum and a one-shard merge are exact identities). utils/train.py:238-243,
    utils/engine/engine.py:53-66 (the reference's DDP + SyncBN setup)."""
    import torch.distributed as dist
    import bench
    from dformer_amd import decoders as D
    from dformer_amd.segmentor import EncoderDecoder
    from dformer_amd.train import FusedAdamW, GraphedTrainStep, train_step
    dev = torch.device("cuda", 0)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    D.FORCE_COLLECTIVES = True
    try:
        cfg = bench.make_cfg("DFormer-Tiny", "ham")
        cfg["drop_path_rate"] = 0.0
        models = []
        for sync in (True, True, False):
            torch.manual_seed(3)
            m = EncoderDecoder(cfg=cfg, syncbn=sync)
            m.decode_head.dropout_ratio = 0.0
            models.append(m.to(dev).set_compute_dtype(torch.bfloat16))
        ma, mb, mc = models
        assert sum(isinstance(x, torch.nn.SyncBatchNorm) for x in ma.modules()) > 0
        assert not any(isinstance(x, torch.nn.SyncBatchNorm) for x in mc.modules())
        g = torch.Generator(device=dev)
        g.manual_seed(11)
        bases = torch.rand(2, 512, 64, device=dev, generator=g)
        bases = bases / bases.norm(dim=1, keepdim=True)
        opts = []
        for m in models:
            m.decode_head.hamburger.ham.injected_bases = bases
            m.return_logits = False
            m.train()
            opts.append(FusedAdamW(m, lr=1e-3, weight_decay=cfg.weight_decay, world=1, compute_dtype=torch.bfloat16))
        oa, ob, oc = opts
        rgb, dep, lab = bench.synthetic_batch(2, 240, 320, cfg.num_classes, dev, 5)
        calls = {"all_reduce": 0, "all_gather_into_tensor": 0}
        real = {k: getattr(dist, k) for k in calls}

        def counting(name):
            def f(*a, **k):
                calls[name] += 1
                return real[name](*a, **k)
            return f
        for k in calls:
            setattr(dist, k, counting(k))
        try:
            la = [train_step(ma, oa, rgb, dep, lab).item() for _ in range(5)]
        finally:
            for k, f in real.items():
                setattr(dist, k, f)
        assert calls["all_reduce"] > 0 and calls["all_gather_into_tensor"] > 0, calls
        gstep = GraphedTrainStep(mb, ob, rgb, dep, lab, warmup=2)
        lb = [gstep().item() for _ in range(3)]
        D.FORCE_COLLECTIVES = False
        lc = [train_step(mc, oc, rgb, dep, lab).item() for _ in range(5)]
        assert la[2:] == lb, (la, lb)
        assert la == lc, (la, lc)
        for ga, gb, gc in zip(oa.groups, ob.groups, oc.groups):
            assert torch.equal(ga.flat, gb.flat) and torch.equal(ga.m, gb.m) and torch.equal(ga.v, gb.v)
            assert torch.equal(ga.flat, gc.flat) and torch.equal(ga.v, gc.v)
        for (ka, ba), (kc, bc) in zip(ma.state_dict().items(), mc.state_dict().items()):
            assert ka == kc and torch.equal(ba, bc), ka
    except BaseException as e:  # report before the process-group teardown (which may abort on failure)
        print("forced-collectives failure:", repr(e)[:2000], flush=True)
        import traceback
        traceback.print_exc()
        sys.stdout.flush()
        sys.stderr.flush()
        raise
    finally:
        D.FORCE_COLLECTIVES = False
        D._GLOBAL_ROWS.clear()
        D._GLOBAL_TOTAL.clear()
        dist.destroy_process_group()
