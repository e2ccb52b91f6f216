"""Two data-parallel ranks on the one GPU of the box (gloo over device tensors; RCCL refuses two ranks
on one device): the world > 1 code of config 4 — SyncBN statistics all-gathered and merged on the
device, BN backward statistics all-reduced for the input gradient, bucketed gradient all-reduce, the
loss all-reduce — against one rank training on the whole batch (utils/train.py:238-243 DDP +
SyncBatchNorm, utils/engine/engine.py:53-66).

With every label valid both ranks hold the same number of pixels, so DDP's average of the two
half-batch gradients is exactly the whole-batch gradient and SyncBN over the two ranks is BatchNorm
over the whole batch (the stems' plain BatchNorm2d layers, per-rank in the reference as well, run on
their running statistics): everything must agree to fp32 rounding (the step runs in float32).

Two sizes: DFormer-Tiny at 4 x 96 x 128, and BASELINE config 4's own model and image size,
DFormer-Base at 480 x 640 (2 ranks x 4 images against 1 rank x 8; config 4 runs 16 per GPU on 8 GPUs
over RCCL, which a one-GPU box cannot host: RCCL at N > 1 stays unmeasured here)."""
import os
import socket
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = {"tiny": ("DFormer-Tiny", 4, 96, 128), "base480": ("DFormer-Base", 8, 480, 640)}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(rank, world, case):
    """One train step of the case's model + ham on this rank's share of a fixed batch; returns the
    flat gradients divided by world (the buffers hold the SUM over ranks), the BN running statistics
    and the all-reduced loss."""
    import bench
    backbone, BATCH, H, W = CASES[case]
    from dformer_amd.segmentor import EncoderDecoder
    from dformer_amd.train import FusedAdamW, train_step
    dev = torch.device("cuda", 0)
    cfg = bench.make_cfg(backbone, "ham")
    cfg["drop_path_rate"] = 0.0
    torch.manual_seed(3)
    model = EncoderDecoder(cfg=cfg, syncbn=world > 1)
    if case == "base480":
        # layer scales O(1) as in the goldens: at the 1e-6 init the gradients behind 20
        # Blocks' branches are ~1e-11, pure fp32 rounding noise, and no relative gate means anything
        g0 = torch.Generator().manual_seed(7)
        for n, p in model.named_parameters():
            if "layer_scale" in n:
                p.data.uniform_(0.5, 1.0, generator=g0)
    model.decode_head.dropout_ratio = 0.0
    model = model.to(dev).set_compute_dtype(torch.float32)
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    bases = torch.rand(BATCH, 512, 64, device=dev, generator=g)
    bases = bases / bases.norm(dim=1, keepdim=True)
    rgb, dep, lab = bench.synthetic_batch(BATCH, H, W, cfg.num_classes, dev, 5)
    lab[lab == 255] = 0  # equal valid-pixel counts per rank
    per = BATCH // world
    sl = slice(rank * per, (rank + 1) * per)
    model.decode_head.hamburger.ham.injected_bases = bases[sl].contiguous()
    model.return_logits = False
    model.train()
    # the stems' BatchNorm2d layers are per-rank BN in the reference too (DFormer.py:194-211 builds
    # them as nn.BatchNorm2d whatever norm_cfg says): frozen on running statistics here so the
    # two-rank step can equal the whole-batch step; every SyncBN layer stays in training mode
    bb = model.encoder_backbone
    frozen = [m for stem in (bb.downsample_layers[0], bb.downsample_layers_e[0]) for m in stem
              if isinstance(m, torch.nn.BatchNorm2d)]
    assert len(frozen) == 4 and any(isinstance(m, torch.nn.SyncBatchNorm) for m in model.modules()) == (world > 1)
    for m in frozen:
        m.eval()
    opt = FusedAdamW(model, lr=0.0, weight_decay=cfg.weight_decay, world=world, compute_dtype=torch.float32)
    loss = train_step(model, opt, rgb[sl].contiguous(), dep[sl].contiguous(), lab[sl].contiguous())
    torch.cuda.synchronize()
    grads = [(gr.grad / world).cpu() for gr in opt.groups]
    bn_grads = {}
    for name, m in model.named_modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm) and m.training:  # the synchronised layers
            for gr in opt.groups:
                if m.weight in gr.slots:
                    off, k = gr.slots[m.weight]
                    bn_grads[name] = (gr.grad[off:off + k] / world).cpu()
    running = {k: v.cpu() for k, v in model.state_dict().items() if "running" in k}
    return grads, bn_grads, running, float(loss)


def _worker(rank, world, port, q, case):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        grads, bn_grads, running, loss = _run(rank, world, case)
        # numpy copies travel by value: a torch CPU tensor would be shared through a file descriptor
        # that vanishes when this process exits before the parent unpickles it
        q.put((rank, ([g.numpy() for g in grads], {k: v.numpy() for k, v in bn_grads.items()},
                      {k: v.numpy() for k, v in running.items()}, loss), None))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.mark.timeout(900)
@pytest.mark.parametrize("case", ["tiny", "base480"])
def test_two_ranks_syncbn_ddp_equal_whole_batch(case):
    """The attention-backward side stream and the bucket hooks' join_streams are active (eager step)."""
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    import torch.multiprocessing as mp
    ref_grads, ref_bn, ref_run, ref_loss = _run(0, 1, case)
    torch.cuda.empty_cache()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, case)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (out, err)) for r, out, err in (q.get(timeout=400) for _ in procs))
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        assert res[r][1] is None, res[r][1]
    out = {r: ([torch.from_numpy(g) for g in v[0][0]], {k: torch.from_numpy(t) for k, t in v[0][1].items()},
               {k: torch.from_numpy(t) for k, t in v[0][2].items()}, v[0][3]) for r, v in res.items()}
    grads, bn_grads, running, loss = out[0]
    assert abs(loss - ref_loss) <= 1e-5 * abs(ref_loss), (loss, ref_loss)
    for a, b in zip(grads, ref_grads):
        assert _rel(a, b) < 1e-4, _rel(a, b)
    # the BN affine gradients are local statistics averaged by DDP, not all-reduced twice: a doubled
    # or a missing all-reduce is a relative error of 0.5-1.0 on a layer. The per-layer gate is 1e-2
    # because at 480 x 640 one SyncBN layer's dgamma sums dy * xhat over 153,600 rows with heavy
    # cancellation (|dgamma| ~1e-5 from O(1) terms) and the two-rank summation order differs: measured
    # 4e-4 .. 1.1e-3 (downsample_layers(_e).1.0), fp32 noise; the flat buffers above hold at 1e-4
    assert len(bn_grads) >= 4
    for k, v in bn_grads.items():
        assert _rel(v, ref_bn[k]) < 1e-2, (k, _rel(v, ref_bn[k]))
    for k, v in running.items():
        if v.dtype.is_floating_point:
            assert _rel(v, ref_run[k]) < 1e-5, (k, _rel(v, ref_run[k]))
    # both ranks hold identical all-reduced gradients
    for a, b in zip(out[1][0], grads):
        assert torch.equal(a, b)
