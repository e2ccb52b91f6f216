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
    from dformer_amd import decoders
    decoders.BN_PROBE = {}
    try:
        loss = train_step(model, opt, rgb[sl].contiguous(), dep[sl].contiguous(), lab[sl].contiguous())
        torch.cuda.synchronize()
        probe = decoders.BN_PROBE
    finally:
        decoders.BN_PROBE = None
    grads = [(gr.grad / world).cpu() for gr in opt.groups]
    bn_grads = {}
    for name, m in model.named_modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm) and m.training:  # the synchronised layers
            for gr in opt.groups:
                if m.weight in gr.slots:
                    off, k = gr.slots[m.weight]
                    # [dgamma, dbeta] of this rank (fp32, all-reduced sum / world) and its local float64
                    # sums [sum dy*xhat, sum dy, sum |dy*xhat|, sum |dy|] over the same rows
                    kb = gr.slots[m.bias][0]
                    bn_grads[name] = (torch.stack([gr.grad[off:off + k], gr.grad[kb:kb + k]]).cpu() / world,
                                      probe[id(m)].cpu())
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
        q.put((rank, ([g.numpy() for g in grads], {k: (v[0].numpy(), v[1].numpy()) for k, v in bn_grads.items()},
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
    out = {r: ([torch.from_numpy(g) for g in v[0][0]],
               {k: (torch.from_numpy(t[0]), torch.from_numpy(t[1])) for k, t in v[0][1].items()},
               {k: torch.from_numpy(t) for k, t in v[0][2].items()}, v[0][3]) for r, v in res.items()}
    grads, bn_grads, running, loss = out[0]
    assert abs(loss - ref_loss) <= 1e-5 * abs(ref_loss), (loss, ref_loss)
    for a, b in zip(grads, ref_grads):
        assert _rel(a, b) < 1e-4, _rel(a, b)
    # SyncBN affine gradients (dgamma = sum dy * xhat, dbeta = sum dy over the batch), gated on the
    # rounding scale of the sum: |a - b| / sum |terms| per channel (the float64 sums of bn_grad_stats'
    # probe over the very dy / x̂ each run reduced). A doubled or missing all-reduce is an error of
    # 0.5 - 1 of |dgamma|; at 480 x 640 |dgamma| ~1e-5 arises from O(1) terms with heavy cancellation,
    # so a plain relative gate measures upstream fp32 noise in dy, not this reduction.
    def nerr(a, b, scale):
        live = scale > 0
        assert torch.equal(a[~live].double(), b[~live].double())  # all-zero terms: both sums exactly 0
        return float(((a.double() - b.double()).abs()[live] / scale[live]).max()) if live.any() else 0.0

    assert len(bn_grads) >= 4
    worst = {}
    for k, (v, p2) in bn_grads.items():
        r1, p1 = ref_bn[k]
        p2 = p2 + out[1][1][k][1]  # the other rank's local float64 sums (the gradient buffers hold the rank sum)
        for j in range(2):  # 0: gamma (sum dy*xhat, scale sum |dy*xhat|), 1: beta (sum dy, scale sum |dy|)
            e1 = nerr(r1[j], p1[j], p1[2 + j])                   # 1 rank vs its own float64 sum
            e2 = nerr(v[j], p2[j] / 2, p2[2 + j] / 2)            # 2 ranks vs theirs
            e12 = nerr(v[j], r1[j], torch.maximum(p1[2 + j], p2[2 + j] / 2))  # 2 ranks vs 1 rank
            worst[(k, j)] = (e1, e2, e12)
            assert e1 < 1e-4 and e2 < 1e-4, (k, j, e1, e2)
            assert e12 < 1e-3, (k, j, e12)
        if case == "tiny":  # well conditioned at this size: the plain relative gate holds as well
            assert _rel(v[0], r1[0]) < 1e-4, (k, _rel(v[0], r1[0]))
    print("SyncBN affine gradients, worst normalised errors (1 rank vs fp64, 2 ranks vs fp64, 2 vs 1):",
          [max(w[i] for w in worst.values()) for i in range(3)])
    for k, v in running.items():
        if v.dtype.is_floating_point:
            assert _rel(v, ref_run[k]) < 1e-5, (k, _rel(v, ref_run[k]))
    # both ranks hold identical all-reduced gradients
    for a, b in zip(out[1][0], grads):
        assert torch.equal(a, b)
