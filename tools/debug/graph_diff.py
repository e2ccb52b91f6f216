"""Which parameters differ between eager steps and GraphedTrainStep replays (debug tool, GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))

import bench  # noqa: E402
from test_graph_gpu import _build  # noqa: E402
from dformer_amd.train import FusedAdamW, GraphedTrainStep, train_step  # noqa: E402

dec = sys.argv[1] if len(sys.argv) > 1 else "ham"
if os.environ.get("DET") == "1":
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
nrep = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
cfg, ma = _build(dec)
_, mb = _build(dec)
ma = ma.to(dev).set_compute_dtype(torch.bfloat16)
mb = mb.to(dev).set_compute_dtype(torch.bfloat16)
if dec == "ham":
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
la = [train_step(ma, oa, rgb, dep, lab).item() for _ in range(2 + nrep)]
mode = sys.argv[3] if len(sys.argv) > 3 else "side"
if mode == "side":
    gs = GraphedTrainStep(mb, ob, rgb, dep, lab, warmup=2)
    lb = [gs().item() for _ in range(nrep)]
elif mode == "main":  # warm-up eagerly on the current stream, capture without side-stream warm-up
    for _ in range(2):
        train_step(mb, ob, rgb, dep, lab)
    gs = GraphedTrainStep(mb, ob, rgb, dep, lab, warmup=0)
    lb = [gs().item() for _ in range(nrep)]
else:  # eager only, warm-up on a side stream (is the side-stream warm-up itself the culprit?)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        lb = [train_step(mb, ob, rgb, dep, lab).item() for _ in range(2 + nrep)]
    torch.cuda.current_stream().wait_stream(side)
print("losses", la, lb)
names = {id(p): n for n, p in mb.named_parameters()}
namesa = {id(p): n for n, p in ma.named_parameters()}
rows = []
for ga, gb in zip(oa.groups, ob.groups):
    for (pa, (off, k)), (pb, _) in zip(ga.slots.items(), gb.slots.items()):
        d = (ga.flat[off:off + k] - gb.flat[off:off + k]).abs().max().item()
        s = ga.flat[off:off + k].abs().max().item()
        rows.append((d / max(s, 1e-12), d, namesa[id(pa)]))
rows.sort(reverse=True)
for r in rows[:15]:
    print("%.3e %.3e %s" % r)
