"""Micro-benchmark of the fused ConvFFN kernels at a DFormer-B stage shape (bf16), timed with HIP
events; also the target of rocprofv3 PMC passes (tools/ffn_bench.py [stage] [iters])."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dformer_amd import kernels as K  # noqa: E402

STAGES = {0: (16, 120, 160, 64, 8), 1: (16, 60, 80, 64, 8), 2: (16, 30, 40, 64, 8), 3: (16, 120, 160, 32, 8)}
st = int(sys.argv[1]) if len(sys.argv) > 1 else 0
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
B, H, W, C, r = STAGES[st]
hid = r * C
dt = torch.bfloat16
dev = "cuda"
P = B * H * W
xn = torch.randn(P, C, device=dev).to(dt)
x = torch.randn(P, C, device=dev).to(dt)
w1 = (torch.randn(hid, C, device=dev) / C ** 0.5).to(dt)
w2 = (torch.randn(C, hid, device=dev) / hid ** 0.5).to(dt)
b1, bpos, b2 = (0.1 * torch.randn(n, device=dev) for n in (hid, hid, C))
wpos = torch.randn(hid, 1, 3, 3, device=dev) / 3
ls = torch.rand(C, device=dev)
df = torch.randn(P, C, device=dev).to(dt)


def fwd():
    return K.convffn_fwd(xn, x, (B, H, W), w1, b1, wpos, bpos, w2, b2, ls)


def bwd():
    return K.convffn_bwd(xn, df, (B, H, W), w1, b1, wpos, bpos, w2)


for name, fn in (("fwd", fwd), ("bwd", bwd)):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    flops = (4 if name == "fwd" else 6) * P * C * hid
    print(f"stage{st} {name} B={B} H={H} W={W} C={C} hid={hid}: {us:.1f} us  ({flops / us / 1e6:.1f} TFLOP/s, "
          f"{P * hid / us / 1e3:.2f} Gelem/ms hidden)", flush=True)
