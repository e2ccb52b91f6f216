"""A/B of the ConvFFN (LN -> fc1 -> DW3x3 + id -> GELU -> fc2 -> residual) as the fused kernels vs
the separate kernels, forward and forward+backward, at every DFormer-B ConvFFN shape (bf16, bs 16,
480x640). Prints ms per call, measured with HIP events."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dformer_amd import functional as Fn  # noqa: E402

SHAPES = [("s0 main", 120, 160, 64, 8), ("s0 e2", 120, 160, 32, 8), ("s1 main", 60, 80, 128, 8),
          ("s1 e2", 60, 80, 64, 8), ("s2 main", 30, 40, 256, 4), ("s2 e2", 30, 40, 128, 4),
          ("s3 main", 15, 20, 512, 4), ("s3 e2", 15, 20, 256, 4)]
B = 16
dev, dt = "cuda", torch.bfloat16
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10


def run(fused, shape):
    _, H, W, C, r = shape
    hid = r * C
    torch.manual_seed(0)
    p = [1 + 0.1 * torch.randn(C, device=dev), 0.1 * torch.randn(C, device=dev),
         torch.randn(hid, C, device=dev) / C ** 0.5, 0.1 * torch.randn(hid, device=dev),
         torch.randn(hid, 1, 3, 3, device=dev) / 3, 0.1 * torch.randn(hid, device=dev),
         torch.randn(C, hid, device=dev) / hid ** 0.5, 0.1 * torch.randn(C, device=dev), torch.rand(C, device=dev)]
    p = [t.requires_grad_() for t in p]
    x = torch.randn(B * H * W, C, device=dev).to(dt).requires_grad_()
    gy = torch.randn(B * H * W, C, device=dev).to(dt)
    Fn.FUSED_FFN = fused
    Fn.invalidate_weights()

    def fwd():
        return Fn.ConvFFNFn.apply(x, (B, H, W), None, *p)

    def step():
        fwd().backward(gy)

    out = {}
    for name, fn in (("fwd", fwd), ("fwd+bwd", step)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name] = e0.elapsed_time(e1) / iters
    return out


for sh in SHAPES:
    a, b = run(False, sh), run(True, sh)
    print(f"{sh[0]:8s} C={sh[3]:3d}  unfused fwd {a['fwd']:.3f} f+b {a['fwd+bwd']:.3f} ms | fused fwd {b['fwd']:.3f} "
          f"f+b {b['fwd+bwd']:.3f} ms", flush=True)
