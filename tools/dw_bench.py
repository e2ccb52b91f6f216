"""Time the depthwise-conv kernels on the DFormer-B bs=16 480x640 shapes (GPU only).
Algorithmic bytes: fwd reads x, writes y (+ GELU out); bwd-data reads dy, writes dx; wgrad reads x and dy."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dformer_amd import kernels as K  # noqa: E402


def t(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


def main():
    dev = torch.device("cuda", 0)
    B = 16
    shapes = [(120, 160, 512, 3), (120, 160, 256, 3), (60, 80, 1024, 3), (60, 80, 512, 3), (30, 40, 1024, 3),
              (15, 20, 2048, 3), (120, 160, 64, 7), (120, 160, 32, 7), (60, 80, 128, 7), (60, 80, 64, 7),
              (30, 40, 256, 7), (15, 20, 512, 7)]
    tot = {}
    for H, W, C, k in shapes:
        P = B * H * W
        x = torch.randn(P, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(P, C, device=dev).to(torch.bfloat16)
        w = torch.randn(C, 1, k, k, device=dev) / k
        b = torch.randn(C, device=dev)
        y = torch.empty_like(x)
        g = torch.empty_like(x)
        ident = k == 3
        gl = g if k == 3 else None
        f = t(lambda: K.dwconv(x, (B, H, W), w, b, k, ident, out=y, gelu_out=gl))
        bd = t(lambda: K.dwconv_bwd_data(dy, (B, H, W), w, k, ident, dx=y))
        wg = t(lambda: K.dwconv_bwd_weight(x, dy, (B, H, W), k))
        nb = P * C * 2
        out = f"{H}x{W} C={C:5d} k={k}: fwd {f:7.1f}us ({nb * (3 if gl is not None else 2) / f / 1e3:5.0f} GB/s)  "
        out += f"bwd_data {bd:7.1f}us ({2 * nb / bd / 1e3:5.0f} GB/s)  wgrad {wg:7.1f}us ({2 * nb / wg / 1e3:5.0f} GB/s)"
        print(out, flush=True)


if __name__ == "__main__":
    main()
