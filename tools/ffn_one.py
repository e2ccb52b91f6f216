"""Run only the fused ConvFFN forward + backward at one DFormer-B bf16 bs16 stage shape, N times
(profiling target for rocprofv3 --pmc / --kernel-trace; GPU only).

    python tools/ffn_one.py [stage 0-3] [branch mlp|mlp_e2] [iters]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dformer_amd import kernels as K  # noqa: E402

STAGES = {0: (120, 160, 64, 8), 1: (60, 80, 128, 8), 2: (30, 40, 256, 4), 3: (15, 20, 512, 4)}


def main():
    st = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    br = sys.argv[2] if len(sys.argv) > 2 else "mlp"
    it = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    H, W, C, r = STAGES[st]
    if br == "mlp_e2":
        C //= 2
    B, hid, dev, bf = 16, r * C, torch.device("cuda", 0), torch.bfloat16
    P = B * H * W
    x = torch.randn(P, C, device=dev).to(bf)
    lnw, lnb = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    w1 = (torch.randn(hid, C, device=dev) / C ** 0.5).to(bf)
    b1 = torch.randn(hid, device=dev) * 0.1
    wpos = torch.randn(hid, 1, 3, 3, device=dev) / 3
    bpos = torch.randn(hid, device=dev) * 0.1
    w2 = (torch.randn(C, hid, device=dev) / hid ** 0.5).to(bf)
    b2 = torch.randn(C, device=dev) * 0.1
    ls, rs = torch.rand(C, device=dev), torch.rand(B, device=dev)
    dout = torch.randn(P, C, device=dev).to(bf)
    for _ in range(it):
        out, f, h, xn, mu, rstd = K.convffn_fwd(x, (B, H, W), lnw, lnb, w1, b1, wpos, bpos, w2, b2, ls, rs)
        K.convffn_bwd(dout, x, h, xn, f, mu, rstd, (B, H, W), lnw, lnb, w1, wpos, bpos, w2, ls, rs)
    torch.cuda.synchronize()
    print("ok", st, br, it)


if __name__ == "__main__":
    main()
