"""Isolated timing of the attention-side launches of one DFormer-B bf16 bs=16 Block at each stage's
geometry (profiling tool, GPU only): the 7x7 depthwise forward / input gradient / weight gradient,
the pooled MFMA attention forward + combine and backward + dQ reduce, pool7 / bilinear, LayerNorm
forward / backward and the layer-scale residual backward, against their algorithmic HBM bytes.

    python tools/attn_kernels_bench.py [stage ...] [--json out.json]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dformer_amd import kernels as K  # noqa: E402
from ffn_kernels_bench import HBM, timed  # noqa: E402

STAGES = {0: (120, 160, 64, 1), 1: (60, 80, 128, 2), 2: (30, 40, 256, 4), 3: (15, 20, 512, 8)}


def bench_stage(st):
    H, W, C, heads = STAGES[st]
    B = 16
    P = B * H * W
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    E = 2
    x = torch.randn(P, C, device=dev).to(bf)
    dy = torch.randn(P, C, device=dev).to(bf)
    w7 = torch.randn(C, 1, 7, 7, device=dev) / 7
    b7 = torch.randn(C, device=dev) * 0.1
    y = torch.empty_like(x)
    dx = torch.empty_like(x)
    lnw, lnb = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    xn, mu, rstd = K.layernorm(x, lnw, lnb)
    ls = torch.rand(C, device=dev)
    rows = [
        ("dw7_fwd", lambda: K.dwconv(x, (B, H, W), w7, b7, 7, out=y), P * C * E * 2),
        ("dw7_bwd_data", lambda: K.dwconv_bwd_data(dy, (B, H, W), w7, 7, dx=dx), P * C * E * 2),
        ("dw7_wgrad", lambda: K.dwconv_bwd_weight(x, dy, (B, H, W), 7), P * C * E * 2),
        ("dw7_bwd_fused", lambda: K.dwconv_bwd(x, dy, (B, H, W), w7, 7, dx=dx), P * C * E * 3),
        ("ln_fwd", lambda: K.layernorm(x, lnw, lnb, out=xn), P * C * E * 2),
        ("ln_bwd", lambda: K.layernorm_bwd(x, dy, lnw, mu, rstd, dx=dx), P * C * E * 3),
        ("residual_bwd", lambda: K.residual_bwd(dy, x, ls, None, H * W, df=dx), P * C * E * 3),
        ("pool7", lambda: K.pool7(xn, (B, H, W)), P * C * E),
    ]
    if st > 0:
        Ch = C // 2
        dh = Ch // heads
        m = torch.randn(B * 49, Ch, device=dev).to(bf)
        kv = torch.randn(P, C, device=dev).to(bf)
        o, lse = K.pooled_attn(m, kv[:, :Ch], kv[:, Ch:], B, heads, P // B, dh, dh ** -0.5)
        do = torch.randn_like(o)
        dm = torch.empty_like(m)
        dkv = torch.empty(P, C, device=dev, dtype=bf)
        rows += [
            ("attn_fwd", lambda: K.pooled_attn(m, kv[:, :Ch], kv[:, Ch:], B, heads, P // B, dh, dh ** -0.5),
             P * C * E),
            ("attn_bwd", lambda: K.pooled_attn_bwd(m, kv[:, :Ch], kv[:, Ch:], o, do, lse, B, heads, P // B, dh,
                                                   dh ** -0.5, dm, dkv[:, :Ch], dkv[:, Ch:]), P * C * E * 2),
            ("bilinear", lambda: K.bilinear(o, (7, 7), (H, W), B), P * Ch * E),
        ]
    res = []
    for name, fn, nb in rows:
        us = timed(fn)
        res.append({"stage": st, "kernel": name, "us": us, "bytes": nb, "frac": nb / us / 1e-6 / HBM})
        print(f"s{st} {name:14s} {us:8.1f} us  {nb / 1e6:8.1f} MB  {nb / us / 1e3:7.0f} GB/s  "
              f"{nb / (us * 1e-6) / HBM:5.2f} of 6.3 TB/s", flush=True)
    return res


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    stages = [int(a) for a in args if a.isdigit()] or [0, 1, 2, 3]
    allr = []
    for st in stages:
        allr += bench_stage(st)
    if out:
        with open(out, "w") as fh:
            json.dump(allr, fh, indent=1)


if __name__ == "__main__":
    main()
