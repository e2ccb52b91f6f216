"""Isolated timing of every launch of one ConvFFN forward + backward (DFormer.py:48-67) at the
DFormer-B bf16 bs=16 480x640 stage shapes, against its algorithmic HBM bytes (profiling tool, GPU
only): which of the memory-bound kernels is furthest from the ~6.3 TB/s a streaming kernel reaches.

    python tools/ffn_kernels_bench.py [stage ...] [--json out.json]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dformer_amd import kernels as K  # noqa: E402

STAGES = {0: (120, 160, 64, 8), 1: (60, 80, 128, 8), 2: (30, 40, 256, 4), 3: (15, 20, 512, 4)}
HBM = 6.3e12


def timed(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(it):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


def bench_stage(st, branch="mlp"):
    H, W, C, r = STAGES[st]
    if branch == "mlp_e2":
        C //= 2
    B = 16
    P = B * H * W
    hid = r * C
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    x = torch.randn(P, C, device=dev).to(bf)
    lnw, lnb = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    w1 = (torch.randn(hid, C, device=dev) / C ** 0.5).to(bf)
    b1 = torch.randn(hid, device=dev) * 0.1
    wpos = torch.randn(hid, 1, 3, 3, device=dev) / 3
    bpos = torch.randn(hid, device=dev) * 0.1
    w2 = (torch.randn(C, hid, device=dev) / hid ** 0.5).to(bf)
    b2 = torch.randn(C, device=dev) * 0.1
    ls = torch.rand(C, device=dev)
    rs = torch.rand(B, device=dev)
    xn, mu, rstd = K.layernorm(x, lnw, lnb)
    h = K.linear(xn, w1, b1)
    g = torch.empty_like(h)
    gp = K.dwconv(h, (B, H, W), wpos, bpos, 3, add_identity=True, gelu_out=g, out_gelu_grad=True)
    f = torch.empty(P, C, device=dev, dtype=bf)
    out = K.linear(g, w2, b2, preact=f, res=x, colscale=ls, rowscale=rs, rows_per_scale=H * W)
    dout = torch.randn(P, C, device=dev).to(bf)
    df, _ = K.residual_bwd(dout, f, ls, rs, H * W)
    dhpre = K.linear_dgrad(df, w2, mul=gp)
    dh, _, _ = K.dwconv_bwd(h, dhpre, (B, H, W), wpos, 3, add_identity=True)
    E = 2  # bytes per element
    rows = [
        ("ln_fwd", lambda: K.layernorm(x, lnw, lnb, out=xn), P * C * E * 2),
        ("fc1", lambda: K.linear(xn, w1, b1, out=h), P * (C + hid) * E),
        ("dw3+gelu", lambda: K.dwconv(h, (B, H, W), wpos, bpos, 3, add_identity=True, out=gp, gelu_out=g,
                                      out_gelu_grad=True), P * hid * E * 3),
        ("fc2+res", lambda: K.linear(g, w2, b2, preact=f, res=x, colscale=ls, rowscale=rs, rows_per_scale=H * W,
                                     out=out), P * (hid + 3 * C) * E),
        ("residual_bwd", lambda: K.residual_bwd(dout, f, ls, rs, H * W, df=df), P * C * E * 3),
        ("fc2_dgrad*gp", lambda: K.linear_dgrad(df, w2, mul=gp, out=dhpre), P * (C + 2 * hid) * E),
        ("dw3_bwd", lambda: K.dwconv_bwd(h, dhpre, (B, H, W), wpos, 3, add_identity=True, dx=dh), P * hid * E * 3),
        ("fc1_dgrad", lambda: K.linear_dgrad(dh, w1, out=xn), P * (hid + C) * E),
        ("wgrad fc2+fc1", lambda: _wg(df, g, dh, xn), P * (C + hid + hid + C) * E),
        ("ln_bwd", lambda: K.layernorm_bwd(x, xn, lnw, mu, rstd, dres=dout), P * C * E * 4),
    ]
    if K.convffn_supported(bf, (B, H, W), C, hid):  # the fused ConvFFN entry points on the same operands
        fo = K.convffn_fwd(x, (B, H, W), lnw, lnb, w1, b1, wpos, bpos, w2, b2, ls, rs)
        rows += [
            ("FUSED fwd", lambda: K.convffn_fwd(x, (B, H, W), lnw, lnb, w1, b1, wpos, bpos, w2, b2, ls, rs),
             P * (3 * C + hid) * E),
            ("FUSED bwd", lambda: K.convffn_bwd(dout, x, fo[2], fo[3], fo[1], fo[4], fo[5], (B, H, W), lnw, lnb, w1,
                                                wpos, bpos, w2, ls, rs),
             P * (3 * C + 2 * C + 3 * hid + 5 * C) * E),
            ("FUSED fwd+g", lambda: K.convffn_fwd(x, (B, H, W), lnw, lnb, w1, b1, wpos, bpos, w2, b2, ls, rs,
                                                  save_gelu=True),
             P * (3 * C + 3 * hid) * E),
        ]
    res = []
    for name, fn, nb in rows:
        us = timed(fn)
        res.append({"stage": st, "branch": branch, "kernel": name, "us": us, "bytes": nb,
                    "GBps": nb / us / 1e3, "frac": nb / us / 1e-6 / HBM})
        print(f"s{st}.{branch:6s} {name:14s} {us:8.1f} us  {nb / 1e6:8.1f} MB  {nb / us / 1e3:7.0f} GB/s  "
              f"{nb / (us * 1e-6) / HBM:5.2f} of 6.3 TB/s", flush=True)
    return res


def _wg(df, g, dh, xn):
    with K.wgrad_group():
        K.linear_wgrad(df, g, bias_grad=True)
        K.linear_wgrad(dh, xn, bias_grad=True)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    stages = [int(a) for a in args if a.isdigit()] or [0, 1, 2]
    allr = []
    for st in stages:
        for br in ("mlp", "mlp_e2"):
            allr += bench_stage(st, br)
    for st in stages:
        for br in ("mlp", "mlp_e2"):
            rr = [r for r in allr if r["stage"] == st and r["branch"] == br]
            unf = [r["us"] for r in rr if not r["kernel"].startswith("FUSED")]
            fus = {r["kernel"]: r["us"] for r in rr if r["kernel"].startswith("FUSED")}
            if fus:
                print(f"s{st}.{br:6s} unfused fwd {sum(unf[:4]):7.1f} us bwd {sum(unf[4:]):7.1f} us | fused fwd "
                      f"{fus['FUSED fwd']:7.1f} us bwd {fus['FUSED bwd']:7.1f} us | fused fwd+g "
                      f"{fus['FUSED fwd+g']:7.1f} us")
    allr = [r for r in allr if not r["kernel"].startswith("FUSED")]
    tot = sum(r["us"] for r in allr)
    ideal = sum(r["bytes"] for r in allr) / HBM * 1e6
    print(f"total {tot:.1f} us, HBM ideal at 6.3 TB/s {ideal:.1f} us ({ideal / tot:.2f})")
    if out:
        with open(out, "w") as fh:
            json.dump(allr, fh, indent=1)


if __name__ == "__main__":
    main()
