"""Column reductions (colsum, BN stats, BN backward stats) vs float64 over row counts (GPU diagnostic).

    python tools/debug/colred_check.py            (DFM_LIB_PATH=dformer_amd/variants/lib_<name>.so selects a variant)
    python tools/debug/colred_check.py e2e        + every reduction inside the fp32 e2e_tiny_small step, checked
                                                  call by call in float64 on the same operands, then the audit

It first prints the library path and dfm_build_tag(), so a record names the build it measured (round 5's
colred_base.txt / colred_new.txt were byte-identical: the "new" run had loaded the default library).
Errors are rel-to-max against float64 and, for the e2e calls, also against sum|terms| (the conditioning-
free measure: an fp32 sum of n terms is off by <~ n * 6e-8 of sum|terms| whatever the summation order).
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
from dformer_amd import _lib, kernels as K  # noqa: E402

print("library", _lib.LIB_PATH, "build", _lib.BUILD_TAG, flush=True)

ROWS = (7, 64, 100, 160, 192, 193, 255, 256, 257, 512, 1000, 4800, 4801, 65537, 76800)


def rel(a, b):
    return ((a.double() - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def sweep():
    torch.manual_seed(0)
    worst = 0.0
    for dt in (torch.float32, torch.bfloat16, torch.float16):
        for rows in ROWS:
            for C in (16, 48, 512):
                x = (torch.randn(rows, C, device="cuda") * 3 + 1).to(dt)
                y = torch.randn(rows, C, device="cuda").to(dt)
                xd, yd = x.double(), y.double()
                e1 = rel(K.colsum(x), xd.sum(0))
                st = K.bn_stats(x)
                k = xd[0]
                e2 = max(rel(st[0], (xd - k).sum(0)), rel(st[1], ((xd - k) ** 2).sum(0)), rel(st[2], k))
                mean = torch.randn(C, device="cuda")
                rstd = torch.rand(C, device="cuda") + 0.5
                s2 = K.bn_bwd_stats(x, y, mean, rstd)
                e3 = max(rel(s2[0], yd.sum(0)), rel(s2[1], (yd * (xd - mean.double()) * rstd.double()).sum(0)))
                worst = max(worst, e1, e2, e3)
                flag = "  <-- BAD" if max(e1, e2, e3) > 1e-4 else ""
                print(f"{str(dt)[6:]:9s} rows {rows:6d} C {C:4d} colsum {e1:.1e} bn_stats {e2:.1e} bn_bwd {e3:.1e}{flag}",
                      flush=True)
    print("worst", worst)


def e2e():
    """Every column reduction of the fp32 e2e_tiny_small step against float64 on its own operands."""
    from test_segmentor_gpu import fp32_audit
    calls = []
    orig = (K.colsum, K.bn_stats, K.bn_bwd_stats)

    def cond(terms, got):  # |got - exact| / sum|terms| per column, worst column; and rel-to-max
        exact = terms.sum(0)
        return (((got.double() - exact).abs() / terms.abs().sum(0).clamp_min(1e-30)).max().item(),
                rel(got, exact))

    def colsum(x, mul=None, rowscale=None, rows_per_scale=1, out=None, accumulate=False):
        prev = out.detach().double().clone() if (out is not None and accumulate) else 0.0
        r = orig[0](x, mul, rowscale, rows_per_scale, out, accumulate)
        t = x.double() * (mul.double() if mul is not None else 1.0)
        if rowscale is not None:
            t = t * rowscale.double().repeat_interleave(rows_per_scale)[:, None]
        calls.append(("colsum", tuple(x.shape)) + cond(t, r.double() - prev))
        return r

    def bn_stats(x):
        st = orig[1](x)
        xd = x.double() - x.double()[0]
        calls.append(("bn_stats.sum", tuple(x.shape)) + cond(xd, st[0]))
        calls.append(("bn_stats.sq", tuple(x.shape)) + cond(xd * xd, st[1]))
        return st

    def bn_bwd_stats(x, dy, mean, rstd, out=None):
        st = orig[2](x, dy, mean, rstd, out)
        yd = dy.double()
        xh = (x.double() - mean.double()) * rstd.double()
        calls.append(("bn_bwd.dbeta", tuple(x.shape)) + cond(yd, st[0]))
        calls.append(("bn_bwd.dgamma", tuple(x.shape)) + cond(yd * xh, st[1]))
        return st

    K.colsum, K.bn_stats, K.bn_bwd_stats = colsum, bn_stats, bn_bwd_stats
    try:
        errs = fp32_audit("e2e_tiny_small", "DFormer-Tiny", "ham", 40)
    finally:
        K.colsum, K.bn_stats, K.bn_bwd_stats = orig
    print(f"{len(calls)} reductions in the step; worst 12 by error / sum|terms|:")
    for c in sorted(calls, key=lambda c: -c[2])[:12]:
        print(f"  {c[0]:14s} {str(c[1]):14s} err/sum|terms| {c[2]:.2e}   rel-to-max {c[3]:.2e}")
    bad = sorted(((v, k) for k, v in errs.items() if v > 1e-4), reverse=True)
    print(f"audit: worst {max(errs.values()):.3e}; {len(bad)} entries over 1e-4")
    for v, k in bad[:10]:
        print(f"   {v:.3e}  {k}")


if __name__ == "__main__":
    sweep()
    if len(sys.argv) > 1 and sys.argv[1] == "e2e":
        e2e()
