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
    orig = (K.colsum, K.bn_stats, K.bn_bwd_stats, K.bn_bwd_apply)

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

    def bn_bwd_apply(x, dy, mean, rstd, gamma, stats2, count, dx=None, accumulate=False):
        prev = dx.detach().double().clone() if (dx is not None and accumulate) else 0.0
        r = orig[3](x, dy, mean, rstd, gamma, stats2, count, dx, accumulate)
        xh = (x.double() - mean.double()) * rstd.double()
        yd = dy.double()
        want = gamma.double() * rstd.double() * (yd - yd.sum(0) / count - xh * (yd * xh).sum(0) / count)
        got = r.double() - prev
        calls.append(("bn_bwd_apply", tuple(x.shape), rel(got, want), rel(got, want)))
        return r

    # every autograd Function of the package: host copies of what its forward saved, compared bit for bit
    # with what its backward reads (a tensor overwritten in between = a buffer lifetime / aliasing fault);
    # host copies, so the device allocation pattern is the one the step has
    import dformer_amd.decoders as D
    import dformer_amd.encoder as E
    import dformer_amd.functional as Fn
    changed = []
    wrapped = []
    for mod in (D, E, Fn):
        for nm in dir(mod):
            cls = getattr(mod, nm)
            if not (isinstance(cls, type) and issubclass(cls, torch.autograd.Function)) or cls in [w[0] for w in wrapped]:
                continue
            f0, b0 = cls.forward, cls.backward

            def fwd(ctx, *a, _f=f0, _n=nm):
                r = _f(ctx, *a)
                ctx._snap = [t.detach().cpu().clone() if torch.is_tensor(t) else None
                             for t in (getattr(ctx, "to_save", None) or ())]
                return r

            def bwd(ctx, *g, _b=b0, _n=nm):
                for i, (t, s0) in enumerate(zip(ctx.saved_tensors, ctx._snap)):
                    if s0 is not None and not torch.equal(t.detach().cpu(), s0):
                        d = (t.detach().cpu().double() - s0.double()).abs().max().item()
                        changed.append((_n, i, tuple(t.shape), d))
                return _b(ctx, *g)
            wrapped.append((cls, f0, b0))
            cls.forward, cls.backward = staticmethod(fwd), staticmethod(bwd)
    K.colsum, K.bn_stats, K.bn_bwd_stats, K.bn_bwd_apply = colsum, bn_stats, bn_bwd_stats, bn_bwd_apply
    try:
        errs = fp32_audit("e2e_tiny_small", "DFormer-Tiny", "ham", 40)
    finally:
        K.colsum, K.bn_stats, K.bn_bwd_stats, K.bn_bwd_apply = orig
        for cls, f0, b0 in wrapped:
            cls.forward, cls.backward = staticmethod(f0), staticmethod(b0)
    print(f"saved tensors overwritten between forward and backward: {len(changed)}")
    for c in changed[:20]:
        print(f"  {c[0]} saved[{c[1]}] {c[2]} max change {c[3]:.3e}")
    for k in sorted(k for k in errs if not k.startswith("grad/")):
        print(f"  {errs[k]:.3e}  {k}")
    for k in sorted(k for k in errs if k.startswith("grad/decode_head")):
        print(f"  {errs[k]:.3e}  {k}")
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
