"""Column reductions (colsum, BN stats, BN backward stats) vs float64 over row counts (GPU diagnostic).
    python tools/debug/colred_check.py      (DFM_LIB_PATH selects another library build)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dformer_amd import kernels as K  # noqa: E402


def rel(a, b):
    return ((a.double() - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


torch.manual_seed(0)
worst = 0.0
for dt in (torch.float32, torch.bfloat16):
    for rows in (7, 64, 100, 160, 512, 1000, 4800, 76800):
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
