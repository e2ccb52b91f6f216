"""Diagnose a fused ConvFFN forward mismatch: same inputs, 5 runs, bitwise comparison across runs and
the error location against the op-level chain (GPU only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_convffn_gpu import make_case, run_fn  # noqa: E402
from dformer_amd import kernels as K  # noqa: E402

for dt in (torch.float16, torch.bfloat16):
    for case in [(2, 11, 13, 64, 512), (1, 17, 23, 128, 512), (2, 7, 9, 256, 1024)]:
        B, H, W, C, R = case
        p, x, dout, rowscale = make_case(B, H, W, C, R, dt, seed=C + R + H, droppath=(H % 2 == 0))
        W1, W2 = p["w1"].to(dt), p["w2"].to(dt)
        outs = []
        for _ in range(5):
            o = K.convffn_fwd(x, (B, H, W), p["ln_w"], p["ln_b"], W1, p["b1"], p["wpos"], p["bpos"], W2, p["b2"],
                              p["ls"], rowscale)
            torch.cuda.synchronize()
            outs.append([t.clone() for t in o])
        same = [all(torch.equal(a, b) for a, b in zip(outs[0], o)) for o in outs[1:]]
        uo = run_fn(p, x, dout, (B, H, W), rowscale, False)[0]
        err = (outs[0][0].float() - uo.float()).abs()
        pix = err.amax(1)
        bad = (pix > 0.05 * uo.float().abs().max()).nonzero().flatten().tolist()
        print(dt, case, "repeat-equal", same, "max err", err.max().item(), "bad pixels", len(bad), bad[:20], flush=True)
