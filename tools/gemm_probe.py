"""A/B probe of single GEMM shapes (GPU only): our dfm_gemm vs torch.matmul (hipBLASLt) vs a
device copy of the same number of bytes, to see how far each HBM-bound shape is from what the
chip can stream. Env knobs of the library (DFM_GEMM_*) can be set per run for A/B variants.

    python tools/gemm_probe.py [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dformer_amd import kernels as K  # noqa: E402

# (label, M, N, K, kind)   kind: fwd = x @ w^T (+bias), dgrad = dy @ w, wgrad = dy^T @ x
SHAPES = [
    ("fc1 s0 fwd", 307200, 512, 64, "fwd"),
    ("fc2 s0 fwd", 307200, 64, 512, "fwd"),
    ("fc2 s0 dgrad", 307200, 512, 64, "dgrad"),
    ("fc1 s0 dgrad", 307200, 64, 512, "dgrad"),
    ("fc1 s1 fwd", 76800, 1024, 128, "fwd"),
    ("fc2 s1 fwd", 76800, 128, 1024, "fwd"),
    ("fc1 s2 fwd", 19200, 1024, 256, "fwd"),
    ("fc2 s2 fwd", 19200, 256, 1024, "fwd"),
    ("qcl s2 fwd", 19200, 640, 256, "fwd"),
    ("proj s2 fwd", 19200, 256, 512, "fwd"),
    ("fc1 s0 wgrad", 307200, 512, 64, "wgrad"),
    ("fc2 s2 wgrad", 19200, 256, 1024, "wgrad"),
    ("fc1 s2 wgrad", 19200, 1024, 256, "wgrad"),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    for label, M, N, Kd, kind in SHAPES:
        if kind == "fwd":
            a = torch.randn(M, Kd, device=dev).to(bf)
            w = torch.randn(N, Kd, device=dev).to(bf)
            bias = torch.randn(N, device=dev)
            out = torch.empty(M, N, device=dev, dtype=bf)
            ours = lambda: K.linear(a, w, bias, out=out)  # noqa: E731
            ref = lambda: torch.matmul(a, w.t(), out=out)  # noqa: E731
            nbytes = 2 * (M * Kd + N * Kd + M * N)
        elif kind == "dgrad":
            a = torch.randn(M, Kd, device=dev).to(bf)  # dy [M, Kd]
            w = torch.randn(Kd, N, device=dev).to(bf)  # W [Kd(out), N(in)]
            out = torch.empty(M, N, device=dev, dtype=bf)
            ours = lambda: K.linear_dgrad(a, w, out=out)  # noqa: E731
            ref = lambda: torch.matmul(a, w, out=out)  # noqa: E731
            nbytes = 2 * (M * Kd + N * Kd + M * N)
        else:  # wgrad: dW[N, Kd] = dy[M, N]^T @ x[M, Kd]
            dy = torch.randn(M, N, device=dev).to(bf)
            x = torch.randn(M, Kd, device=dev).to(bf)
            out = torch.empty(N, Kd, device=dev, dtype=torch.float32)
            ours = lambda: K.linear_wgrad(dy, x, out=out)  # noqa: E731
            ref = lambda: torch.matmul(dy.t(), x)  # noqa: E731
            nbytes = 2 * (M * N + M * Kd) + 4 * N * Kd
        src = torch.empty(nbytes // 2, device=dev, dtype=bf)
        dst = torch.empty_like(src)
        t_ours = timeit(ours, args.iters)
        t_ref = timeit(ref, args.iters)
        t_copy = timeit(lambda: dst.copy_(src), args.iters)  # reads + writes nbytes: 2x the traffic
        print(f"{label:14s} M={M:6d} N={N:5d} K={Kd:5d}: ours {t_ours:7.1f}us ({nbytes / t_ours / 1e3:5.0f} GB/s)  "
              f"torch {t_ref:7.1f}us ({nbytes / t_ref / 1e3:5.0f} GB/s)  copy(2x bytes) {t_copy:7.1f}us "
              f"({2 * nbytes / t_copy / 1e3:5.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
