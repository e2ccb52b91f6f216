"""Launch only the dominant kernel of the step (stage-0 ConvFFN fc2 GEMM with its fused epilogue,
the kernel bench.py rooflines) `--iters` times on synthetic operands of the step's shape, so
rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE, one counter group per pass) see nothing else.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python3 tools/dominant_kernel.py
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dformer_amd import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--M", type=int, default=16 * 120 * 160)
    ap.add_argument("--C", type=int, default=64)
    ap.add_argument("--hidden", type=int, default=512)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    M, N, Kd = a.M, a.C, a.hidden
    g = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, Kd, device=dev) / Kd ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    x = torch.randn(M, N, device=dev).to(torch.bfloat16)
    f = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ls = torch.rand(N, device=dev)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    for _ in range(a.iters):
        K.linear(g, w, b, preact=f, res=x, colscale=ls, out=out)
    torch.cuda.synchronize()
    print(f"launched {a.iters}x gemm M={M} N={N} K={Kd}; algorithmic bytes/launch {2 * (M * Kd + N * Kd + 3 * M * N)}")


if __name__ == "__main__":
    main()
