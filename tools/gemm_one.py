"""Replay one plain GEMM shape through dfm_gemm (profiling driver for rocprofv3, GPU only).

    python tools/gemm_one.py M N K ak bk [iters] [splits] [dtype: bf16|f32] [batch]
Prints the mean microseconds per launch from HIP events on the launch stream.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dformer_amd import _lib, kernels as K  # noqa: E402


def main():
    M, N, Kd, ak, bk = (int(v) for v in sys.argv[1:6])
    iters = int(sys.argv[6]) if len(sys.argv) > 6 else 20
    splits = int(sys.argv[7]) if len(sys.argv) > 7 else 0
    dt = torch.float32 if len(sys.argv) > 8 and sys.argv[8] == "f32" else torch.bfloat16
    batch = int(sys.argv[9]) if len(sys.argv) > 9 else 1
    code = _lib.F32 if dt == torch.float32 else _lib.BF16
    dev = torch.device("cuda", 0)
    a = torch.randn(batch, M if ak else Kd, Kd if ak else M, device=dev).to(dt)
    b = torch.randn(batch, N if bk else Kd, Kd if bk else N, device=dev).to(dt)
    c = torch.empty(batch, M, N, device=dev, dtype=dt)
    desc = _lib.GemmDesc(M, N, Kd, batch, ak, bk, a.shape[2], b.shape[2], N, a.shape[1] * a.shape[2],
                         b.shape[1] * b.shape[2], M * N, 1.0, 0.0, 0, None, 0, None, 0, None, 0, None, 0,
                         None, None, 1, splits, 0, None, 0, 0)
    ws = K._ws(_lib.lib.dfm_gemm_workspace_size(desc), dev)
    desc.workspace_bytes = ws.numel() if ws is not None else 0
    s = _lib.stream()

    def launch():
        _lib.check(_lib.lib.dfm_gemm(code, desc, a.data_ptr(), b.data_ptr(), c.data_ptr(), _lib.ptr(ws), s),
                   "dfm_gemm")

    launch()
    torch.cuda.synchronize()
    ref = torch.matmul((a if ak else a.transpose(1, 2)).float(), (b.transpose(1, 2) if bk else b).float())
    err = ((c.float() - ref).norm() / ref.norm()).item()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        launch()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    ideal = max((a.numel() + b.numel() + c.numel()) * a.element_size() / 6.0e6, 2.0 * batch * M * N * Kd / 1.2e9)
    print(f"M={M} N={N} K={Kd} ak={ak} bk={bk} b={batch} splits={splits} cfg={os.environ.get('DFM_GEMM_CFG', '-')} "
          f"{us:.1f} us (ideal {ideal:.1f}) err={err:.2e}", flush=True)


if __name__ == "__main__":
    main()
