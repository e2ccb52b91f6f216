"""Per-shape comparison of dfm_gemm with the vendor BLAS (torch.matmul -> hipBLASLt) on the GEMM
census of the DFormer-B step (profiling tool, GPU only; not part of the product path).

Reads the shape table written by tools/gemm_sweep.py, replays every bf16 / fp32 shape as a plain
GEMM (no epilogue) through dfm_gemm and through torch.matmul on the same strided operands, and
prints per-shape microseconds and per-step totals. Tells which shapes the hand-written kernel
loses on and by how much, i.e. what the tile/pipeline work has left to win.

    python tools/gemm_blas.py --sweep gpurun_out/gemm_sweep_r02.json --out gpurun_out/gemm_blas.json

Batched shapes are skipped: in round 3 a run faulted the GPU (illegal address) on the first batched
bf16 shape of the list (M=4800, N=512, K=896, batch 16, transposed-B view), inside the timed pair of
this tool's own launches, after 79 shapes had completed; the library kernel of that shape runs in
every training step (the NMF backward's input gradient), so the torch.matmul / hipBLASLt call on the
strided batched view is the suspect, not confirmed. Results of that run: profiles/r03_gemm_blas.txt.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dformer_amd import _lib, kernels as K  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def run(d):
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16 if d["dtype"] == _lib.BF16 else torch.float32
    M, N, Kd, batch = d["M"], d["N"], d["K"], max(1, d["batch"])
    ak, bk = d["a_kcontig"], d["b_kcontig"]
    a = torch.randn(batch, M if ak else Kd, Kd if ak else M, device=dev).to(dt)
    b = torch.randn(batch, N if bk else Kd, Kd if bk else N, device=dev).to(dt)
    am = a if ak else a.transpose(1, 2)       # [batch, M, K]
    bm = b.transpose(1, 2) if bk else b       # [batch, K, N]
    c = torch.empty(batch, M, N, device=dev, dtype=dt)
    desc = _lib.GemmDesc(M, N, Kd, batch, ak, bk, a.shape[2], b.shape[2], N, a.shape[1] * a.shape[2],
                         b.shape[1] * b.shape[2], M * N, 1.0, 0.0, 0, None, 0, None, 0, None, 0, None, 0,
                         None, None, 1, 0, 0, None, 0, 0)
    ws = K._ws(_lib.lib.dfm_gemm_workspace_size(desc), dev)
    desc.workspace_bytes = ws.numel() if ws is not None else 0
    s = _lib.stream()

    def mine():
        _lib.check(_lib.lib.dfm_gemm(d["dtype"], desc, a.data_ptr(), b.data_ptr(), c.data_ptr(), _lib.ptr(ws), s),
                   "dfm_gemm")

    def blas():
        torch.matmul(am, bm, out=c)

    t_mine, t_blas = timeit(mine), timeit(blas)
    ref = torch.matmul(am.float(), bm.float())
    err = ((c.float() - ref).norm() / ref.norm().clamp_min(1e-30)).item()
    mine()
    err_m = ((c.float() - ref).norm() / ref.norm().clamp_min(1e-30)).item()
    return t_mine, t_blas, err_m, err


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweep", default="gpurun_out/gemm_sweep_r02.json")
    ap.add_argument("--out", default="gpurun_out/gemm_blas.json")
    ap.add_argument("--max-k", type=int, default=0, help="only shapes with K <= this (0: all)")
    args = ap.parse_args()
    rows = json.load(open(args.sweep))["rows"]
    out, tm, tb, td = [], 0.0, 0.0, 0.0
    for r in rows:
        d = r["desc"]
        if d["batch"] > 1 or (args.max_k and d["K"] > args.max_k):
            continue
        t_mine, t_blas, em, eb = run(d)
        cnt = r["count"]
        tm += cnt * t_mine
        tb += cnt * t_blas
        td += cnt * r["t_default"]
        out.append({"count": cnt, "M": d["M"], "N": d["N"], "K": d["K"], "batch": d["batch"], "ak": d["a_kcontig"],
                    "bk": d["b_kcontig"], "dtype": d["dtype"], "t_mine_plain": t_mine, "t_blas": t_blas,
                    "t_mine_epilogue": r["t_default"], "err_mine": em, "err_blas": eb})
        print(f"{cnt:3d}x M={d['M']:6d} N={d['N']:5d} K={d['K']:6d} b={d['batch']:3d} ak={d['a_kcontig']} "
              f"bk={d['b_kcontig']} dt={d['dtype']} mine={t_mine:8.1f}us blas={t_blas:8.1f}us "
              f"(epi {r['t_default']:7.1f})", flush=True)
    print(f"per step: mine plain {tm / 1e3:.2f} ms, blas {tb / 1e3:.2f} ms, mine with epilogues {td / 1e3:.2f} ms")
    with open(args.out, "w") as f:
        json.dump({"rows": out, "ms_mine": tm / 1e3, "ms_blas": tb / 1e3, "ms_mine_epi": td / 1e3}, f, indent=1)


if __name__ == "__main__":
    main()
