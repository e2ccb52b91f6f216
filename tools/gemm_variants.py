"""Time the LDS-DMA ring GEMM at several tile / ring-depth / occupancy points (tools/gemm_variants/) on
every bf16 forward / input-gradient GEMM shape of one DFormer-B training step (profiling tool, GPU
only). Prints per shape the library's current time and each variant's, and per-step totals for the
current routing and for the best variant per shape.

    python tools/gemm_variants.py [--out gpurun_out/gemm_variants.json]
"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from dformer_amd import _lib  # noqa: E402
import gemm_sweep  # noqa: E402

ctypes.CDLL(_lib.LIB_PATH, mode=ctypes.RTLD_GLOBAL)  # the variants resolve the library's runtime symbols
GV = ctypes.CDLL(os.path.join(ROOT, "tools", "gemm_variants", "libgemm_variants.so"))
GV.gv_run.argtypes = [ctypes.c_int, ctypes.POINTER(_lib.GemmDesc), ctypes.c_void_p, ctypes.c_void_p,
                      ctypes.c_void_p, ctypes.c_void_p]
NAMES = ["64x64 r2 x4", "64x64 r3 x3", "64x64 r4 x2", "64x128 r2 x3", "64x128 w8 r2", "128x64 r2 x3",
         "128x128 w8 r2", "64x256 w8 r2", "128x128 w8 r3"]


def graph_time(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    out_path = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    dev = torch.device("cuda", 0)
    groups = {}
    for d in gemm_sweep.capture(16, "DFormer-Base", "ham"):
        if d["dtype"] != _lib.BF16 or not d["a_kcontig"] or d["K"] < 128 or d["batch"] > 1 or d["out_f32"]:
            continue
        groups.setdefault(gemm_sweep.key(d), [d, 0])[1] += 1
    rows = []
    tot_cur, tot_best = 0.0, 0.0
    for d, cnt in groups.values():
        M, N, Kd = d["M"], d["N"], d["K"]
        a = torch.randn(M * d["lda"], device=dev).to(torch.bfloat16)
        b = torch.randn((N if d["b_kcontig"] else Kd) * d["ldb"], device=dev).to(torch.bfloat16)
        c = torch.randn(M * d["ldc"], device=dev).to(torch.bfloat16)
        keep = []

        def buf(n, t=torch.bfloat16):
            x = torch.randn(max(n, 1), device=dev).to(t)
            keep.append(x)
            return x.data_ptr()

        ptrs = {f: None for f in gemm_sweep.PTR_FIELDS}
        for f, n, t in (("bias", N, torch.float32), ("preact", M * d["ldpre"], torch.bfloat16),
                        ("mul", M * d["ldmul"], torch.bfloat16), ("res", M * d["ldres"], torch.bfloat16),
                        ("colscale", N, torch.float32), ("rowscale", M, torch.float32)):
            if d[f]:
                ptrs[f] = buf(n, t)
        desc = _lib.GemmDesc(M, N, Kd, 1, d["a_kcontig"], d["b_kcontig"], d["lda"], d["ldb"], d["ldc"],
                             0, 0, 0, 1.0, d["beta"], d["c_f32"], ptrs["bias"], d["act"], ptrs["preact"],
                             d["ldpre"], ptrs["mul"], d["ldmul"], ptrs["res"], d["ldres"], ptrs["colscale"],
                             ptrs["rowscale"], d["rows_per_scale"], 0, d["act_col0"], None, 0,
                             d["mul_gelu_grad"], 0)
        nws = _lib.lib.dfm_gemm_workspace_size(desc)
        ws = torch.empty(max(nws, 1), device=dev, dtype=torch.uint8)
        desc.workspace_bytes = nws
        cur = graph_time(lambda: _lib.check(_lib.lib.dfm_gemm(_lib.BF16, desc, a.data_ptr(), b.data_ptr(),
                                                              c.data_ptr(), ws.data_ptr(), _lib.stream()), "dfm_gemm"))
        ts = []
        for v in range(GV.gv_count()):
            def run(v=v):
                r = GV.gv_run(v, desc, a.data_ptr(), b.data_ptr(), c.data_ptr(), _lib.stream())
                if r != 0:
                    raise RuntimeError(f"variant {v}: {r}")
            try:
                ts.append(graph_time(run))
            except RuntimeError:
                ts.append(float("nan"))
        best = min((t for t in ts if t == t), default=cur)
        tot_cur += cnt * cur
        tot_best += cnt * min(best, cur)
        rows.append({"count": cnt, "M": M, "N": N, "K": Kd, "bk": d["b_kcontig"],
                     "epi": [f for f in ("bias", "preact", "mul", "res") if d[f]] + (["beta"] if d["beta"] else []),
                     "t_lib": cur, "t_var": ts})
        print(f"{cnt:3d}x M={M:6d} N={N:5d} K={Kd:5d} bk={d['b_kcontig']} lib={cur:7.1f} | " +
              " ".join(f"{t:7.1f}" for t in ts) + f" | best {NAMES[ts.index(best)] if best in ts else 'lib'}",
              flush=True)
    print("variants: " + ", ".join(f"{i}={n}" for i, n in enumerate(NAMES)))
    print(f"per step: library {tot_cur / 1e3:.2f} ms, best variant per shape {tot_best / 1e3:.2f} ms")
    if out_path:
        with open(out_path, "w") as fh:
            json.dump({"names": NAMES, "rows": rows, "ms_lib": tot_cur / 1e3, "ms_best": tot_best / 1e3}, fh, indent=1)


if __name__ == "__main__":
    main()
