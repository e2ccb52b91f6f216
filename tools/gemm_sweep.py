"""GEMM shape census + split-K sweep for the DFormer-B training step (profiling tool, GPU only).

Runs one bf16 training step of the bench configuration with kernels.GEMM_TRACE on, de-duplicates
the GEMM descriptors it launched, then replays every distinct shape on synthetic operands with
the library's default split choice and with forced split counts, and writes a JSON table:
per shape the call count, algorithmic bytes / flops, and the time of each variant. The
per-step totals show where the GEMM time goes and what a better split heuristic would buy.

    python tools/gemm_sweep.py --out gpurun_out/gemm_sweep.json [--batch 16]
"""
import argparse
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from dformer_amd import _lib, kernels as K  # noqa: E402

COLD = None  # --cold: a 1 GiB buffer rewritten before every timed launch
GRAPH = False  # --graph: time launches replayed from a captured graph (device time, no host pacing)

PTR_FIELDS = ("bias", "preact", "mul", "res", "colscale", "rowscale", "colsum")


def capture(batch, arch, decoder):
    from dformer_amd.segmentor import EncoderDecoder
    from dformer_amd.train import FusedAdamW, train_step
    dev = torch.device("cuda", 0)
    cfg = bench.make_cfg(arch, decoder)
    model = EncoderDecoder(cfg=cfg).to(dev).set_compute_dtype(torch.bfloat16)
    model.return_logits = False
    model.train()
    opt = FusedAdamW(model, lr=cfg.lr, weight_decay=cfg.weight_decay, compute_dtype=torch.bfloat16)
    rgb, dep, lab = bench.synthetic_batch(batch, 480, 640, cfg.num_classes, dev, 1)
    train_step(model, opt, rgb, dep, lab)
    K.GEMM_TRACE = []
    train_step(model, opt, rgb, dep, lab)
    torch.cuda.synchronize()
    tr, K.GEMM_TRACE = K.GEMM_TRACE, None
    return tr


def key(d):
    return tuple((k, (v is not None and v != 0) if k in PTR_FIELDS else v) for k, v in sorted(d.items()))


def mat_elems(rows, ld, batch, stride):
    return rows * ld + (batch - 1) * stride


def replay(d, splits, iters=20):
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16 if d["dtype"] == _lib.BF16 else torch.float32
    M, N, Kd, batch = d["M"], d["N"], d["K"], max(1, d["batch"])
    a = torch.randn(mat_elems(M if d["a_kcontig"] else Kd, d["lda"], batch, d["stride_a"]), device=dev).to(dt)
    b = torch.randn(mat_elems(N if d["b_kcontig"] else Kd, d["ldb"], batch, d["stride_b"]), device=dev).to(dt)
    odt = torch.float32 if d["out_f32"] else dt
    c = torch.randn(mat_elems(M, d["ldc"], batch, d["stride_c"]), device=dev).to(odt)
    keep = []

    def buf(n, t=dt):
        x = torch.randn(max(n, 1), device=dev).to(t)
        keep.append(x)
        return x.data_ptr()

    ptrs = {f: None for f in PTR_FIELDS}
    if d["bias"]:
        ptrs["bias"] = buf(N, torch.float32)
    if d["preact"]:
        ptrs["preact"] = buf(M * d["ldpre"])
    if d["mul"]:
        ptrs["mul"] = buf(M * d["ldmul"])
    if d["res"]:
        ptrs["res"] = buf(M * d["ldres"])
    if d["colscale"]:
        ptrs["colscale"] = buf(N, torch.float32)
    if d["rowscale"]:
        ptrs["rowscale"] = buf(M, torch.float32)
    if d["colsum"]:
        ptrs["colsum"] = buf(M, torch.float32)
    desc = _lib.GemmDesc(M, N, Kd, batch, d["a_kcontig"], d["b_kcontig"], d["lda"], d["ldb"], d["ldc"],
                         d["stride_a"], d["stride_b"], d["stride_c"], 1.0, d["beta"], d["c_f32"], ptrs["bias"],
                         d["act"], ptrs["preact"], d["ldpre"], ptrs["mul"], d["ldmul"], ptrs["res"], d["ldres"],
                         ptrs["colscale"], ptrs["rowscale"], d["rows_per_scale"], splits, d["act_col0"],
                         ptrs["colsum"], d["colsum_accumulate"], d["mul_gelu_grad"])
    ws = K._ws(_lib.lib.dfm_gemm_workspace_size(desc), dev)
    desc.workspace_bytes = ws.numel() if ws is not None else 0
    s = _lib.stream()

    def launch():
        _lib.check(_lib.lib.dfm_gemm(d["dtype"], desc, a.data_ptr(), b.data_ptr(), c.data_ptr(),
                                     _lib.ptr(ws), s), "dfm_gemm")

    for _ in range(3):
        launch()
    if COLD is not None:  # evict the operands from L2 and the 256 MiB Infinity Cache before every launch
        ts = []
        for _ in range(iters // 2):
            COLD.add_(1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launch()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        return ts[len(ts) // 2]
    if GRAPH:  # device time per launch: the launches replayed from a HIP graph (no host pacing)
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            with torch.cuda.graph(g, stream=cs):
                for _ in range(iters):
                    _lib.check(_lib.lib.dfm_gemm(d["dtype"], desc, a.data_ptr(), b.data_ptr(), c.data_ptr(),
                                                 _lib.ptr(ws), _lib.stream()), "dfm_gemm")
        torch.cuda.current_stream().wait_stream(cs)
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / iters)
        return min(ts)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        launch()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters  # us


def algo(d):
    es = 2 if d["dtype"] == _lib.BF16 else 4
    oes = 4 if d["out_f32"] else es
    M, N, Kd, b = d["M"], d["N"], d["K"], max(1, d["batch"])
    nbytes = b * (es * (M * Kd + N * Kd) + oes * M * N * (2 if d["beta"] else 1))
    for f in ("preact", "mul", "res"):
        if d[f]:
            nbytes += b * M * N * es
    return nbytes, 2.0 * b * M * N * Kd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/gemm_sweep.json")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--arch", default="DFormer-Base")
    ap.add_argument("--decoder", default="ham")
    ap.add_argument("--no-splits", action="store_true", help="time only the default split choice")
    ap.add_argument("--cold", action="store_true", help="operands evicted from L2 / Infinity Cache per launch")
    ap.add_argument("--replay", default="", help="replay the shapes of an earlier sweep JSON instead of capturing")
    ap.add_argument("--graph", action="store_true", help="time graph-replayed launches (device time)")
    ap.add_argument("--min-count", type=int, default=1, help="replay only shapes called at least this often")
    ap.add_argument("--wgrad-only", action="store_true", help="only the weight-gradient layout (both row-contiguous)")
    args = ap.parse_args()
    global COLD, GRAPH
    GRAPH = args.graph
    if args.cold:
        COLD = torch.zeros(256 << 20, device="cuda")
    groups = collections.OrderedDict()
    if args.replay:
        for r in json.load(open(args.replay))["rows"]:
            d = dict(r["desc"])
            groups[key(d)] = [d, r["count"]]
    else:
        for d in capture(args.batch, args.arch, args.decoder):
            groups.setdefault(key(d), [d, 0])[1] += 1
    rows = []
    for _, (d, cnt) in groups.items():
        if cnt < args.min_count or (args.wgrad_only and (d["a_kcontig"] or d["b_kcontig"])):
            continue
        nbytes, flops = algo(d)
        r = {"count": cnt, "desc": {k: (bool(v) if k in PTR_FIELDS else v) for k, v in d.items()},
             "bytes": nbytes, "flops": flops, "t_default": replay(d, 0)}
        cands = {}
        for sp in (() if args.no_splits else (1, 2, 4, 8, 16, 32, 64, 128, 256)):
            if sp > 1 and d["K"] // sp < 256:
                break
            cands[sp] = replay(d, sp)
        r["t_split"] = cands
        r["ideal_us"] = max(nbytes / 6.0e6, flops / 1.2e9)  # 6 TB/s achievable, 1.2 PF/s sustained
        rows.append(r)
        print(f"{cnt:3d}x M={d['M']:6d} N={d['N']:5d} K={d['K']:6d} b={d['batch']:3d} ak={d['a_kcontig']} "
              f"bk={d['b_kcontig']} dt={d['dtype']} def={r['t_default']:8.1f}us best="
              f"{min(cands.values(), default=r['t_default']):8.1f}us@{min(cands, key=cands.get, default=0):3d} "
              f"ideal={r['ideal_us']:7.1f}us",
              flush=True)
    tot_def = sum(r["count"] * r["t_default"] for r in rows) / 1e3
    tot_best = sum(r["count"] * min(r["t_split"].values(), default=r["t_default"]) for r in rows) / 1e3
    tot_ideal = sum(r["count"] * r["ideal_us"] for r in rows) / 1e3
    print(f"per step: default {tot_def:.2f} ms, best-split {tot_best:.2f} ms, ideal {tot_ideal:.2f} ms")
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump({"rows": rows, "ms_default": tot_def, "ms_best": tot_best, "ms_ideal": tot_ideal}, f, indent=1)


if __name__ == "__main__":
    main()
