#!/usr/bin/env python3
"""DFormer-Base + ham decoder, 480x640, bs=16 per GPU, bf16 training-step throughput (images/s).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  (N > 1: one rank per GPU over RCCL/xGMI. Launched by torch.distributed.run it uses the
  WORLD_SIZE/RANK/LOCAL_RANK it finds; started directly with --gpus N > 1 it re-launches itself
  under torch.distributed.run as a child process before touching the GPU.)

One step = forward + fused CE loss + backward (bucketed RCCL all-reduce overlapped) + fused AdamW,
on synthetic inputs resident in HBM (BASELINE.json config 3 / 4). Rank 0 prints one JSON line:
whole-job images/s over the K timed steps (barrier + synchronize on both sides, max over ranks),
per-step median / p10 / p90, the roofline of the dominant kernel and of the whole step, and the
CPU-oracle baseline.

Measurement:
  * census step (untimed, after warm-up): the library's launch tracer times every kernel it
    launches with HIP events on the launching stream, and kernels.ACCOUNT charges every entry
    point's algorithmic FLOPs / HBM bytes to the kernel it launched -> per-kernel table
    (launches, F_k, B_k, ideal = sum max(F/P, B/BW), measured). The dominant kernel is the one with
    the largest measured time; the table is written with --table-out.
  * timed steps: only the dominant kernel's launches carry HIP events; its average duration over
    the timed region gives roofline.achieved = algorithmic bytes (or FLOPs) per launch / duration.
  * roofline.step: sum_k max(F_k/P, B_k/BW) over the census / ms_per_step; and SURVEY §8d's
    fused-model bound for DFormer-B bs16 (4.33 TFLOP at the bf16 MFMA peak) / ms_per_step.
"""
import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "images/s training-step, DFormer-B 480×640 bs=16/GPU, 1/2/4/8 MI355X"  # BASELINE.json config 3 / 4


def metric_name(args):
    """BASELINE.json's metric for its own workload (DFormer-B + ham, 480x640, bs 16 per GPU, bf16);
    any other configuration (configs 2 and 5) is named by its own workload."""
    if (args.arch, args.decoder, args.height, args.width, args.batch, args.dtype) == \
            ("DFormer-Base", "ham", 480, 640, 16, "bf16"):
        return METRIC
    return (f"images/s training-step, {args.arch}+{args.decoder} {args.height}×{args.width} bs={args.batch}/GPU, "
            f"{args.dtype}, MI355X")


HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
MFMA_PEAK_TFS = {"bf16": 2500.0, "f32": 157.3}  # dense bf16 MFMA; f32-input MFMA (= vector rate)
# DFormer-B fwd 90.3 GFLOP/img, training step ~3x -> 4.33 TFLOP per bs-16 step
SURVEY_TFLOP_PER_IMG = 4.33 / 16


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--arch", default="DFormer-Base")
    ap.add_argument("--decoder", default="ham")
    ap.add_argument("--ncls", type=int, default=40, help="classes (NYUDepthv2 40, SUNRGBD 37)")
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"],
                    help="compute dtype; fp16 = the reference's --amp (dynamic loss scaling decided on the device, graph replay)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-census", action="store_true")
    ap.add_argument("--eager", action="store_true",
                    help="issue every kernel from Python each step instead of replaying the captured HIP graph")
    ap.add_argument("--table-out", default=None, help="write the per-kernel F/B/time table (JSON) here")
    return ap.parse_args()


def relaunch_distributed(args):
    """--gpus N > 1 without a torch.distributed.run environment: start N ranks as a child
    torch.distributed.run (nothing has touched the GPU in this process) and exit with its code."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


class Cfg(dict):
    __getattr__ = dict.__getitem__


def make_cfg(arch="DFormer-Base", decoder="ham", ncls=40):
    # local_configs/NYUDepthv2/DFormer_Base.py + _base_/datasets/NYUDepthv2.py
    return Cfg(backbone=arch, decoder=decoder, decoder_embed_dim=512, num_classes=ncls, drop_path_rate=0.1,
               bn_eps=1e-3, bn_momentum=0.1, background=255, lr=6e-5, weight_decay=0.01)


def synthetic_batch(B, H, W, ncls, device, seed):
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    mean = torch.tensor([0.485, 0.456, 0.406], device=device).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], device=device).view(1, 3, 1, 1)
    rgb = (torch.randint(0, 256, (B, 3, H, W), device=device, generator=g).float() / 255 - mean) / std
    dep = (torch.randint(0, 256, (B, 1, H, W), device=device, generator=g).float() / 255 - 0.48) / 0.28
    lab = torch.randint(0, ncls, (B, H, W), device=device, generator=g)
    lab[torch.rand(B, H, W, device=device, generator=g) < 0.1] = 255
    return rgb, dep, lab


def census(step_fn):
    """One untimed step with every library kernel timed and every entry point's algorithmic
    FLOPs / bytes charged to the first kernel it launched. Returns {kernel: row}."""
    import torch
    from dformer_amd import kernels as K
    torch.cuda.synchronize()
    K.ACCOUNT = []
    K.trace(3)
    step_fn()
    torch.cuda.synchronize()
    timed = K.trace_read()
    K.trace(0)
    acct, K.ACCOUNT = K.ACCOUNT, None
    tags, tagk = {}, {}
    i = 0  # launches are recorded in order: each accounted call owns the next len(funcs) timings
    for funcs, *_rest in acct:
        tag = _rest[-1] or "other"
        for _ in funcs:
            if i < len(timed):
                tags[tag] = tags.get(tag, 0.0) + timed[i][1]
                key = (tag, timed[i][0][:90])
                n, t = tagk.get(key, (0, 0.0))
                tagk[key] = (n + 1, t + timed[i][1])
            i += 1
    table = {}
    for name, ms in timed:
        r = table.setdefault(name, dict(launches=0, measured_ms=0.0, flops=0.0, bytes=0.0, ideal_ms=0.0, peak=None))
        r["launches"] += 1
        r["measured_ms"] += ms
    for funcs, flops, nbytes, peak, _tag in acct:
        if not funcs:
            continue
        name = K.kernel_name(funcs[0])
        r = table.setdefault(name, dict(launches=0, measured_ms=0.0, flops=0.0, bytes=0.0, ideal_ms=0.0, peak=None))
        r["flops"] += flops
        r["bytes"] += nbytes
        r["peak"] = peak
        r["ideal_ms"] += max(flops / (MFMA_PEAK_TFS[peak] * 1e12), nbytes / (HBM_PEAK_GBS * 1e9)) * 1e3
    census.tags = tags
    census.tag_kernels = tagk
    return table


def pmc_traffic(name):
    """HBM bytes per launch of kernel `name` from the newest PMC record under profiles/ that names it
    (tools/pmc_dominant.py output: r<round>_pmc_*.json, r02_dominant_pmc.json), with the file it came from."""
    import glob
    import re
    recs = []
    for path in glob.glob(os.path.join(HERE, "profiles", "r*_*pmc*.json")):
        m = re.match(r"r(\d+)_", os.path.basename(path))
        try:
            with open(path) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        if isinstance(rec, dict) and rec.get("kernel") == name and rec.get("traffic_bytes_per_launch"):
            recs.append((int(m.group(1)) if m else 0, os.path.basename(path), rec["traffic_bytes_per_launch"]))
    if not recs:
        return None, None
    _, src, traffic = max(recs)
    return traffic, "profiles/" + src


# the census kernels the timed region probes: the measured-dominant one and every kernel within
# PROBE_WITHIN of it (the top two swap between boxes when their census times are that close)
PROBE_WITHIN = 0.05


def probed_kernels(table):
    order = sorted(table, key=lambda n: -table[n]["measured_ms"])
    top = table[order[0]]["measured_ms"]
    return [n for n in order[:3] if table[n]["measured_ms"] >= (1.0 - PROBE_WITHIN) * top]


def dominant_roofline(table, name, durations_ms):
    r = table[name]
    n_c = max(r["launches"], 1)
    fl, by = r["flops"] / n_c, r["bytes"] / n_c
    avg_s = sum(durations_ms) / len(durations_ms) * 1e-3
    peak = MFMA_PEAK_TFS[r["peak"] or "bf16"]
    t_mfma, t_hbm = fl / (peak * 1e12), by / (HBM_PEAK_GBS * 1e9)
    traffic, traffic_src = pmc_traffic(name)
    if t_mfma >= t_hbm:
        ach = fl / avg_s / 1e12
        out = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s", "frac": round(ach / peak, 4)}
    else:
        ach = by / avg_s / 1e9
        out = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": round(ach / HBM_PEAK_GBS, 4)}
    # exact per-launch roofline: sum over the census launches of max(F_i/P, B_i/BW) (launches of one kernel
    # have different shapes, some HBM-, some MFMA-bound) over the probe's mean launch time
    out["frac_exact"] = round(r["ideal_ms"] / n_c * 1e-3 / avg_s, 4)
    out.update(traffic=traffic, traffic_source=traffic_src, kernel=name, launches=len(durations_ms),
               avg_us=round(avg_s * 1e6, 2),
               bytes_per_launch=round(by), flops_per_launch=round(fl),
               census_share=round(r["measured_ms"] / max(sum(t["measured_ms"] for t in table.values()), 1e-9), 4))
    return out


def cpu_baseline(model_sd, seconds):
    """The CPU oracle (oracle/dformer_ref.py, parity-pinned to the reference goldens) timed on this
    host's cores, fp32: DFormer-B + ham fwd+bwd bs=2 at 480x640 (the GPU metric's workload), plus
    BASELINE config 1 (DFormer-Tiny forward, bs=2, 480x640) as a second leg."""
    import torch
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import dformer_ref as R
    import gen
    ncores = len(os.sched_getaffinity(0))
    threads = max(1, min(ncores, int(os.environ.get("OMP_NUM_THREADS", ncores))))
    torch.set_num_threads(threads)
    B, H, W = 2, 480, 640
    rgb, dep, lab = synthetic_batch(B, H, W, 40, "cpu", 0)
    bases = torch.from_numpy(gen.nmf_bases(B, 512, 64)).float()

    def timeit(fn, budget, max_iter):
        fn()  # warm-up
        n, t = 0, 0.0
        while t < budget and n < max_iter:
            t0 = time.perf_counter()
            fn()
            t += time.perf_counter() - t0
            n += 1
        return B * n / t, n

    p = {k: v.detach().float().cpu().clone().requires_grad_(v.is_floating_point() and "running" not in k)
         for k, v in model_sd.items() if not k.endswith("num_batches_tracked")}

    def base_step():
        _, _, loss = R.segmentor_forward(p, "DFormer-Base", "ham", rgb, dep, bases, True, lab)
        loss.backward()

    v_base, n_base = timeit(base_step, seconds, 20)
    shapes = R.segmentor_shapes("DFormer-Tiny", "ham", 40)
    pt = {k: torch.from_numpy(v).float() for k, v in gen.state_dict_values(shapes.items()).items()}

    def tiny_fwd():
        with torch.no_grad():
            R.segmentor_forward(pt, "DFormer-Tiny", "ham", rgb, dep, bases, False, None)

    v_tiny, n_tiny = timeit(tiny_fwd, seconds * 0.5, 60)
    return {"value": round(v_base, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"oracle DFormer-B+ham fwd+bwd fp32 bs=2 480x640, {n_base} timed iters",
            "config1": {"value": round(v_tiny, 3), "unit": "images/s",
                        "sample": f"oracle DFormer-Tiny+ham forward fp32 bs=2 480x640 (BASELINE config 1), "
                                  f"{n_tiny} timed iters"}}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_distributed(args))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from dformer_amd import kernels as K
    from dformer_amd.segmentor import EncoderDecoder
    from dformer_amd.train import FusedAdamW, GraphedTrainStep, train_step

    torch.manual_seed(8964 + rank)
    cfg = make_cfg(args.arch, args.decoder, args.ncls)
    model = EncoderDecoder(cfg=cfg, syncbn=world > 1)
    for m in model.decode_head.modules():  # init_func.init_weight: kaiming on decoder convs
        if isinstance(m, torch.nn.Conv2d):
            torch.nn.init.kaiming_normal_(m.weight, mode="fan_in", nonlinearity="relu")
    sd_cpu = {k: v.clone() for k, v in model.state_dict().items()} if rank == 0 else None
    cdt = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    model = model.to(dev).set_compute_dtype(cdt)
    if world > 1:
        for t in model.state_dict().values():
            dist.broadcast(t, 0)
    model.return_logits = False
    model.train()
    opt = FusedAdamW(model, lr=cfg.lr, weight_decay=cfg.weight_decay, world=world, compute_dtype=cdt)
    rgb, dep, lab = synthetic_batch(args.batch, args.height, args.width, cfg.num_classes, dev, 8964 + rank)

    def step():
        return train_step(model, opt, rgb, dep, lab)

    for _ in range(args.warmup):
        step()
    table, dom, probes = None, None, []
    if not args.no_census:
        table = census(step)
        probes = probed_kernels(table)
        dom = probes[0]
    # HIP-graph mode: the whole step is captured once and replayed, so ~1.6k kernel launches cost one
    # graph launch. Default at world 1 (DFM_GRAPH=0 disables). At world > 1 the step runs EAGERLY unless
    # DFM_GRAPH=1: a captured multi-rank RCCL step has never run on N > 1 hardware (only the one-rank
    # RCCL capture of tests/test_graph_gpu.py has, and one capture_end abort was seen there before the
    # capture waited for the watchdog), and an abort inside a capture cannot be caught and would lose
    # the whole run. The bench line's "launch" field says which mode ran.
    graph_env = os.environ.get("DFM_GRAPH", "1" if world == 1 else "0")
    use_graph = not args.eager and graph_env != "0"
    if use_graph:
        step = GraphedTrainStep(model, opt, rgb, dep, lab)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if dom is not None and not use_graph:
        K.trace(2, probes)
    s = torch.cuda.current_stream()
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    marks[0].record(s)
    loss = None
    for i in range(args.steps):
        loss = step()
        marks[i + 1].record(s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    dom_ms = None
    if dom is not None:
        if use_graph:
            # launches inside a replayed graph cannot be bracketed from the host: the dominant
            # kernel is timed by the same per-launch HIP events over a window of eager steps run
            # right after the timed region (same kernels, same stream, same shapes)
            K.trace(2, probes)
            for _ in range(3):
                step.eager()
            torch.cuda.synchronize()
        probe_ms = {}
        for nm, ms in K.trace_read():
            probe_ms.setdefault(nm, []).append(ms)
        dom_ms = probe_ms.get(dom)
        K.trace(0)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = elapsed.item()
    per_step = sorted(marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps))
    q = statistics.quantiles(per_step, n=10) if len(per_step) >= 2 else [per_step[0]] * 9
    images = world * args.batch * args.steps
    value = images / elapsed
    ms_step = elapsed / args.steps * 1e3
    result = {
        "metric": metric_name(args), "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (random-init weights)",
        "config": {"workload": f"{args.arch}+{args.decoder} train step fwd+bwd+AdamW",
                   "global_batch": world * args.batch, "per_gpu_batch": args.batch,
                   "image": [args.height, args.width], "parallelism": f"dp{world}"},
        "step_ms_gpu": {"median": round(statistics.median(per_step), 3), "p10": round(q[0], 3),
                        "p90": round(q[-1], 3)},
        "launch": "hip_graph" if use_graph else "eager",
        "loss": round(float(loss.item()), 4) if loss is not None else None,
    }
    if rank == 0:
        if table is not None and dom_ms:
            roof = dominant_roofline(table, dom, dom_ms)
            # the other census kernels within PROBE_WITHIN of the dominant one, with the same fields
            roof["close"] = [dominant_roofline(table, n, probe_ms[n]) for n in probes[1:] if probe_ms.get(n)]
            ideal = sum(r["ideal_ms"] for r in table.values())
            traced = sum(r["measured_ms"] for r in table.values())
            survey_ms = None
            if (args.arch, args.decoder, args.height, args.width) == ("DFormer-Base", "ham", 480, 640):
                survey_ms = SURVEY_TFLOP_PER_IMG * args.batch / MFMA_PEAK_TFS["bf16"] * 1e3
            top = sorted(table.items(), key=lambda kv: -kv[1]["measured_ms"])[:5]
            roof["step"] = {
                "ideal_ms": round(ideal, 3), "frac": round(ideal / ms_step, 4),
                "survey_bound_ms": round(survey_ms, 3) if survey_ms else None,
                "survey_frac": round(survey_ms / ms_step, 4) if survey_ms else None,
                "census_traced_ms": round(traced, 3),
                # per-kernel HIP events serialise and pad short kernels: traced time / graph step time
                "census_over_step": round(traced / per_step[len(per_step) // 2], 3),
                "census_launches": sum(r["launches"] for r in table.values()),
                "top": [{"kernel": n[:120], "ms": round(r["measured_ms"], 3), "ideal_ms": round(r["ideal_ms"], 3),
                         "launches": r["launches"]} for n, r in top]}
            result["roofline"] = roof
            if args.table_out:
                os.makedirs(os.path.dirname(os.path.abspath(args.table_out)), exist_ok=True)
                with open(args.table_out, "w") as f:
                    json.dump({"config": result["config"], "ms_per_step": result["ms_per_step"],
                               "by_component_ms": {k: round(v, 4) for k, v in sorted(census.tags.items(),
                                                                                     key=lambda kv: -kv[1])},
                               "by_component_kernel": [[t, k, n, round(ms, 4)] for (t, k), (n, ms) in
                                                       sorted(census.tag_kernels.items(), key=lambda kv: -kv[1][1])],
                               "peaks": {"hbm_GBs": HBM_PEAK_GBS, "mfma_TFs": MFMA_PEAK_TFS},
                               "kernels": {n: {k: (round(v, 6) if isinstance(v, float) else v) for k, v in r.items()}
                                           for n, r in sorted(table.items(), key=lambda kv: -kv[1]["measured_ms"])}},
                              f, indent=1)
        else:
            result["roofline"] = None
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(sd_cpu, args.cpu_seconds)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
