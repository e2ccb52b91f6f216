"""Attribute the step's torch-side device copies / elementwise launches to Python call sites.

Runs the default bench workload eagerly (no graph) under torch.profiler for one step and prints the
aten ops that launch device work (copy_, clone, fill_, add_, ...) grouped by Python stack.
    python tools/torchprof_copies.py [--batch 16]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile

    import bench
    from dformer_amd.segmentor import EncoderDecoder
    from dformer_amd.train import FusedAdamW, train_step

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = bench.make_cfg()
    model = EncoderDecoder(cfg=cfg, syncbn=False).to(dev).set_compute_dtype(torch.bfloat16)
    model.return_logits = False
    model.train()
    opt = FusedAdamW(model, lr=cfg.lr, weight_decay=cfg.weight_decay, world=1, compute_dtype=torch.bfloat16)
    rgb, dep, lab = bench.synthetic_batch(args.batch, 480, 640, cfg.num_classes, dev, 0)
    for _ in range(3):
        train_step(model, opt, rgb, dep, lab)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        train_step(model, opt, rgb, dep, lab)
        torch.cuda.synchronize()
    kernels = [e for e in prof.events() if e.device_type.name == "CUDA"]
    by = {}
    for e in kernels:
        by.setdefault(e.name[:60], [0, 0.0])
        by[e.name[:60]][0] += 1
        by[e.name[:60]][1] += e.device_time
    print("device events:", len(kernels))
    for n, (c, t) in sorted(by.items(), key=lambda kv: -kv[1][0])[:25]:
        print(f"{c:6d} {t / 1000:8.3f} ms  {n}")
    watch = ("aten::copy_", "aten::clone", "aten::fill_", "aten::zero_", "aten::add_", "aten::add", "aten::cat",
             "aten::contiguous", "aten::mul", "aten::mul_", "aten::div", "aten::sum", "aten::to", "aten::_to_copy",
             "aten::index_put_", "aten::floor", "aten::linalg_vector_norm", "aten::stack")
    rows = prof.key_averages(group_by_stack_n=6)
    rows = [r for r in rows if r.key in watch]
    rows.sort(key=lambda r: -r.count)
    for r in rows[:args.top]:
        print(f"\n{r.count:5d} x {r.key}  device {r.device_time_total / 1000:.3f} ms")
        for fr in (r.stack or [])[:6]:
            print("        ", fr)


if __name__ == "__main__":
    main()
