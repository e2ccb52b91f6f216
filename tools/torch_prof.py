"""Where do the non-library GPU ops of a training step come from? (profiling tool, GPU only)

Runs bench.py's DFormer-B step under torch.profiler with Python stacks and prints, per op name
that is not one of libdformer_hip's kernels, the launch count per step and the top call sites.

    python tools/torch_prof.py [--steps 2]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--batch", type=int, default=16)
    args = ap.parse_args()
    from dformer_amd.segmentor import EncoderDecoder
    from dformer_amd.train import FusedAdamW, train_step
    dev = torch.device("cuda", 0)
    cfg = bench.make_cfg()
    model = EncoderDecoder(cfg=cfg).to(dev).set_compute_dtype(torch.bfloat16)
    model.return_logits = False
    model.train()
    opt = FusedAdamW(model, lr=cfg.lr, weight_decay=cfg.weight_decay, compute_dtype=torch.bfloat16)
    rgb, dep, lab = bench.synthetic_batch(args.batch, 480, 640, cfg.num_classes, dev, 1)
    for _ in range(2):
        train_step(model, opt, rgb, dep, lab)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=False) as prof:
        for _ in range(args.steps):
            train_step(model, opt, rgb, dep, lab)
        torch.cuda.synchronize()
    sites = collections.defaultdict(collections.Counter)
    counts = collections.Counter()
    for ev in prof.events():
        name = ev.name
        if not name.startswith("aten::") or name in ("aten::empty", "aten::view", "aten::as_strided",
                                                     "aten::reshape", "aten::slice", "aten::select",
                                                     "aten::detach", "aten::unbind", "aten::t",
                                                     "aten::permute", "aten::empty_strided", "aten::alias",
                                                     "aten::_reshape_alias", "aten::expand", "aten::unsqueeze",
                                                     "aten::split", "aten::narrow", "aten::transpose",
                                                     "aten::lift_fresh", "aten::squeeze", "aten::resize_",
                                                     "aten::result_type", "aten::is_nonzero", "aten::item",
                                                     "aten::_local_scalar_dense", "aten::empty_like",
                                                     "aten::contiguous", "aten::_unsafe_view", "detach",
                                                     "aten::view_as", "aten::_has_compatible_shallow_copy_type"):
            continue
        counts[name] += 1
        stack = [f for f in (ev.stack or []) if "dformer_amd" in f or "bench" in f or "torch/nn" in f]
        sites[name][" <- ".join(stack[:3]) or "(no python frame)"] += 1
    for name, n in counts.most_common(30):
        print(f"{n / args.steps:7.1f}/step {name}")
        for site, k in sites[name].most_common(4):
            print(f"          {k / args.steps:6.1f}  {site[:220]}")


if __name__ == "__main__":
    main()
