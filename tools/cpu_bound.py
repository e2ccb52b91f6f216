"""Is the training step launch-bound? (profiling tool, GPU only)

Measures, for the bench configuration: (a) GPU ms/step from events; (b) host ms/step spent issuing
a step (no synchronisation inside); (c) GPU ms/step for steps queued behind a long GPU sleep, i.e.
with the host far ahead of the device: if (c) < (a) the normal step has launch bubbles.
    python tools/cpu_bound.py [--steps 10]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=16)
    args = ap.parse_args()
    from dformer_amd.segmentor import EncoderDecoder
    from dformer_amd.train import FusedAdamW, train_step
    dev = torch.device("cuda", 0)
    cfg = bench.make_cfg("DFormer-Base", "ham")
    model = EncoderDecoder(cfg=cfg).to(dev).set_compute_dtype(torch.bfloat16)
    model.return_logits = False
    model.train()
    opt = FusedAdamW(model, lr=cfg.lr, weight_decay=cfg.weight_decay, compute_dtype=torch.bfloat16)
    rgb, dep, lab = bench.synthetic_batch(args.batch, 480, 640, cfg.num_classes, dev, 1)
    for _ in range(5):
        train_step(model, opt, rgb, dep, lab)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    # (a) + (b)
    ev[0].record()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        train_step(model, opt, rgb, dep, lab)
    host = (time.perf_counter() - t0) * 1e3 / args.steps
    ev[1].record()
    torch.cuda.synchronize()
    gpu = ev[0].elapsed_time(ev[1]) / args.steps
    # (c): queue the steps behind a ~1.5 s GPU sleep
    e2 = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda._sleep(int(1.5e9 * 2.1))
    e2[0].record()
    n = min(args.steps, 20)
    for _ in range(n):
        train_step(model, opt, rgb, dep, lab)
    e2[1].record()
    torch.cuda.synchronize()
    ahead = e2[0].elapsed_time(e2[1]) / n
    print(f"gpu {gpu:.2f} ms/step, host issue {host:.2f} ms/step, host-ahead gpu {ahead:.2f} ms/step", flush=True)
    # host time per phase (a phase that blocks on the device shows up as a long host time)
    from dformer_amd.train import all_reduce_mean
    torch.cuda.synchronize()
    torch.cuda._sleep(int(0.5e9 * 2.1))
    t = [time.perf_counter()]
    loss, _ = model(rgb, dep, lab)
    t.append(time.perf_counter())
    all_reduce_mean(loss.detach(), opt.world)
    loss.backward()
    t.append(time.perf_counter())
    opt.step(None)
    t.append(time.perf_counter())
    torch.cuda.synchronize()
    t.append(time.perf_counter())
    print("host ms: forward %.1f backward %.1f opt %.1f then wait %.1f" % tuple((b - a) * 1e3 for a, b in zip(t, t[1:])),
          flush=True)
    torch.cuda.set_sync_debug_mode(1)
    train_step(model, opt, rgb, dep, lab)
    torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
