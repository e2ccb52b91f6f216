"""Host-side cost of one graph replay of the default bench step: is the replayed step host-bound?

Times graph.replay() on the host (perf_counter, no sync) for back-to-back replays and for a replay
issued onto an idle GPU, next to the per-step GPU time from HIP events. If the host needs about as
long to issue a replay as the GPU needs to run it, the GPU catches up with the host and idles at
the start of each step (the gaps seen between the stem kernels in the round-6 traces)."""
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

import bench  # noqa: E402
from dformer_amd.segmentor import EncoderDecoder  # noqa: E402
from dformer_amd.train import FusedAdamW, GraphedTrainStep  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(8964)
    cfg = bench.make_cfg("DFormer-Base", "ham", 40)
    model = EncoderDecoder(cfg=cfg, syncbn=False).to(dev).set_compute_dtype(torch.bfloat16)
    model.return_logits = False
    model.train()
    opt = FusedAdamW(model, lr=cfg.lr, weight_decay=cfg.weight_decay, world=1, compute_dtype=torch.bfloat16)
    rgb, dep, lab = bench.synthetic_batch(16, 480, 640, 40, dev, 8964)
    step = GraphedTrainStep(model, opt, rgb, dep, lab)
    for _ in range(3):
        step()
    torch.cuda.synchronize()

    idle = []
    for _ in range(5):  # one replay onto an idle GPU
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        idle.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()

    n = 12
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    host = []
    ev[0].record(s)
    t_all = time.perf_counter()
    for i in range(n):
        t0 = time.perf_counter()
        step()
        host.append((time.perf_counter() - t0) * 1e3)
        ev[i + 1].record(s)
    t_issue = (time.perf_counter() - t_all) * 1e3
    torch.cuda.synchronize()
    t_wall = (time.perf_counter() - t_all) * 1e3
    gpu = [ev[i].elapsed_time(ev[i + 1]) for i in range(n)]
    # replays queued behind a long sleep: the host issues them while the GPU is busy, so the GPU
    # runs them without waiting on the host (compare the per-step GPU time with the loop above)
    torch.cuda.synchronize()
    ev2 = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    for _ in range(60):  # ~100 ms of matmuls: keeps the clocks up while the host queues the replays
        torch.mm(a, a)
    ev2[0].record(s)
    t0 = time.perf_counter()
    hq = []
    for i in range(3):
        t1 = time.perf_counter()
        step()
        hq.append((time.perf_counter() - t1) * 1e3)
        ev2[i + 1].record(s)
    t_q = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    gq = [ev2[i].elapsed_time(ev2[i + 1]) for i in range(3)]
    print(f"behind a sleep: host ms per replay {[round(x, 2) for x in hq]} (issue {t_q:.1f} ms), "
          f"GPU ms per step {[round(x, 2) for x in gq]}")
    print(f"replay onto idle GPU: host ms {[round(x, 2) for x in idle]}")
    print(f"back-to-back host ms per replay: {[round(x, 2) for x in host]}")
    print(f"back-to-back GPU ms per step:    {[round(x, 2) for x in gpu]}")
    print(f"issue of {n} replays {t_issue:.1f} ms, wall to drain {t_wall:.1f} ms, "
          f"median host {statistics.median(host):.2f} ms vs GPU {statistics.median(gpu):.2f} ms")


if __name__ == "__main__":
    main()
