"""Sweep the row-streaming 3x3 depthwise kernels' launch geometry (target waves, minimum rows per
chunk) over the DFormer-B bf16 bs=16 480x640 ConvFFN shapes (GPU only, profiling tool).

The sweep needs an experiment build whose w3_geom / f3_geom read a fixed wave target and minimum
chunk height from DFM_X_W3T / DFM_X_W3R (backward) and DFM_X_F3T / DFM_X_F3R (forward), once per
process, so every point runs in its own child process (SWEEP_T / SWEEP_R list the grid). Without
SWEEP_T it times the library's own geometry once.

    SWEEP_T=1536,3072 SWEEP_R=2,4 python tools/dw3_geom_sweep.py   # grid (experiment build)
    python tools/dw3_geom_sweep.py                                  # the built geometry
"""
import json
import os
import subprocess
import sys

SHAPES = [(120, 160, 512), (120, 160, 256), (60, 80, 1024), (60, 80, 512), (30, 40, 1024), (30, 40, 512),
          (15, 20, 2048), (15, 20, 1024)]
COUNT = {0: 2, 1: 2, 2: 12, 3: 2}  # blocks per stage (DFormer-B depths)


def child():
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dformer_amd import kernels as K

    def timed(fn, it=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / it

    dev = torch.device("cuda", 0)
    B = 16
    out = []
    for i, (H, W, C) in enumerate(SHAPES):
        P = B * H * W
        h = torch.randn(P, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(P, C, device=dev).to(torch.bfloat16)
        w = torch.randn(C, 1, 3, 3, device=dev) / 3
        b = torch.randn(C, device=dev) * 0.1
        gp, g, dh = torch.empty_like(h), torch.empty_like(h), torch.empty_like(h)
        f = timed(lambda: K.dwconv(h, (B, H, W), w, b, 3, add_identity=True, out=gp, gelu_out=g, out_gelu_grad=True))
        bw = timed(lambda: K.dwconv_bwd(h, dy, (B, H, W), w, 3, add_identity=True, dx=dh))
        out.append({"shape": [H, W, C], "stage": i // 2, "fwd_us": f, "bwd_us": bw})
    print("JSON " + json.dumps(out), flush=True)


def main():
    grid = []
    if "SWEEP_T" not in os.environ:
        p = subprocess.run([sys.executable, "-u", __file__, "--child"], capture_output=True, text=True, timeout=240)
        rows = json.loads([x for x in p.stdout.splitlines() if x.startswith("JSON ")][0][5:])
        tf = sum(COUNT[x["stage"]] * x["fwd_us"] for x in rows)
        tb = sum(COUNT[x["stage"]] * x["bwd_us"] for x in rows)
        print(f"built geometry: step fwd {tf:7.1f} us  bwd {tb:7.1f} us  | " +
              " ".join(f"{x['fwd_us']:.0f}/{x['bwd_us']:.0f}" for x in rows), flush=True)
        return
    ts = [int(v) for v in os.environ["SWEEP_T"].split(",")]
    rs = [int(v) for v in os.environ.get("SWEEP_R", "2,4,8").split(",")]
    for t in ts:
        for r in rs:
            grid.append((t, r))
    res = {}
    for t, r in grid:
        env = dict(os.environ, DFM_X_W3T=str(t), DFM_X_W3R=str(r), DFM_X_F3T=str(t), DFM_X_F3R=str(r))
        p = subprocess.run([sys.executable, "-u", __file__, "--child"], env=env, capture_output=True, text=True,
                           timeout=240)
        line = [x for x in p.stdout.splitlines() if x.startswith("JSON ")]
        if p.returncode != 0 or not line:
            print(f"T={t} R={r}: failed rc={p.returncode} {p.stderr[-400:]}", flush=True)
            break
        rows = json.loads(line[0][5:])
        res[f"{t},{r}"] = rows
        tf = sum(COUNT[x["stage"]] * x["fwd_us"] for x in rows)
        tb = sum(COUNT[x["stage"]] * x["bwd_us"] for x in rows)
        print(f"T={t:6d} R={r}: step fwd {tf:7.1f} us  bwd {tb:7.1f} us  | " +
              " ".join(f"{x['fwd_us']:.0f}/{x['bwd_us']:.0f}" for x in rows), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/dw3_geom_sweep.json", "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    child() if "--child" in sys.argv else main()
