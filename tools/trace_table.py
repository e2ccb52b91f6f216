"""Per-step tables from a rocprofv3 --kernel-trace CSV of bench.py (tools/trace_step.sh).

Splits the dispatch stream into training steps at the AdamW kernel (the last launch of a step),
keeps the last complete step, and prints: the step's device span (first start -> last end), the
sum of kernel durations, and the kernels grouped by (name, grid) with count / total / mean.

    python tools/trace_table.py gpurun_out/r03a_eager/.../k_kernel_trace.csv [--top 60] [--json out.json]
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"\((?:[^()]|\([^()]*\))*\)$", "", name)  # argument list
    return name.replace("unsigned short", "bf16").replace("void ", "")


def load(path):
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def steps(rows):
    out, cur = [], []
    for r in rows:
        cur.append(r)
        if "adamw" in r["Kernel_Name"]:
            out.append(cur)
            cur = []
    # a step has two AdamW launches (decay / no-decay groups): merge pairs
    merged = []
    for s in out:
        if merged and len(s) <= 2:
            merged[-1].extend(s)
        else:
            merged.append(s)
    return merged


def table(step):
    g = collections.OrderedDict()
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        grid = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        k = (short(r["Kernel_Name"]), grid)
        e = g.setdefault(k, [0, 0.0])
        e[0] += 1
        e[1] += d
    return g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--json", default=None)
    ap.add_argument("--by-name", action="store_true", help="group by kernel name only")
    a = ap.parse_args()
    rows = load(a.trace)
    st = steps(rows)
    print(f"{len(rows)} dispatches, {len(st)} steps; step sizes {[len(s) for s in st]}")
    s = st[-2] if len(st) >= 2 else st[-1]
    t0 = int(s[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in s)
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s) / 1e6
    print(f"step: {len(s)} kernels, span {(t1 - t0) / 1e6:.3f} ms, sum of kernel durations {busy:.3f} ms")
    g = table(s)
    if a.by_name:
        h = collections.OrderedDict()
        for (n, _), (c, t) in g.items():
            e = h.setdefault((n, "*"), [0, 0.0])
            e[0] += c
            e[1] += t
        g = h
    items = sorted(g.items(), key=lambda kv: -kv[1][1])
    for (n, grid), (c, t) in items[:a.top]:
        print(f"{t / 1e3:8.3f} ms {c:4d}x {t / c:8.2f} us  grid {grid:>9}  {n[:120]}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"span_ms": (t1 - t0) / 1e6, "busy_ms": busy, "kernels": len(s),
                       "rows": [{"name": n, "grid": grid, "count": c, "total_us": t} for (n, grid), (c, t) in items]},
                      f, indent=1)


if __name__ == "__main__":
    main()
