"""HBM traffic and MFMA busy of several kernels of the training step, from unfiltered rocprofv3 PMC
passes over bench.py's eager steps, each against the census's algorithmic bytes / FLOPs for the same
launches (bench.py --table-out). Writes <out_prefix>_<tag>.json per kernel and, for the step's
measured-dominant kernel (first table row), <out_prefix>_dominant.json (read by bench.py).

  rocprofv3 --pmc FETCH_SIZE -d <fetch_dir> -- python3 bench.py --eager ...          (one pass each)
  rocprofv3 --pmc WRITE_SIZE -d <write_dir> ...
  rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d <mfma_dir> ...
  python tools/pmc_kernels.py <step_table.json> <fetch_dir> <write_dir> <mfma_dir> <out_prefix> tag=regex ...

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB counters; FETCH_SIZE counts wide streaming reads
at half their bytes on gfx950, MI355X_MICROARCH.md HBM section). MFMA busy = per-SIMD share of the
GUI-active cycles (SQ_VALU_MFMA_BUSY_CYCLES summed over 1024 SIMDs, GRBM_GUI_ACTIVE over 8 XCDs)."""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

PEAK_TFS = {"bf16": 2500.0, "f32": 157.3}
HBM = 8000.0


def load(d, counters):
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") in counters:
                    vals[row["Counter_Name"]][row.get("Kernel_Name", "")].append(float(row["Counter_Value"]))
    return vals


def pick(vals, name):
    out = []
    for k, v in vals.items():
        if k.startswith(name[:80]):
            out += v
    return out


def summarize(name, row, fetch, write, mfma):
    n = max(row["launches"], 1)
    algo, flops = row["bytes"] / n, row["flops"] / n
    f, w = pick(fetch["FETCH_SIZE"], name), pick(write["WRITE_SIZE"], name)
    busy, gui = pick(mfma["SQ_VALU_MFMA_BUSY_CYCLES"], name), pick(mfma["GRBM_GUI_ACTIVE"], name)
    rec = {"kernel": name, "census_launches_per_step": row["launches"], "census_ms_per_step": round(row["measured_ms"], 4),
           "algorithmic_bytes_per_launch": round(algo), "algorithmic_flops_per_launch": round(flops),
           "ideal_us_per_launch": round(row["ideal_ms"] / n * 1e3, 3), "peak": row["peak"]}
    if f and w:
        rd, wr = 2 * sum(f) / len(f) * 1024, sum(w) / len(w) * 1024
        rec.update(hbm_read_bytes_per_launch=round(rd), hbm_write_bytes_per_launch=round(wr),
                   traffic_bytes_per_launch=round(rd + wr),
                   traffic_over_algorithmic=round((rd + wr) / algo, 3) if algo else None,
                   launches_profiled=[len(f), len(w), len(busy)])
    if busy and gui:
        rec["mfma_busy_per_simd"] = round(8 * sum(busy) / max(sum(gui), 1) / 1024, 4)
    us = row["measured_ms"] / n * 1e3
    rec["census_us_per_launch"] = round(us, 3)
    rec["hbm_GBs_algorithmic"] = round(algo / (us * 1e-6) / 1e9, 1) if us else None
    rec["TFs_algorithmic"] = round(flops / (us * 1e-6) / 1e12, 2) if us else None
    rec["roofline_frac_exact"] = round(row["ideal_ms"] / max(row["measured_ms"], 1e-12), 4)
    rec["method"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_VALU_MFMA_BUSY_CYCLES+GRBM_GUI_ACTIVE in separate "
                     "unfiltered passes over bench.py --eager steps; FETCH_SIZE x2 (gfx950); averages over every "
                     "launch of the kernel; roofline_frac_exact = sum over launches of max(F/P, B/BW) / census time")
    return rec


def main():
    table_path, fdir, wdir, mdir, prefix = sys.argv[1:6]
    table = json.load(open(table_path))["kernels"]
    fetch, write = load(fdir, {"FETCH_SIZE"}), load(wdir, {"WRITE_SIZE"})
    mfma = load(mdir, {"SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"})
    name, row = next(iter(table.items()))
    rec = summarize(name, row, fetch, write, mfma)
    json.dump(rec, open(f"{prefix}_dominant.json", "w"), indent=1)
    print("dominant", json.dumps(rec)[:400])
    for spec in sys.argv[6:]:
        tag, rx = spec.split("=", 1)
        hits = [(k, v) for k, v in table.items() if re.search(rx, k)]
        if not hits:
            print("no table row for", tag, rx)
            continue
        recs = [summarize(k, v, fetch, write, mfma) for k, v in hits]
        json.dump(recs, open(f"{prefix}_{tag}.json", "w"), indent=1)
        for r in recs:
            print(tag, r["kernel"][:70], r.get("traffic_over_algorithmic"), r.get("mfma_busy_per_simd"),
                  r["roofline_frac_exact"])


if __name__ == "__main__":
    main()
