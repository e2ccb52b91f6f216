"""HBM traffic and MFMA busy of the step's measured-dominant kernel, from rocprofv3 PMC passes over
bench.py's own eager steps (every shape the step launches the kernel with), against the census's
algorithmic bytes for the same launches -> profiles/<round>_dominant_pmc.json (read by bench.py).

  rocprofv3 --pmc FETCH_SIZE --kernel-include-regex <re> -d <fetch_dir> -- python3 bench.py --eager ...
  rocprofv3 --pmc WRITE_SIZE ...                       -d <write_dir> ...
  rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE ... -d <mfma_dir> ...
  python tools/pmc_dominant.py <step_table.json> <fetch_dir> <write_dir> <mfma_dir> <out.json> [kernel substring]

With a kernel substring the record is for the first census kernel whose name contains it instead of
the dominant one (e.g. the 7x7 depthwise / MFMA attention kernels, tools/gpu_pmc_kernels.sh).

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB counters; on gfx950 FETCH_SIZE counts wide
streaming reads at half their bytes, MI355X_MICROARCH.md HBM section). MFMA busy = the per-SIMD
share of GUI-active cycles the MFMA pipe was busy (SQ_VALU_MFMA_BUSY_CYCLES is summed over the
1024 SIMDs of the chip, GRBM_GUI_ACTIVE over its 8 XCDs)."""
import csv
import glob
import json
import sys


def counter_rows(d, counter, name):
    vals = []
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") == counter and row.get("Kernel_Name", "").startswith(name[:80]):
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    table_path, fdir, wdir, mdir, out = sys.argv[1:6]
    sub = sys.argv[6] if len(sys.argv) > 6 else None
    with open(table_path) as f:
        table = json.load(f)
    if sub:
        name, row = next((k, r) for k, r in table["kernels"].items() if sub in k)
    else:
        name, row = next(iter(table["kernels"].items()))  # sorted by measured time: the dominant kernel
    algo = row["bytes"] / row["launches"]
    flops = row["flops"] / row["launches"]
    fetch = counter_rows(fdir, "FETCH_SIZE", name)
    write = counter_rows(wdir, "WRITE_SIZE", name)
    busy = counter_rows(mdir, "SQ_VALU_MFMA_BUSY_CYCLES", name)
    gui = counter_rows(mdir, "GRBM_GUI_ACTIVE", name)
    if not fetch or not write:
        raise SystemExit(f"no FETCH_SIZE / WRITE_SIZE rows for {name[:80]}")
    rd = 2 * sum(fetch) / len(fetch) * 1024
    wr = sum(write) / len(write) * 1024
    ms = row["measured_ms"] / row["launches"]
    rec = {"kernel": name, "launches_profiled": [len(fetch), len(write), len(busy)],
           "census_ms_per_launch": round(ms, 4),
           "algorithmic_GBs": round(algo / ms / 1e6, 1), "algorithmic_frac_of_8TBs": round(algo / ms / 1e6 / 8000, 4),
           "census_launches_per_step": row["launches"],
           "algorithmic_bytes_per_launch": round(algo), "algorithmic_flops_per_launch": round(flops),
           "hbm_read_bytes_per_launch": round(rd), "hbm_write_bytes_per_launch": round(wr),
           "traffic_bytes_per_launch": round(rd + wr), "traffic_over_algorithmic": round((rd + wr) / algo, 3),
           # SQ_VALU_MFMA_BUSY_CYCLES summed over the 1024 SIMDs, GRBM_GUI_ACTIVE over the 8 XCDs
           # (MI355X_MICROARCH.md): busy share of a SIMD's cycles while the kernel ran
           "mfma_busy_per_simd": round(8 * sum(busy) / max(sum(gui), 1) / 1024, 4) if busy and gui else None,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_VALU_MFMA_BUSY_CYCLES+GRBM_GUI_ACTIVE in separate "
                     "passes over bench.py --eager steps, filtered to the kernel; FETCH_SIZE x2 (gfx950); "
                     "averages over every launch of the kernel in the profiled steps"}
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
