"""Turn two rocprofv3 PMC passes over tools/dominant_kernel.py into profiles/<round>_dominant_pmc.json.

HBM traffic per launch = 2 x FETCH_SIZE + WRITE_SIZE: on gfx950 FETCH_SIZE counts wide coalesced
streaming reads at half their bytes (MI355X_MICROARCH.md, HBM section); both counters are in KiB.
    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r01_dominant_pmc.json
"""
import csv
import glob
import json
import statistics
import sys


def per_launch(d, counter):
    vals = []
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if "gemm_" in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for a gemm kernel under {d}")
    return statistics.median(vals), len(vals)


def main():
    fdir, wdir, out = sys.argv[1:4]
    M, N, Kd = 16 * 120 * 160, 64, 512
    fetch_kib, nf = per_launch(fdir, "FETCH_SIZE")
    write_kib, nw = per_launch(wdir, "WRITE_SIZE")
    fetch = 2 * fetch_kib * 1024
    write = write_kib * 1024
    algo = 2 * (M * Kd + N * Kd + 3 * M * N)
    rec = {"key": [M, N, Kd, 1, 1], "kernel": "gemm_stream_kernel bf16 fc2 stage0 (persistent M-streaming, fused bias+residual epilogue)",
           "fetch_size_kib_median": fetch_kib, "write_size_kib_median": write_kib, "launches": [nf, nw],
           "hbm_read_bytes_per_launch": fetch, "hbm_write_bytes_per_launch": write,
           "traffic_bytes_per_launch": fetch + write, "algorithmic_bytes_per_launch": algo,
           "traffic_over_algorithmic": round((fetch + write) / algo, 3),
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH_SIZE x2 (gfx950)"}
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
