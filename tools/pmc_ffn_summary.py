"""Summarise tools/pmc_ffn.sh: per kernel, mean of every counter over its launches (+ derived ratios)."""
import csv
import glob
import sys
from collections import defaultdict


def main(tag):
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(f"gpurun_out/{tag}_p*/**/*counter_collection.csv", recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "")[:90]
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(k)
        for c in sorted(m):
            print(f"    {c:28s} {m[c]:16.1f}")
        if "SQ_WAVE_CYCLES" in m and m.get("SQ_WAVES"):
            print(f"    VALU-active / wave-cycles   {m.get('SQ_ACTIVE_INST_VALU', 0) / m['SQ_WAVE_CYCLES']:.3f}")
            print(f"    wait-any / wave-cycles      {m.get('SQ_WAIT_ANY', 0) / m['SQ_WAVE_CYCLES']:.3f}")
        if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
            print(f"    HBM bytes (2*FETCH+WRITE KiB) {(2 * m.get('FETCH_SIZE', 0) + m.get('WRITE_SIZE', 0)) * 1024 / 1e6:.1f} MB")


if __name__ == "__main__":
    main(sys.argv[1])
