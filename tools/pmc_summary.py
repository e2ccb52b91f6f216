"""Summarise rocprofv3 PMC passes (counter_collection.csv under <prefix>_p*/) per kernel: the
median per-dispatch value of every counter, plus derived ratios. Profiling tool.
    python tools/pmc_summary.py gpurun_out/g1 [kernel-substring]
"""
import collections
import csv
import glob
import statistics
import sys


def main():
    pre = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(f"{pre}_p*/**/*counter_collection.csv", recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "")
                if sub in k:
                    vals[k.split("(")[0][:90]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in vals.items():
        m = {c: statistics.median(v) for c, v in cs.items()}
        print(k)
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:14.0f}")
        g = lambda c: m.get(c, float("nan"))
        print(f"   busy-per-wave-cycle: wait_any {g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.2f} "
              f"wait_inst {g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES'):.2f} "
              f"active {g('SQ_ACTIVE_INST_ANY') / g('SQ_WAVE_CYCLES'):.2f}; "
              f"lds conflict/active {g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):.2f}; "
              f"L2 hit {g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.2f}; "
              f"mfma busy/gui {g('SQ_VALU_MFMA_BUSY_CYCLES') / g('GRBM_GUI_ACTIVE') / 1024:.2f} (per SIMD); "
              f"fetch {2 * g('FETCH_SIZE') / 1024:.1f} MB")


if __name__ == "__main__":
    main()
