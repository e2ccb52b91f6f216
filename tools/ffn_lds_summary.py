"""Summarise tools/ffn_lds_pmc.sh: per skip mask and kernel, per-wave LDS instructions, LDS-array
cycles, bank-conflict cycles and VALU instructions (median over dispatches)."""
import collections
import csv
import glob
import re
import statistics
import sys

pre = sys.argv[1]
for path in sorted(glob.glob(f"{pre}_m*")):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(path + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            m = re.search(r"(convffn_\w+_kernel)<([^>]*)>", row["Kernel_Name"])
            if m:
                vals[m.group(1) + "<" + m.group(2) + ">"][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in sorted(vals.items()):
        g = {c: statistics.median(v) for c, v in cs.items()}
        w = g["SQ_WAVES"]
        print(f"{path.split('_')[-1]:4s} {k:40s} lds/wave {g['SQ_INSTS_LDS'] / w:7.0f}  lds_active/wave "
              f"{g['SQ_LDS_IDX_ACTIVE'] / w:8.0f}  conflict/wave {g['SQ_LDS_BANK_CONFLICT'] / w:8.0f}  valu/wave "
              f"{g['SQ_INSTS_VALU'] / w:7.0f}  wave_cycles/wave {g['SQ_WAVE_CYCLES'] / w:8.0f}  wait_lds "
              f"{g['SQ_WAIT_INST_LDS'] / g['SQ_WAVE_CYCLES']:.2f}")
