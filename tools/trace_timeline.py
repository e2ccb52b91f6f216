"""Timeline of the last training step in a rocprofv3 kernel_trace.csv: per launch the start offset
from the step start, duration, queue, grid blocks and short kernel name (profiling tool).
    python tools/trace_timeline.py trace.csv [first_index] [count]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"],
             int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) //
             max(1, int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])))
            for r in rows)
idx = [i for i, k in enumerate(ks) if "adamw" in k[2]]
groups, prev = [], None
for i in idx:
    if prev is None or i != prev + 1:
        groups.append(i)
    prev = i
seg = ks[groups[-2] + 1:groups[-1] + 1] if len(groups) >= 2 else ks
t0 = seg[0][0]
first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
count = int(sys.argv[3]) if len(sys.argv) > 3 else len(seg)
for n, (s, e, name, q, g) in enumerate(seg[first:first + count], first):
    short = re.sub(r"\(anonymous namespace\)::", "", name)
    short = re.sub(r"\((?:[^()]|\([^()]*\))*\)$", "", short).replace("void ", "")
    print(f"{n:5d} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} q{q} {g:7d} {short[:90]}")
