"""Per-kernel time of the last N training steps of a rocprofv3 kernel trace (steps split at AdamW
launches): launches per step, ms per step, mean us. Usage: python tools/trace_top.py trace.csv [N] [top]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
N = int(sys.argv[2]) if len(sys.argv) > 2 else 3
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // max(1, int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"]))) for r in rows))
idx = [i for i, k in enumerate(ks) if "adamw" in k[2]]
# last N steps: after the (N+1)-th last adamw group
groups, prev = [], None
for i in idx:
    if prev is None or i != prev + 1:
        groups.append(i)
    prev = i
start = groups[-N - 1] + 1 if len(groups) > N else 0
seg = ks[start:]
tot = defaultdict(lambda: [0, 0.0])
for s, e, n, g in seg:
    short = re.sub(r"\(anonymous namespace\)::", "", n)
    short = re.sub(r"\((?:[^()]|\([^()]*\))*\)$", "", short)
    tot[short][0] += 1
    tot[short][1] += (e - s) / 1e3
allms = sum(v[1] for v in tot.values()) / N / 1e3
print(f"{N} steps, kernel time {allms:.2f} ms/step, {len(seg) / N:.0f} launches/step")
for n, (c, us) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{c / N:6.0f} {us / N / 1e3:7.3f} ms {us / c:8.1f} us  {n[:120]}")
