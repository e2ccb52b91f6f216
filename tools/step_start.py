"""The first milliseconds of the last complete training step in a rocprofv3 trace: every kernel (and,
given a memory-copy trace, every copy) with its start relative to the step start, duration, queue
and the idle gap before it. Used to find what the device waits on at a replayed step's start.
Usage: python tools/step_start.py kernel_trace.csv [memory_copy_trace.csv] [window_ms]"""
import csv
import sys

kt = sys.argv[1]
mc = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2].endswith(".csv") else None
win = float(sys.argv[-1]) if not sys.argv[-1].endswith(".csv") else 2.0

ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70],
       "q" + r["Queue_Id"]) for r in csv.DictReader(open(kt))]
if mc:
    for r in csv.DictReader(open(mc)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   f"COPY {r.get('Direction', '')} {r.get('Bytes', r.get('Size', ''))}B", "copy"))
ev.sort()
ad = [i for i, e in enumerate(ev) if "adamw" in e[2]]
# step boundaries: the last AdamW of each consecutive group
ends = [ad[j] for j in range(len(ad)) if j + 1 == len(ad) or ad[j + 1] != ad[j] + 1]
if len(ends) < 3:
    sys.exit("fewer than three steps in the trace")
a, b = ends[-3], ends[-2]  # the step between the last two complete boundaries
t0 = ev[a][1]
print(f"step start = end of {ev[a][2]} at {t0}; window {win} ms")
last_end = t0
for s, e, n, q in ev[a + 1:b + 1]:
    if s - t0 > win * 1e6:
        break
    gap = (s - last_end) / 1e3
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:7.1f}  gap {gap:7.1f}  {q:5s} {n}")
    last_end = max(last_end, e)
