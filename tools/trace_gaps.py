"""Idle-gap analysis of a rocprofv3 kernel trace: splits the trace into steps at AdamW launches
(the last kernel of a training step), and per step reports wall time, the union of kernel busy
intervals, idle time, the number of launches and how much of the step ran with >1 kernel in flight.
Usage: python tools/trace_gaps.py kernel_trace.csv [marker-substring]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "adamw"
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows))
ends = [i for i, k in enumerate(ks) if marker in k[2]]
# a step ends at the last marker launch of a consecutive group
bounds, prev = [], None
for i in ends:
    if prev is not None and i != prev + 1 and (not bounds or bounds[-1] != prev):
        bounds.append(prev)
    prev = i
if prev is not None:
    bounds.append(prev)
start = 0
for b in bounds:
    seg = ks[start:b + 1]
    start = b + 1
    if len(seg) < 100:
        continue
    t0, t1 = seg[0][0], max(k[1] for k in seg)
    busy, cur_s, cur_e, overlap = 0, None, None, 0
    ev = sorted([(k[0], 1) for k in seg] + [(k[1], -1) for k in seg])
    depth, last = 0, t0
    for t, d in ev:
        if depth > 0:
            busy += t - last
        if depth > 1:
            overlap += t - last
        depth += d
        last = t
    wall = t1 - t0
    queues = sorted({k[3] for k in seg})
    print(f"step: {len(seg)} launches, wall {wall/1e6:.2f} ms, busy {busy/1e6:.2f} ms, idle {(wall-busy)/1e6:.2f} ms "
          f"({100*(wall-busy)/wall:.1f}%), >1 kernel in flight {overlap/1e6:.2f} ms, queues {queues}")
