"""Idle-gap analysis of a rocprofv3 kernel trace: splits the trace into steps at AdamW launches
(the last kernel of a training step), and per step reports wall time, the union of kernel busy
intervals, idle time, the number of launches and how much of the step ran with >1 kernel in flight;
per hardware queue its busy time and, with --queues, its largest kernels (the queue busy for about
the whole step is the critical path: time saved on the other one only fills overlap).
Usage: python tools/trace_gaps.py kernel_trace.csv [marker-substring] [--queues]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
args = [a for a in sys.argv[2:] if not a.startswith("--")]
marker = args[0] if args else "adamw"
show_q = "--queues" in sys.argv
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
    for q in queues:
        qs = sorted((k for k in seg if k[3] == q))
        qb, ce = 0, None
        for a, e, _, _ in qs:  # union of this queue's intervals
            if ce is None or a > ce:
                qb += e - a
                ce = e
            elif e > ce:
                qb += e - ce
                ce = e
        print(f"  queue {q}: {len(qs)} launches, busy {qb/1e6:.2f} ms")
        if show_q:
            tot = {}
            for a, e, n, _ in qs:
                n = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:90]
                c, t = tot.get(n, (0, 0))
                tot[n] = (c + 1, t + e - a)
            for n, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1])[:15]:
                print(f"    {c:4d} {t/1e6:7.3f} ms  {n}")
