"""Per-step kernel time by family from a rocprofv3 --stats kernel_stats.csv (steps = profiled steps)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 6
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / steps / 1e6:.2f} ms/step")
fam = {}
for r in rows:
    n = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "")
    key = n.split("<")[0].split("(")[0][:48]
    fam[key] = fam.get(key, 0) + float(r["TotalDurationNs"]) / steps / 1e6
for k, v in sorted(fam.items(), key=lambda x: -x[1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{v:7.2f} ms  {k}")
