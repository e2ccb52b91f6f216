"""Average duration of one kernel at one grid shape from a rocprofv3 kernel_trace.csv (the
rocprof side of bench.py's live HIP-event roofline; --stats groups all shapes of a template).
A persistent kernel launches the same grid for every shape, so an optional MIN_US keeps only the
launches at least that long (the dominant shape's duration cluster).
    python tools/trace_kernel.py gpurun_out/r01b_prof/r01b_kernel_trace.csv 'gemm_stream_kernel<unsigned short, 128, 64' 131072 100
"""
import csv
import statistics
import sys

path, name, gx = sys.argv[1], sys.argv[2], sys.argv[3]
min_us = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(path))
     if name in r["Kernel_Name"] and r["Grid_Size_X"] == gx]
d = [t for t in d if t >= min_us]
print(f"kernel {name} grid_x={gx} (launches >= {min_us} us): launches {len(d)}, mean {statistics.mean(d):.2f} us, "
      f"median {statistics.median(d):.2f} us, min {min(d):.2f} us, max {max(d):.2f} us")
