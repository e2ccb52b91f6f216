"""Average duration of one kernel at one grid shape from a rocprofv3 kernel_trace.csv (the
rocprof side of bench.py's live HIP-event roofline; --stats groups all shapes of a template).
    python tools/trace_kernel.py gpurun_out/r01_prof/r01_kernel_trace.csv 'gemm_kernel<unsigned short, 128, 64, 4, 2, 64, true, true, 1>' 614400
"""
import csv
import statistics
import sys

path, name, gx = sys.argv[1], sys.argv[2], sys.argv[3]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(path))
     if name in r["Kernel_Name"] and r["Grid_Size_X"] == gx]
print(f"kernel {name} grid_x={gx}: launches {len(d)}, mean {statistics.mean(d):.2f} us, "
      f"median {statistics.median(d):.2f} us, min {min(d):.2f} us, max {max(d):.2f} us")
