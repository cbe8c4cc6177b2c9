"""Per-launch durations from a rocprofv3 kernel trace (run_kernel_trace.csv): every launch of
the kernels whose names contain any of the given substrings, in order, with its grid.
  python3 scripts/trace_launches.py TRACE.csv updsolve k_potrf_diag128 k_gemm128"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
keys = sys.argv[2:]
for r in rows:
    n = r["Kernel_Name"]
    if any(k in n for k in keys):
        grid = "x".join(r.get(f"Grid_Size_{a}", "?") for a in "XYZ")
        print(f"{n[:44]:44s} {grid:>16s} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:10.1f} us")
