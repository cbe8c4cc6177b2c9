"""Kernel timeline from a rocprofv3 kernel_trace.csv: the last N dispatches with
their durations and the gap since the previous kernel ended.
Usage: python3 scripts/timeline.py run_kernel_trace.csv [N]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    prev = None
    busy = 0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        busy += e - s
        print(f'{r["Kernel_Name"][:58]:58s} grid {r.get("Grid_Size_X", "?"):>7s} '
              f'{(e - s) / 1e3:8.1f} us  gap {gap:6.1f} us')
        prev = e
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    print(f"span {span:.1f} us, kernels busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
