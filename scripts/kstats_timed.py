#!/usr/bin/env python
"""Per-kernel launch durations from a rocprofv3 kernel trace, over all launches and over the
last K launches (the bench's timed steps follow its warmup steps on the same kernels):

    python scripts/kstats_timed.py KERNEL_TRACE_CSV K [name-substring ...]
"""
import csv
import sys


def main(path, k, names):
    rows = list(csv.DictReader(open(path)))
    for nm in names:
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0 for r in rows if nm in r["Kernel_Name"]]
        if not d:
            continue
        last = d[-k:]
        print(f"{nm}: launches {len(d)}  all {sum(d) / len(d):.1f} us  last {len(last)} {sum(last) / len(last):.1f} us"
              f"  min {min(d):.1f}  max {max(d):.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3:] or ["k_gemm128<1>", "k_fleet_control2<false>", "k_gram_rows<11"])
