#!/usr/bin/env python
"""Per-launch HBM traffic per kernel from two rocprofv3 --pmc passes.

    python scripts/pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON

FETCH_SIZE and WRITE_SIZE (KB, TCC memory-side requests) need separate passes
on gfx950 (TCC slots).  Per MI355X_MICROARCH.md (HBM section) FETCH_SIZE
counts exactly half the bytes of wide coalesced streaming reads on gfx950, so
it is doubled; WRITE_SIZE is taken as is.  Output: per kernel the mean over
its launches of corrected fetch, write and total bytes.
"""
import csv
import json
import re
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = re.sub(r"^void ", "", re.sub(r"\(.*", "", r["Kernel_Name"]).strip())
        acc[name].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main(fetch_csv, write_csv, out_json):
    f, nf = per_kernel(fetch_csv, "FETCH_SIZE")
    w, _ = per_kernel(write_csv, "WRITE_SIZE")
    out = {}
    for k in sorted(set(f) | set(w)):
        fb = 2.0 * f.get(k, 0.0)
        wb = w.get(k, 0.0)
        out[k] = dict(launches=nf.get(k, 0), fetch_bytes=fb, write_bytes=wb, traffic_bytes=fb + wb)
    json.dump({"note": "bytes per launch; FETCH_SIZE x2 (gfx950 streaming-read correction), WRITE_SIZE as is",
               "kernels": out}, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:4])
