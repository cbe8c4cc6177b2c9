"""Summaries of rocprofv3 output (kernel traces, --stats, --pmc counter CSVs):

  traffic FETCH_CSV WRITE_CSV OUT_JSON   per-launch HBM bytes per kernel from two --pmc passes
                                          (FETCH_SIZE x2: the gfx950 streaming-read correction of
                                          MI355X_MICROARCH.md's HBM section; WRITE_SIZE as is)
  mfma PMC_CSV TRACE_CSV                 per kernel: duration, effective clock (GRBM_GUI_ACTIVE / 8
                                          XCDs / duration), matrix-pipe busy (SQ_VALU_MFMA_BUSY_CYCLES /
                                          (GUI_ACTIVE / 8 x 256 CU x 4 SIMD)), F64 MFMA TFLOP/s, waits
  sum PMC_CSV PREFIX                     mean per launch of every counter, kernels starting with PREFIX
  top STATS_CSV [n]                      the n longest kernels of a --stats summary
  kstats TRACE_CSV K [names..]           per-kernel mean duration over all launches and the last K
  timeline TRACE_CSV [n]                 the last n dispatches with durations and gaps
  launches TRACE_CSV names..             every launch of the named kernels with its grid
"""
import csv
import json
import re
import sys
from collections import defaultdict


def _name(k):
    return re.sub(r"^void ", "", re.sub(r"\(.*", "", k).strip())


def _rows(path):
    return list(csv.DictReader(open(path)))


def _dur(r):
    return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def traffic(fetch_csv, write_csv, out_json):
    def per_kernel(path, counter):
        acc = defaultdict(list)
        for r in _rows(path):
            if r["Counter_Name"] == counter:
                acc[_name(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
        return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}

    f, nf = per_kernel(fetch_csv, "FETCH_SIZE")
    w, _ = per_kernel(write_csv, "WRITE_SIZE")
    out = {}
    for k in sorted(set(f) | set(w)):
        fb, wb = 2.0 * f.get(k, 0.0), w.get(k, 0.0)
        out[k] = dict(launches=nf.get(k, 0), fetch_bytes=fb, write_bytes=wb, traffic_bytes=fb + wb)
    json.dump({"note": "bytes per launch; FETCH_SIZE x2 (gfx950 streaming-read correction), WRITE_SIZE as is",
               "kernels": out}, open(out_json, "w"), indent=1)


def mfma(pmc_csv, trace_csv):
    dur = defaultdict(list)
    for r in _rows(trace_csv):
        dur[_name(r["Kernel_Name"])].append(_dur(r))
    acc = defaultdict(lambda: defaultdict(list))
    for r in _rows(pmc_csv):
        acc[_name(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = []
    for k, c in acc.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        d = sum(dur[k]) / len(dur[k]) if dur.get(k) else float("nan")
        gui = m.get("GRBM_GUI_ACTIVE", float("nan"))
        wc = max(m.get("SQ_WAVE_CYCLES", 1), 1)
        rows.append((d, k, len(c.get("GRBM_GUI_ACTIVE", [])), gui / 8 / d if d else float("nan"),
                     m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui / 8 * 256 * 4) if gui else float("nan"),
                     m.get("SQ_INSTS_VALU_MFMA_F64", 0.0) * 2048 / d / 1e3 if d else 0.0,
                     m.get("SQ_WAIT_ANY", 0) / wc, m.get("SQ_WAIT_INST_ANY", 0) / wc))
    rows.sort(reverse=True)
    print(f"{'kernel':60s} {'n':>4s} {'us':>9s} {'GHz':>5s} {'mfma_busy':>9s} {'f64TF':>7s} {'wait':>5s} {'instw':>5s}")
    for d, k, n, clk, busy, tf, w, wi in rows[:40]:
        print(f"{k[:60]:60s} {n:4d} {d / 1e3:9.1f} {clk:5.2f} {busy:9.3f} {tf:7.2f} {w:5.2f} {wi:5.2f}")


def sum_(pmc_csv, prefix):
    acc = defaultdict(lambda: defaultdict(float))
    launches = defaultdict(set)
    for r in _rows(pmc_csv):
        name = _name(r["Kernel_Name"])
        if name.startswith(prefix):
            acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
            launches[name].add(r["Dispatch_Id"])
    for k, cs in sorted(acc.items()):
        n = max(1, len(launches[k]))
        print(k, f"launches={n}")
        for c, v in sorted(cs.items()):
            print(f"  {c:40s} {v / n:16.1f}")


def top(stats_csv, n="12"):
    for r in _rows(stats_csv)[:int(n)]:
        print(f'{r["Name"][:60]:60s} {int(r["Calls"]):6d} {float(r["AverageNs"]) / 1e3:9.1f} us '
              f'{float(r["Percentage"]):6.2f}%')


def kstats(trace_csv, k, *names):
    rows = _rows(trace_csv)
    for nm in names or ("k_gemm128<1>", "k_fleet_control2<false>", "k_gram_rows<11"):
        d = [_dur(r) / 1000.0 for r in rows if nm in r["Kernel_Name"]]
        if d:
            last = d[-int(k):]
            print(f"{nm}: launches {len(d)}  all {sum(d) / len(d):.1f} us  last {len(last)} "
                  f"{sum(last) / len(last):.1f} us  min {min(d):.1f}  max {max(d):.1f}")


def timeline(trace_csv, n="40"):
    rows = sorted(_rows(trace_csv), key=lambda r: int(r["Start_Timestamp"]))[-int(n):]
    prev, busy = None, 0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        busy += e - s
        print(f'{r["Kernel_Name"][:58]:58s} grid {r.get("Grid_Size_X", "?"):>7s} {(e - s) / 1e3:8.1f} us  gap {gap:6.1f} us')
        prev = e
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    print(f"span {span:.1f} us, kernels busy {busy / 1e3:.1f} us")


def launches(trace_csv, *keys):
    for r in _rows(trace_csv):
        n = r["Kernel_Name"]
        if any(k in n for k in keys):
            grid = "x".join(r.get(f"Grid_Size_{a}", "?") for a in "XYZ")
            print(f"{n[:44]:44s} {grid:>16s} {_dur(r) / 1e3:10.1f} us")


def qpstamps(log):
    """GPMPC_QP_STAMPS=1 stderr lines of k_qp_batched (problem 0's phase cycles), averaged."""
    rows = [l.split() for l in open(log) if l.startswith("qp_stamps")]
    it = [int(r[2].rstrip(":")) for r in rows]
    v = [[int(x) for x in r[3:]] for r in rows]
    n = len(rows)
    m = [sum(c) / n for c in zip(*v)]
    ni = sum(it) / n
    print(f"{n} solves, iterations mean {ni:.2f} (min {min(it)}, max {max(it)})")
    names = {1: "clip+scale", 2: "rho+factor", 3: "rhs", 8: "fwd chain (+diag if fused)", 9: "diag / fence",
             10: "backward chain", 4: "post-solve barrier", 5: "z/y update", 6: "check/adapt", 7: "final"}
    for k in [1, 2, 3, 8, 9, 10, 4, 5, 6, 7]:
        print(f"{names[k]:28s} {m[k]:10.0f} cycles {m[k] / m[15] * 100:5.1f}%  per iteration {m[k] / ni:7.0f}")
    print(f"total {m[15]:.0f} shader cycles, {m[14] / 100:.1f} us (100 MHz constant clock)")


COMMANDS = dict(traffic=traffic, mfma=mfma, sum=sum_, top=top, kstats=kstats, timeline=timeline, launches=launches,
                qpstamps=qpstamps)

if __name__ == "__main__":
    if len(sys.argv) < 2 or sys.argv[1] not in COMMANDS:
        sys.exit(__doc__)
    COMMANDS[sys.argv[1]](*sys.argv[2:])
