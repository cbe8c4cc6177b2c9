#!/usr/bin/env python
"""Per-kernel MFMA utilisation and effective clock from a rocprofv3 --pmc pass
(scripts/pmc_mfma.sh).  Per kernel (mean over launches): duration (kernel trace),
GRBM_GUI_ACTIVE / 8 / duration = effective clock (microarch guide, DVFS note:
the sum over the 8 XCDs), SQ_VALU_MFMA_BUSY_CYCLES / (GUI_ACTIVE/8 x 256 CU x 4
SIMD) = matrix-pipe busy fraction, F64 MFMA count x 2048 flop / duration, and
the SQ wait split (quad-cycles)."""
import csv
import re
import sys
from collections import defaultdict


def name(k):
    return re.sub(r"^void ", "", re.sub(r"\(.*", "", k).strip())


def main(pmc_csv, trace_csv):
    dur = defaultdict(list)
    for r in csv.DictReader(open(trace_csv)):
        dur[name(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(pmc_csv)):
        acc[name(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = []
    for k, c in acc.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        d = sum(dur[k]) / len(dur[k]) if dur.get(k) else float("nan")
        gui = m.get("GRBM_GUI_ACTIVE", float("nan"))
        clk = gui / 8 / d if d else float("nan")           # GHz (cycles per ns)
        mf = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        busy = mf / (gui / 8 * 256 * 4) if gui else float("nan")
        f64 = m.get("SQ_INSTS_VALU_MFMA_F64", 0.0) * 2048
        rows.append((d, k, len(c.get("GRBM_GUI_ACTIVE", [])), clk, busy, f64 / d / 1e3 if d else 0,
                     m.get("SQ_WAIT_ANY", 0) / max(m.get("SQ_WAVE_CYCLES", 1), 1),
                     m.get("SQ_WAIT_INST_ANY", 0) / max(m.get("SQ_WAVE_CYCLES", 1), 1)))
    rows.sort(reverse=True)
    print(f"{'kernel':60s} {'n':>4s} {'us':>9s} {'GHz':>5s} {'mfma_busy':>9s} {'f64TF':>7s} {'wait':>5s} {'instw':>5s}")
    for d, k, n, clk, busy, tf, w, wi in rows[:40]:
        print(f"{k[:60]:60s} {n:4d} {d / 1e3:9.1f} {clk:5.2f} {busy:9.3f} {tf:7.2f} {w:5.2f} {wi:5.2f}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
