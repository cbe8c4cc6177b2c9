"""Summarise GPMPC_QP_STAMPS=1 stderr lines of k_qp_batched (problem 0's phase cycles).
python3 scripts/qp_stamps.py LOG"""
import sys

import numpy as np

rows = [l.split() for l in open(sys.argv[1]) if l.startswith("qp_stamps")]
it = np.array([int(r[2].rstrip(":")) for r in rows])
v = np.array([[int(x) for x in r[3:]] for r in rows], float)
print(f"{len(rows)} solves, iterations mean {it.mean():.2f} (min {it.min()}, max {it.max()})")
m = v.mean(0)
names = {1: "clip+scale", 2: "rho+factor", 3: "rhs", 8: "fwd chain (+diag if fused)", 9: "diag / fence",
         10: "backward chain", 4: "post-solve barrier", 5: "z/y update", 6: "check/adapt", 7: "final"}
for k in [1, 2, 3, 8, 9, 10, 4, 5, 6, 7]:
    print(f"{names[k]:28s} {m[k]:10.0f} cycles {m[k] / m[15] * 100:5.1f}%  per iteration {m[k] / it.mean():7.0f}")
print(f"total {m[15]:.0f} shader cycles, {m[14] / 100:.1f} us (100 MHz constant clock)")
