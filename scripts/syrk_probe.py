"""The config-5 FITC SYRK (B = I + A A^T, A 2000 x 4000) alone, 30 timed launches:
min / median ms and FP64 fraction.  For A/B over library builds (GPMPC_LIB)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gp_mpc_rocket_landing_amd import _lib  # noqa: E402

if __name__ == "__main__":
    ctx = _lib.Context(0)
    stream = torch.cuda.ExternalStream(ctx.stream)
    m2, k2 = 2000, 4000
    g = torch.Generator(device="cuda").manual_seed(3)
    As = torch.randn(m2, k2, dtype=torch.float64, device="cuda", generator=g) / k2 ** 0.5
    Bm = torch.eye(m2, dtype=torch.float64, device="cuda")
    ts = []
    for it in range(33):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        _lib._chk(_lib._L.gpmpc_syrk_batched_dev(ctx.h, m2, k2, 1, As.data_ptr(), k2, 0, Bm.data_ptr(),
                                                 m2, 0, 1.0, 1.0), "syrk")
        e1.record(stream)
        ctx.sync()
        if it >= 3:
            ts.append(e0.elapsed_time(e1) * 1e-3)
    fl = m2 * (m2 + 1) * k2
    print(json.dumps({"min_ms": round(min(ts) * 1e3, 4), "median_ms": round(float(np.median(ts)) * 1e3, 4),
                      "frac_min": round(fl / min(ts) / 1e12 / 78.6, 4),
                      "frac_median": round(fl / float(np.median(ts)) / 1e12 / 78.6, 4)}))
