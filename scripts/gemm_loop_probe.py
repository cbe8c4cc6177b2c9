"""Steady-state rate of the 128-tile MFMA loop (k_gemm128, STORE epilogue): a lower SYRK
C = A A^T with beta = 0 (no split-K / stream-K), n = k = 3968 (31 row tiles: 496 lower tiles,
one round of 512 resident workgroups, 248 K steps each).  Prints ms and FP64 fraction;
run under scripts/pmc_mfma.sh for MFMA-busy."""
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
    n = k = int(os.environ.get("LOOP_N", "3968"))
    g = torch.Generator(device="cuda").manual_seed(5)
    A = torch.randn(n, k, dtype=torch.float64, device="cuda", generator=g) / k ** 0.5
    C = torch.zeros(n, n, dtype=torch.float64, device="cuda")
    ts = []
    for it in range(13):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        _lib._chk(_lib._L.gpmpc_syrk_batched_dev(ctx.h, n, k, 1, A.data_ptr(), k, 0, C.data_ptr(), n, 0,
                                                 1.0, 0.0), "syrk")
        e1.record(stream)
        ctx.sync()
        if it >= 3:
            ts.append(e0.elapsed_time(e1) * 1e-3)
    ref = A[:256] @ A[:256].T
    err = float((torch.tril(C[:256, :256]) - torch.tril(ref)).abs().max())
    fl = n * (n + 1) * k  # lower triangle incl. diagonal, 2 flop per multiply-add
    print(json.dumps({"n": n, "k": k, "min_ms": round(min(ts) * 1e3, 4),
                      "median_ms": round(float(np.median(ts)) * 1e3, 4),
                      "frac_min": round(fl / min(ts) / 1e12 / 78.6, 4), "maxerr": err}))
