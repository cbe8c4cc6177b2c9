"""Batched fp64 potrf timing probe: n x n SPD matrices, several batch sizes.
Prints ms and TFLOP/s per (n, batch).  GPMPC_POTRF128=0 selects the 32-step path."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gp_mpc_rocket_landing_amd import _lib  # noqa: E402


def main():
    ctx = _lib.Context(0)
    stream = torch.cuda.ExternalStream(ctx.stream)
    shapes = [(1000, 1), (1000, 14), (1000, 64), (1000, 256), (2000, 1), (2000, 8)]
    if os.environ.get("PROBE_SHAPES"):   # e.g. "1000x1,1000x64"
        shapes = [tuple(int(v) for v in t.split("x")) for t in os.environ["PROBE_SHAPES"].split(",")]
    for n, batch in shapes:
        g = torch.Generator(device="cuda").manual_seed(0)
        G = torch.randn(batch, n, n, dtype=torch.float64, device="cuda", generator=g) / n ** 0.5
        base = G @ G.transpose(1, 2) + torch.eye(n, dtype=torch.float64, device="cuda")
        del G
        A = base.clone()
        info = torch.zeros(batch, dtype=torch.int32, device="cuda")
        ts = []
        for _ in range(4):
            A.copy_(base)
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            _lib._chk(_lib._L.gpmpc_potrf_batched_dev(ctx.h, n, batch, A.data_ptr(), n, n * n,
                                                       info.data_ptr()), "potrf")
            e1.record(stream)
            ctx.sync()
            ts.append(e0.elapsed_time(e1) * 1e-3)
        assert int(info.abs().sum()) == 0
        pick = [0, batch - 1]              # first and last matrix (different chunks when split)
        ref = torch.linalg.cholesky(base[pick])
        err = float((torch.tril(A[pick]) - ref).abs().max())
        t = min(ts[1:])
        fl = batch * (n ** 3 / 3 + n ** 2 / 2 + n / 6)
        print(f"n={n} batch={batch}: {t * 1e3:.3f} ms  {fl / t / 1e12:.2f} TFLOP/s  "
              f"{fl / t / 78.6e12 * 100:.1f}% fp64 peak  maxerr {err:.2e}", flush=True)
        del A, base


if __name__ == "__main__":
    main()
