"""Probe: does splitting a batched potrf into independent sub-batches on separate
HIP streams (contexts) overlap one group's latency-bound diagonal factors with the
other group's SYRKs?  n = 1000; total batch 64 / 256 as G groups."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gp_mpc_rocket_landing_amd import _lib  # noqa: E402


def run(total, groups, n=1000, reps=4):
    ctxs = [_lib.Context(0) for _ in range(groups)]
    g = torch.Generator(device="cuda").manual_seed(0)
    G = torch.randn(total, n, n, dtype=torch.float64, device="cuda", generator=g) / n ** 0.5
    base = torch.baddbmm(torch.eye(n, dtype=torch.float64, device="cuda").expand(total, n, n), G, G.transpose(1, 2))
    del G
    A = base.clone()
    info = torch.zeros(total, dtype=torch.int32, device="cuda")
    per = total // groups
    best = None
    for _ in range(reps):
        A.copy_(base)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i, c in enumerate(ctxs):
            _lib._chk(_lib._L.gpmpc_potrf_batched_dev(c.h, n, per, A[i * per].data_ptr(), n, n * n,
                                                       info[i * per:].data_ptr()), "potrf")
        for c in ctxs:
            c.sync()
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    assert int(info.abs().sum()) == 0
    fl = total * (n ** 3 / 3)
    print(f"total={total} groups={groups}: {best * 1e3:.3f} ms  {fl / best / 78.6e12 * 100:.1f}% peak", flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    for total, groups in [(64, 1), (64, 2), (64, 4), (256, 1), (256, 2), (256, 4), (1024, 1), (1024, 4)]:
        run(total, groups)
