"""Probe: where do the control kernel's waves land?  For each landing of the
1024-landing fleet, the HW_ID (SIMD, CU, SE, XCC) of its two waves and its
start/end realtime, over one control step; prints how many KKT-chain waves
share a SIMD and how the per-landing span relates to its ADMM iterations.
GPMPC_FLEET_ALTWAVE=1 runs the chain on wave (workgroup & 1).  The chain-sharing
lines assume the chain wave is 0 (or alternates): run with GPMPC_FLEET_SIMD=0 for
them, since by default each workgroup claims its chain SIMD at run time."""
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gp_mpc_rocket_landing_amd import _lib  # noqa: E402
from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions  # noqa: E402


def decode(v):
    v = int(v)
    hw = v & 0xFFFFFFFF
    return dict(wave=hw & 15, simd=(hw >> 4) & 3, cu=(hw >> 8) & 15, sh=(hw >> 12) & 1,
                se=(hw >> 13) & 7, xcc=(v >> 32) & 15)


def main(B=1024):
    alt = os.environ.get("GPMPC_FLEET_ALTWAVE", "0") == "1"
    ctx = _lib.Context(0)
    gp = fit_gp(ctx, n_train=1000)
    fl = Fleet(ctx, gp, B, horizon=20)
    fl.reset(initial_conditions(B))
    fl.step(3)
    tr = torch.zeros(B * 4, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    _lib._chk(_lib._L.gpmpc_fleet_set_trace(fl.h, tr.data_ptr()), "trace")
    rec0, _ = fl.read()
    fl.step(1)
    ctx.sync()
    rec1, _ = fl.read()
    t = tr.cpu().numpy().reshape(B, 4).view(np.uint64)
    its = rec1[:, 11] - rec0[:, 11]
    span = (t[:, 1].astype(np.float64) - t[:, 0].astype(np.float64)) / 100.0  # us
    t0 = t[:, 0].astype(np.float64).min()
    start = (t[:, 0].astype(np.float64) - t0) / 100.0
    w = [decode(v) for v in t[:, 2]]
    w1 = [decode(v) for v in t[:, 3]]
    cu_key = lambda d: (d["xcc"], d["se"], d["sh"], d["cu"])  # noqa: E731
    per_cu = Counter(cu_key(d) for d in w)
    print(f"alt_wave={alt}: {len(per_cu)} CUs used, landings per CU {Counter(per_cu.values())}")
    same_cu = sum(cu_key(a) == cu_key(b) for a, b in zip(w, w1))
    print(f"both waves on one CU: {same_cu}/{B}; wave0/wave1 same SIMD: "
          f"{sum(a['simd'] == b['simd'] for a, b in zip(w, w1))}")
    chain = [(w if not alt or (i & 1) == 0 else w1)[i] for i in range(B)]
    # the kernel is launched in dispatch order; blockIdx parity is not recorded,
    # so with alt_wave this is approximate (order[] maps slots to landings)
    simd_load = Counter((cu_key(d), d["simd"]) for d in chain)
    print(f"chain waves per SIMD: {Counter(simd_load.values())}")
    all_load = Counter((cu_key(d), d["simd"]) for d in w + w1)
    print(f"all waves per SIMD: {Counter(all_load.values())}")
    print(f"start spread {start.min():.1f}..{start.max():.1f} us; span us by iterations:")
    for k in sorted(set(its.astype(int))):
        m = its == k
        print(f"  it={k:3d}: {m.sum():4d} landings, span {span[m].mean():7.1f} us "
              f"(min {span[m].min():.1f}, max {span[m].max():.1f})")
    # does sharing a SIMD with another chain wave slow a 50-iteration landing?
    crowd = np.array([simd_load[(cu_key(d), d["simd"])] for d in chain])
    for c in sorted(set(crowd)):
        m = (crowd == c) & (its == its.max())
        if m.any():
            print(f"  chain-sharing {c}: {m.sum()} max-it landings, span {span[m].mean():.1f} us "
                  f"(p90 {np.percentile(span[m], 90):.1f}, max {span[m].max():.1f})")
    # what sets the slow long landings apart: co-resident long landings, XCC, SE
    longs = its == its.max()
    cu_long = Counter(cu_key(d) for d, l in zip(w, longs) if l)
    nl = np.array([cu_long[cu_key(d)] for d in w])
    for c in sorted(set(nl[longs])):
        m = longs & (nl == c)
        print(f"  long landings on the CU = {c}: {m.sum():4d} long landings, span {span[m].mean():.1f} us "
              f"(max {span[m].max():.1f})")
    xcc = np.array([d["xcc"] for d in w])
    print("  long-landing span by XCC: " + ", ".join(
        f"{x}: {span[longs & (xcc == x)].mean():.0f}/{span[longs & (xcc == x)].max():.0f}"
        for x in sorted(set(xcc))))
    rho = rec1[:, 15]
    print("  long-landing span by rho: " + ", ".join(
        f"{r:.3g}: n={np.sum(longs & (rho == r))} {span[longs & (rho == r)].mean():.0f}"
        for r in sorted(set(rho[longs]))[:8]))
    sl = np.argsort(-span)[:12]
    print("  slowest: " + "; ".join(f"b={i} it={its[i]:.0f} span={span[i]:.0f} rho={rho[i]:.3g} "
                                    f"cu_long={nl[i]}" for i in sl))
    fl.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1024)
