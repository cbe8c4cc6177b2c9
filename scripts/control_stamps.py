"""Phase cycles (s_memtime) of landing 0's control-kernel workgroup over a few
control steps of the 1024-landing fleet (gpmpc_fleet_set_stamps: the stamped
kernel instance).  Slots: 0 assembly, 1 scaling, 2 factor, 3 rhs, 4 KKT block
solve (rest), 5 x/z/y update, 6 checks + adaptive rho, 7 plant + tail, 8-10 the
KKT solve's forward chain / diagonal blocks / backward chain, 11/12 the rhs and
update compute before their barriers, 14 realtime
(100 MHz), 15 total shader cycles."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gp_mpc_rocket_landing_amd import _lib  # noqa: E402
from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions  # noqa: E402


def main(steps=4, B=1024):
    ctx = _lib.Context(0)
    gp = fit_gp(ctx, n_train=1000)
    fl = Fleet(ctx, gp, B, horizon=20)
    fl.reset(initial_conditions(B))
    fl.step(3)
    st = torch.zeros(16, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    _lib._chk(_lib._L.gpmpc_fleet_set_stamps(fl.h, st.data_ptr()), "stamps")
    rec0, _ = fl.read()
    fl.step(steps)
    ctx.sync()
    rec1, _ = fl.read()
    s = st.cpu().numpy().astype(np.float64)
    it = rec1[0, 11] - rec0[0, 11]
    names = ["assembly", "scaling", "factor", "rhs", "kkt_solve(rest)", "update", "checks", "tail",
             "kkt_forward", "kkt_diagonal", "kkt_backward", "rhs_compute", "update_compute", "unused"]
    tot = s[15]
    print(f"B={B} landing 0: {steps} steps, {it:.0f} ADMM iterations, {tot:.0f} shader cycles "
          f"({s[14] / 100e6 * 1e6:.1f} us realtime)")
    for i, nm in enumerate(names):
        print(f"  {nm:10s} {s[i]:10.0f} cycles  {s[i] / tot * 100:5.1f}%  {s[i] / max(it, 1):8.0f} per iteration")


if __name__ == "__main__":
    main(B=int(sys.argv[1]) if len(sys.argv) > 1 else 1024)
