#!/usr/bin/env python
"""How much of the configs[3] Monte-Carlo's integer record is a property of the
algorithm and how much of its arithmetic (CPU only, the oracle against itself).

The oracle closed loop (oracle/mc_oracle.closed_loop_landing: monte_carlo.py
:401-583 with the numpy GP, numpy QP assembly and the C OSQP-0.6 restatement)
is run over the 1024 landings of BASELINE configs[3] three ways:
  base   as committed (tests/golden/mc_oracle_1024.npz);
  ulp    the GP weights alpha scaled by (1 + 2^-52) -- a one-ulp change;
  fma    the C ADMM compiled with -ffp-contract=fast (FMA contraction), i.e. the
         same algorithm with a different rounding of its products.
Free-running, the records are compared landing by landing; step-locked (the
perturbed oracle's step from the base oracle's state at every step), the
integer fields of every control step.  Then the tight-QP SQP step of the
fleet's sqp test (100 passes, eps 1e-7, max_iter 2000) base vs fma.

    python scripts/mc_sensitivity.py [--out profiles/r4_mc_sensitivity.json]   # ~8 min on 8 cores
"""
import argparse
import json
import os
import pickle
import subprocess
import sys
import tempfile
from multiprocessing import get_context

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

FIELDS = [0, 1, 11, 12, 13, 14]   # outcome, steps, ADMM iterations, solved count, m0, last status
_ST = None
FMA_LIB = os.path.join(tempfile.gettempdir(), "libadmm_ref_fma.so")


def _init(mode):
    global _ST
    if mode == "fma":
        import oracle.admm_ref as ar
        ar._LIB_PATH = FMA_LIB
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data
    from oracle import gp_oracle
    X, U, D = synthetic_training_data(1000, seed=0)
    a = gp_oracle.exact_fit(gp_oracle.features_3dof(X, U), D)
    b = dict(a)
    b["alpha"] = a["alpha"] * (1.0 + 2.0 ** -52)
    _ST = (a, b if mode == "ulp" else a)


def _fly(i):
    from oracle import mc_oracle
    return mc_oracle.closed_loop_landing(_ST[1], mc_oracle.sample_initial_condition(42 + i))[0]


def _steplock(i):
    from oracle import mc_oracle
    a, b = _ST
    S = mc_oracle.new_landing(mc_oracle.sample_initial_condition(42 + i), 20)
    bad = steps = 0
    worst = 0.0
    for _ in range(302):
        if S["rec"][0] != 0:
            break
        A, ia = mc_oracle.landing_step(a, S)
        Bs, _ = mc_oracle.landing_step(b, S)
        steps += 1
        if not np.array_equal(A["rec"][FIELDS], Bs["rec"][FIELDS]):
            bad += 1
        elif ia is not None and A["rec"][0] == 0:
            worst = max(worst, float(np.max(np.abs(A["x"] - Bs["x"]) / np.maximum(np.abs(A["x"]), 1.0))))
        S = A
    return bad, steps, worst


def _records(mode, n):
    with get_context("spawn").Pool(min(8, os.cpu_count() or 1), initializer=_init, initargs=(mode,)) as p:
        return np.array(p.map(_fly, range(n), chunksize=8))


def _compare(R, G):
    d = np.nonzero(R[:, 11] != G[:, 11])[0]
    return {"outcome_differs": int(np.sum(R[:, 0] != G[:, 0])), "steps_differ": int(np.sum(R[:, 1] != G[:, 1])),
            "admm_total_differs": int(len(d)), "admm_total_delta": (R[d, 11] - G[d, 11]).astype(int).tolist(),
            "solved_count_differs": int(np.sum(R[:, 12] != G[:, 12])),
            "max_rel_fuel_diff": float(np.max(np.abs(R[:, 2] - G[:, 2]) / np.maximum(np.abs(G[:, 2]), 1.0)))}


def _tight(mode, states=None):
    """The tight-QP SQP control step (sqp_iters 100, eps 1e-7, max_iter 2000) of 8 landings x 3 steps."""
    _init(mode)
    from gp_mpc_rocket_landing_amd.fleet import initial_conditions
    from oracle import admm_ref, mc_oracle
    qs = admm_ref.default_settings(eps_abs=1e-7, eps_rel=1e-7, max_iter=2000)
    out = []
    if states is None:
        for x0 in initial_conditions(8):
            S = mc_oracle.new_landing(x0, 20)
            for _ in range(3):
                if S["rec"][0] != 0:
                    break
                A, _ = mc_oracle.landing_step(_ST[0], S, sqp_iters=100, sqp_tol=1e-4, qp_settings=qs)
                out.append((S, A))
                S = A
        return out
    worst, same = {}, True
    for S, A in states:
        Bs, _ = mc_oracle.landing_step(_ST[0], S, sqp_iters=100, sqp_tol=1e-4, qp_settings=qs)
        same &= bool(np.array_equal(A["rec"][FIELDS], Bs["rec"][FIELDS]))
        for key in ("x", "Xw", "Uw", "y"):
            fl = np.abs(A[key]).max() if key == "y" else 1.0
            worst[key] = max(worst.get(key, 0.0), float(np.max(np.abs(A[key] - Bs[key]) / np.maximum(np.abs(A[key]), fl))))
    return {"integers_identical": same, "max_rel_diff": worst}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r4_mc_sensitivity.json"))
    ap.add_argument("--landings", type=int, default=1024)
    ap.add_argument("--tight-child", choices=["base", "fma"], default=None)
    a = ap.parse_args()
    if a.tight_child:   # child process: the tight SQP step with one ADMM build
        st = pickle.load(sys.stdin.buffer) if a.tight_child == "fma" else None
        pickle.dump(_tight(a.tight_child, st), sys.stdout.buffer)
        return
    subprocess.run(["gcc", "-O2", "-fPIC", "-ffp-contract=fast", "-march=native", "-std=c99", "-shared",
                    os.path.join(REPO, "oracle", "admm_ref.c"), "-o", FMA_LIB, "-lm"], check=True)
    n = a.landings
    base = _records("base", n)
    out = {"landings": n, "control_steps": int(base[:, 1].sum()),
           "base_equals_golden": bool(np.array_equal(
               base, np.load(os.path.join(REPO, "tests", "golden", "mc_oracle_1024.npz"))["records"][:n]))}
    out["free_running_ulp"] = _compare(_records("ulp", n), base)
    out["free_running_fma"] = _compare(_records("fma", n), base)
    with get_context("spawn").Pool(min(8, os.cpu_count() or 1), initializer=_init, initargs=("ulp",)) as p:
        r = p.map(_steplock, range(n), chunksize=4)
    out["step_locked_ulp"] = {"steps": sum(x[1] for x in r), "steps_with_integer_mismatch": sum(x[0] for x in r),
                              "max_rel_state_diff": max(x[2] for x in r)}
    me = [sys.executable, os.path.abspath(__file__)]
    base_t = subprocess.run(me + ["--tight-child", "base"], check=True, capture_output=True).stdout
    fma_t = subprocess.run(me + ["--tight-child", "fma"], input=base_t, check=True, capture_output=True).stdout
    out["tight_sqp_step_fma"] = pickle.loads(fma_t)
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
