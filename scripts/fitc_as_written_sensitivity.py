#!/usr/bin/env python
"""How far the reference's as-written FITC mean (K*u alpha, sparse_gp.py:280-283,
SURVEY D1) moves a configs[4] rollout when only the arithmetic changes -- the
bound test_gpu_rollouts6.py's M = 2000 as-written test states (CPU only, the
oracle against itself).

The config-5 GP pair (StructuredRocketGP, M = 2000 kmeans2 inducing points, N =
4000 rows, unit SE-ARD, noise 1e-4, jitter 1e-6) is fitted by the oracle three
ways:
  base   gp_oracle.fitc_fit as committed;
  alpha  the weights alpha scaled by (1 + 2^-52): a one-ulp change of the
         as-written mean's own coefficients (VERDICT r4's definition);
  gram   every kernel value the fit and the predictions form scaled by
         (1 + r 2^-52), r in {-1, 0, 1} fixed per entry -- what a second correct
         implementation with its own exp and summation orders looks like.
The 16 rollouts x 12 control steps of the device test are flown by the base
oracle; at every step the perturbed oracles step from the base state
(step-locked), and the plans, states, forward simulation and GP means are
compared in the tolerance metric of tests/conftest.close (units of 1e-6
relative with a unit floor).

    python scripts/fitc_as_written_sensitivity.py [--out profiles/r6_fitc_as_written_sensitivity.json]
"""
import argparse
import json
import os
import sys
import time

os.environ.setdefault("OPENBLAS_NUM_THREADS", "8")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
from scipy.cluster.vq import kmeans2  # noqa: E402


def _close(a, b, scale=1.0, rtol=1e-6):
    a = np.asarray(a, float); b = np.asarray(b, float)
    return float(np.max(np.abs(a - b) / (rtol * np.maximum(np.abs(b), scale))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--rollouts", type=int, default=16)
    ap.add_argument("--steps", type=int, default=12)
    a = ap.parse_args()
    from gp_mpc_rocket_landing_amd.data import synthetic_6dof_training_data
    from gp_mpc_rocket_landing_amd.gp.features import CombinedFeatureExtractor
    from gp_mpc_rocket_landing_amd.rollouts6 import initial_conditions_6dof
    from oracle import gp_oracle
    from oracle import sixdof_oracle as so

    t0 = time.time()
    X, U, Dv, Dw = synthetic_6dof_training_data(4000, seed=0)
    fe = CombinedFeatureExtractor()
    np.random.seed(0)   # the surface's kmeans2 draws (sparse_gp.py:122-148), v then w
    Zi_v = kmeans2(fe.extract_batch_translational(X, U), 2000, minit="points")[0]
    Zi_w = kmeans2(fe.extract_batch_rotational(X, U), 2000, minit="points")[0]
    Zv, Zw = gp_oracle.features_translational(X, U), gp_oracle.features_rotational(X, U)

    gram0 = gp_oracle.gram

    def fit(perturb_gram):
        if perturb_gram:
            rs = np.random.RandomState(12345)

            def gram_ulp(kind, X1, X2, sigma2, ls):
                K = gram0(kind, X1, X2, sigma2, ls)
                return K * (1.0 + rs.randint(-1, 2, size=K.shape) * 2.0 ** -52)
            gp_oracle.gram = gram_ulp
        try:
            return gp_oracle.fitc_fit(Zi_v, Zv, Dv), gp_oracle.fitc_fit(Zi_w, Zw, Dw)
        finally:
            gp_oracle.gram = gram0

    base = fit(False)
    alpha = tuple(dict(st, alpha=st["alpha"] * (1.0 + 2.0 ** -52)) for st in base)
    gram = fit(True)
    print(f"fits {time.time() - t0:.1f} s", flush=True)

    keys = ("X_pred", "gm", "X", "U", "x", "rho", "y")
    scale = dict(rho=lambda w: 0.0, y=lambda w: float(np.abs(w).max()))   # the test's floors
    worst = {v: {k: 0.0 for k in keys} for v in ("alpha", "gram")}
    ints_differ = {"alpha": 0, "gram": 0}
    x0 = initial_conditions_6dof(a.rollouts)
    steps = 0
    for b in range(a.rollouts):
        S = so.new_rollout(x0[b], 30)
        for k in range(a.steps):
            if S["rec"][0] != 0:
                break
            want, info = so.rollout_step(*base, S, corrected=False)
            if info is None or want["rec"][0] != 0:
                S = want
                continue
            steps += 1
            for name, gps in (("alpha", alpha), ("gram", gram)):
                if name == "gram":
                    # the perturbed predictions too: the gram hook stays on for the step
                    rs = np.random.RandomState(777 + 31 * b + k)

                    def gram_ulp(kind, X1, X2, sigma2, ls, rs=rs):
                        K = gram0(kind, X1, X2, sigma2, ls)
                        return K * (1.0 + rs.randint(-1, 2, size=K.shape) * 2.0 ** -52)
                    gp_oracle.gram = gram_ulp
                try:
                    got, _ = so.rollout_step(*gps, S, corrected=False)
                finally:
                    gp_oracle.gram = gram0
                if not np.array_equal(got["rec"][[0, 1, 11, 12, 14]], want["rec"][[0, 1, 11, 12, 14]]):
                    ints_differ[name] += 1
                    continue
                for key in keys:
                    sc = scale.get(key, lambda w: 1.0)(want[key])
                    worst[name][key] = max(worst[name][key], _close(got[key], want[key], sc))
            S = want
        print(f"rollout {b}: {steps} steps, worst {worst}", flush=True)
    out = dict(rollouts=a.rollouts, steps_per_rollout=a.steps, compared_steps=steps,
               metric="max |a - b| / (1e-6 max(|b|, 1)) (tests/conftest.close)", worst=worst,
               integer_fields_differ=ints_differ, seconds=round(time.time() - t0, 1))
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
