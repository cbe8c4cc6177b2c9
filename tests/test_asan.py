"""Host-side AddressSanitizer + UBSan runs ("-fsanitize=address
host build of the CPU C-ABI shim"), on the CPU.

* libgpmpc_hip built with the host half of every translation unit instrumented
  (``make asan``: -Xarch_host -fsanitize=address,undefined; the device code is
  never instrumented) is loaded by a Python child under the clang ASan runtime,
  and every C-ABI path that runs without a GPU is driven: the version / error
  strings, the default configs and their ctypes mirrors, the argument checks of
  every entry point (NULL handles, negative sizes: -2, no crash), the context
  creation failure without a device.
* oracle/admm_ref.c (the C OSQP-0.6 restatement: the parity checker and the CPU
  baseline) under gcc's -fsanitize=address,undefined with a C harness that
  solves banded MPC-shaped QPs of several sizes, warm-started, with the
  persistent rho / y carried between solves.
"""
import glob
import os
import subprocess
import sys
import textwrap

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "gp_mpc_rocket_landing_amd", "csrc")
ASAN_LIB = os.path.join(CSRC, "build", "asan", "libgpmpc_hip_asan.so")

CHILD = textwrap.dedent(r'''
    import ctypes, numpy as np
    from gp_mpc_rocket_landing_amd import _lib
    L = _lib._L
    assert _lib.abi_version() == _lib.ABI_VERSION == 4 and _lib.LIB_PATH.endswith("libgpmpc_hip_asan.so")
    assert isinstance(L.gpmpc_last_error(), bytes)
    s = _lib.qp_default_settings(max_iter=7)
    assert s.max_iter == 7 and s.rho == 0.1
    c = _lib.fleet_default_config(max_iter=9, sqp_qp=dict(eps_abs=1e-7))
    assert c.qp.max_iter == 9 and c.sqp_qp.max_iter == 9 and c.sqp_qp.eps_abs == 1e-7
    r = _lib.rollout6_default_config(horizon=20, rocket_alpha=0.04)
    assert r.horizon == 20 and r.rocket_alpha == 0.04 and list(r.rocket_r_t) == [-0.25, 0.0, 0.0]
    h = ctypes.c_void_p()
    info = ctypes.c_int(0)
    d = np.zeros(16)
    dp = _lib._d(d)
    # every entry point rejects NULL handles / bad sizes through its argument check (-2)
    bad = [
        L.gpmpc_gram(None, 0, dp, 1, dp, 1, 1, dp, 1.0, dp, 0),
        L.gpmpc_potrf(None, 4, dp, 4, ctypes.byref(info)),
        L.gpmpc_potrf_batched_dev(None, 4, 1, None, 4, 16, None),
        L.gpmpc_trsm_lower(None, 4, 1, dp, 4, dp, 1),
        L.gpmpc_potrs(None, 4, 1, dp, 4, dp, 1),
        L.gpmpc_gp_fit_exact(None, 0, dp, 4, 2, dp, 1, dp, 1.0, 1e-4, ctypes.byref(h), None, None, None, None),
        L.gpmpc_gp_predict(None, None, dp, 1, dp, dp),
        L.gpmpc_fitc_fit(None, dp, 2, dp, 4, 2, dp, 1, dp, 1.0, 1e-4, 1e-6, ctypes.byref(h), None, None, None, None),
        L.gpmpc_fitc_predict(None, None, dp, 1, dp, dp),
        L.gpmpc_fleet_create(None, None, None, 4, ctypes.byref(h)),
        L.gpmpc_fleet_create_shard(None, None, None, 4, 8, ctypes.byref(h)),
        L.gpmpc_fleet_create_fitc(None, None, None, 4, 4, ctypes.byref(h)),
        L.gpmpc_fleet_step(None, 1),
        L.gpmpc_fleet_read(None, dp, dp),
        L.gpmpc_rollout6_create(None, None, None, None, 4, ctypes.byref(h)),
        L.gpmpc_rollout6_step(None, 1),
        L.gpmpc_rollout6_solve_ref(None, dp, dp, None, None, 0, 1, 1e-4, None, None, None, None, None, None),
        L.gpmpc_gather_results(None, None, None, None, 0, None),
        L.gpmpc_comm_init(None, None, 1, 0, ctypes.byref(h)),
        L.gpmpc_comm_count(None, None),
        L.gpmpc_cov_propagate(None, 1, 1, 2, dp, dp, None, 1e-6, dp),
        L.gpmpc_syrk_batched_dev(None, 4, 4, 1, None, 4, 16, None, 4, 16, 1.0, 0.0),
    ]
    assert all(v == -2 for v in bad), bad
    assert L.gpmpc_ctx_destroy(None) == 0 and L.gpmpc_fleet_destroy(None) == 0
    assert L.gpmpc_rollout6_destroy(None) == 0 and L.gpmpc_comm_destroy(None) == 0
    # no GPU in this container: context creation reports an error instead of crashing
    rc = L.gpmpc_ctx_create(0, ctypes.byref(h))
    assert rc != 0 and L.gpmpc_last_error()
    print("asan child ok")
''')

HARNESS = textwrap.dedent(r'''
    #include <math.h>
    #include <stdio.h>
    #include <stdlib.h>
    typedef struct { double rho, sigma, alpha, eps_abs, eps_rel, eps_prim_inf, eps_dual_inf;
                     int max_iter, check_termination, adaptive_rho, adaptive_rho_interval;
                     double adaptive_rho_tolerance; int scaling, warm_start; } ref_settings;
    void ref_qp_default_settings(ref_settings *s);
    int ref_qp_solve(int n, int m, const int *rp, const int *ci, const double *A, const double *P,
                     const double *q, const double *l, const double *u, const ref_settings *s,
                     const double *x_ws, double *rho, double *y, double *x, double *yo, int *it,
                     int *st, double *obj, double *res);
    /* a chain QP: x_{k+1} = a x_k + b u_k, |u| <= 1, quadratic cost; rows: x0, dynamics, bounds */
    static int run(int N, int maxit) {
      const int n = 2 * N + 1, m = (N + 1) + n;
      int *rp = malloc(sizeof(int) * (m + 1)), *ci = malloc(sizeof(int) * (3 * N + 1 + n));
      double *A = malloc(sizeof(double) * (3 * N + 1 + n)), *P = malloc(sizeof(double) * n),
             *q = malloc(sizeof(double) * n), *l = malloc(sizeof(double) * m), *u = malloc(sizeof(double) * m),
             *x = malloc(sizeof(double) * n), *y = calloc(m, sizeof(double)), *yo = malloc(sizeof(double) * m),
             *ws = calloc(n, sizeof(double));
      int k = 0, r = 0;
      rp[0] = 0;
      ci[k] = 0; A[k++] = 1.0; l[r] = u[r] = 1.0; rp[++r] = k;                /* x0 = 1 */
      for (int s = 0; s < N; ++s) {                                           /* a x - ... */
        ci[k] = 2 * s; A[k++] = 0.9; ci[k] = 2 * s + 1; A[k++] = 0.1; ci[k] = 2 * s + 2; A[k++] = -1.0;
        l[r] = u[r] = 0.0; rp[++r] = k;
      }
      for (int j = 0; j < n; ++j) {
        ci[k] = j; A[k++] = 1.0;
        l[r] = (j % 2) ? -1.0 : -1e30; u[r] = (j % 2) ? 1.0 : 1e30; rp[++r] = k;
      }
      for (int j = 0; j < n; ++j) { P[j] = (j % 2) ? 0.01 : 1.0; q[j] = (j % 2) ? 0.0 : -0.5; }
      ref_settings st; ref_qp_default_settings(&st); st.max_iter = maxit;
      double rho = st.rho, obj, res[2];
      int it, status, rc = 0;
      for (int rep = 0; rep < 3 && !rc; ++rep) {                              /* warm-started re-solves */
        rc = ref_qp_solve(n, m, rp, ci, A, P, q, l, u, &st, ws, &rho, y, x, yo, &it, &status, &obj, res);
        for (int j = 0; j < n; ++j) ws[j] = x[j];
      }
      printf("N=%d rc=%d status=%d iter=%d obj=%g\n", N, rc, status, it, obj);
      free(rp); free(ci); free(A); free(P); free(q); free(l); free(u); free(x); free(y); free(yo); free(ws);
      return rc || !(status == 1 || status == 2 || status == -2);
    }
    int main(void) {
      int bad = 0;
      int sizes[] = {1, 2, 7, 20, 64};
      for (int i = 0; i < 5; ++i) bad |= run(sizes[i], i % 2 ? 50 : 400);
      return bad;
    }
''')


def _clang_asan_runtime():
    hits = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return hits[-1] if hits else None


@pytest.mark.skipif(_clang_asan_runtime() is None, reason="no clang ASan runtime in this image")
def test_capi_host_paths_under_asan():
    subprocess.run(["make", "-s", "-j", str(min(8, os.cpu_count() or 1)), "-C", CSRC, "asan"], check=True)
    env = dict(os.environ, LD_PRELOAD=_clang_asan_runtime(), GPMPC_LIB=ASAN_LIB,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               GPMPC_HIP_RUNTIME="system", PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "asan child ok" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]


def test_oracle_admm_under_asan_ubsan(tmp_path):
    src = tmp_path / "harness.c"
    src.write_text(HARNESS)
    exe = tmp_path / "harness"
    subprocess.run(["gcc", "-O1", "-g", "-std=c99", "-ffp-contract=off", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", str(src),
                    os.path.join(REPO, "oracle", "admm_ref.c"), "-o", str(exe), "-lm"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0, (r.stdout, r.stderr[-4000:])
    assert r.stdout.count("rc=0") == 5, r.stdout
