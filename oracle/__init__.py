"""CPU oracle for the GP + QP hot path -- TEST INFRASTRUCTURE ONLY.

This package restates, in plain numpy (and plain C for the ADMM loop, see
``admm_ref.c``), the reference algorithms of shiivashaakeri/gp-mpc-rocket-landing
on the per-control-step hot path:

* ``gp_oracle``   -- SE-ARD / Matern kernels, exact GP, FITC sparse GP, feature
                     extractors, Simple3DoFGP / StructuredRocketGP
                     (reference ``src/gp/*.py``).
* ``qp_oracle``   -- 3-DoF plant restatement, analytic linearisation and the
                     OSQP-RTI QP data assembly (reference ``src/mpc/osqp_rti.py``).
* ``admm_oracle`` -- an OSQP-0.6 ADMM restatement (the reference calls the
                     third-party ``osqp`` C library, which is absent here:
                     parity against OSQP itself is *unpinned*).
* ``mc_oracle``   -- Monte-Carlo initial-condition sampler and landing
                     classification (reference ``src/experiments/monte_carlo.py``).

Who may import this package: ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` -- only as the checker / the timed CPU
baseline, never as the product path.  The product (``gp_mpc_rocket_landing_amd``)
never imports it and fails loudly when its HIP library is missing.

The GP restatement is pinned against golden vectors generated from the
reference itself (``tests/golden/gen_golden.py``, run in the build container
where ``/root/reference`` is importable through a namespace shim).
"""
