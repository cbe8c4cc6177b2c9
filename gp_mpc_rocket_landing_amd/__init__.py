"""gp_mpc_rocket_landing_amd -- MI355X-native GP + QP hot path of
shiivashaakeri/gp-mpc-rocket-landing (drop-in for Simple3DoFGP.fit/predict,
NominalMPC3DoF.solve, GPMPC.solve, FastRTI3DoF.step).

Python mirrors the reference's surfaces; all arithmetic on the path runs in
libgpmpc_hip.so (hand-written HIP for gfx950) through the C-ABI of
include/gpmpc.h.  Importing a compute module without the built library raises.
"""
__version__ = "0.1.0"
