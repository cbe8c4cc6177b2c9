"""MPC surfaces (reference src/mpc): RTI QP controllers on the device ADMM."""
from .gp_mpc import GPMPC, GPMPCConfig
from .nominal_mpc import MPCConfig, MPCSolution, NominalMPC3DoF
from .osqp_rti import FastRTI3DoF, OSQPRTIConfig, OSQPRTIMPC, OSQPRTISolution

__all__ = ["GPMPC", "GPMPCConfig", "MPCConfig", "MPCSolution", "NominalMPC3DoF", "FastRTI3DoF",
           "OSQPRTIConfig", "OSQPRTIMPC", "OSQPRTISolution"]
