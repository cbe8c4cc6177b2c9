"""MPC surfaces (reference src/mpc): RTI QP controllers on the device ADMM,
uncertainty propagation and constraint tightening."""
from .constraints import ConstraintParams, TightenedConstraints
from .cost_functions import CostWeights
from .gp_mpc import GPMPC, GPMPCConfig, SimpleGPPredictor
from .nominal_mpc import MPCConfig, MPCSolution, NominalMPC3DoF
from .osqp_rti import FastRTI3DoF, OSQPRTIConfig, OSQPRTIMPC, OSQPRTISolution
from .uncertainty_prop import (ConstraintTightening, PropagatedUncertainty, TubeBasedRobustness,
                               UncertaintyPropagator)

__all__ = ["GPMPC", "GPMPCConfig", "MPCConfig", "MPCSolution", "NominalMPC3DoF", "FastRTI3DoF",
           "OSQPRTIConfig", "OSQPRTIMPC", "OSQPRTISolution", "ConstraintParams", "TightenedConstraints",
           "ConstraintTightening", "PropagatedUncertainty", "TubeBasedRobustness", "UncertaintyPropagator",
           "CostWeights", "SimpleGPPredictor"]
