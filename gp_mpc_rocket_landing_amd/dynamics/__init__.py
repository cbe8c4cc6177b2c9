"""3-DoF plant used by the controllers (reference src/dynamics; simdyn restated)."""
from .rocket_3dof import Rocket3DoFConfig, Rocket3DoFDynamics, Rocket3DoFParams, create_normalized_rocket

__all__ = ["Rocket3DoFConfig", "Rocket3DoFDynamics", "Rocket3DoFParams", "create_normalized_rocket"]
