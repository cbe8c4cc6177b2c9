"""Plants used by the controllers (reference src/dynamics; simdyn restated)."""
from .rocket_3dof import Rocket3DoFConfig, Rocket3DoFDynamics, Rocket3DoFParams, create_normalized_rocket
from .rocket_6dof import (Rocket6DoFConfig, Rocket6DoFDynamics, Rocket6DoFParams, create_rocket_6dof,
                          create_szmuk_rocket)

__all__ = ["Rocket3DoFConfig", "Rocket3DoFDynamics", "Rocket3DoFParams", "create_normalized_rocket",
           "Rocket6DoFConfig", "Rocket6DoFDynamics", "Rocket6DoFParams", "create_rocket_6dof",
           "create_szmuk_rocket"]
