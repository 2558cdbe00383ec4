"""my_environment.envs (reference envs/__init__.py:1) -> rl_rocket_amd single-env shims."""
from rl_rocket_amd.envs import Rocket, Rocket6DOF  # noqa: F401

__all__ = ["Rocket", "Rocket6DOF"]
