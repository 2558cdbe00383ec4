"""rl_rocket_amd — MI355X-native vectorized rocket-landing environment.

The hot path of Tuxliri/RL_rocket (``Rocket6DOF.step`` / ``Rocket.step`` and their
simulators) as fused gfx950 HIP kernels behind a C-ABI (``include/rocket_hip.h``),
with the reference's gym-0.21 surface on top:

  * ``RocketBatch``    — N envs on one GPU, torch tensors in/out (device-resident)
  * ``RocketVecEnv``   — stable-baselines3 ``VecEnv``-compatible vector env
  * ``RocketVectorEnv`` — the same with the ``gym.vector.VectorEnv`` surface (batched spaces)
  * ``Rocket6DOF`` / ``Rocket`` — single-env gym.Env shims with the reference's API,
    registered as ``my_environment/Falcon6DOF-v0`` / ``Falcon3DOF-v0`` when gym is present.
"""
from .params import (ENV_CONFIG_6DOF, DEFAULTS_6DOF, DEFAULTS_3DOF, MAX_EPISODE_STEPS,  # noqa: F401
                     make_config, lower)

__all__ = ["RocketBatch", "RocketVecEnv", "RocketVectorEnv", "Rocket6DOF", "Rocket", "ENV_CONFIG_6DOF",
           "make_config"]


def __getattr__(name):
    if name == "RocketBatch":
        from .batch import RocketBatch
        return RocketBatch
    if name in ("RocketVecEnv", "RocketVectorEnv"):
        from . import vec_env
        return getattr(vec_env, name)
    if name in ("Rocket6DOF", "Rocket"):
        from . import envs
        return getattr(envs, name)
    raise AttributeError(name)
