"""Minimal restatement of the gym 0.21.0 API surface that the reference's
``my_environment`` package imports (gym is pinned at requirements.txt:29 /
setup.py:6 of the reference but is absent from this image).

FIXTURE-GENERATION ONLY.  This package is put first on ``sys.path`` by
``tests/golden/gen_golden.py`` so that the reference's ``rocket_env.py`` can be
imported in the survey container.  It is never imported by the product
(``rl_rocket_amd``), by ``bench.py`` or by the GPU tests.

What is restated (from gym 0.21.0's published source, behaviour only):
  * ``gym.Env`` / ``gym.Wrapper`` / ``ObservationWrapper`` / ``ActionWrapper``
    base classes (attribute forwarding only),
  * ``gym.spaces.Box`` (dtype casting of bounds, seeded ``RandomState``
    sampling, inclusive ``contains`` with ``np.can_cast``) and ``Discrete``,
  * ``gym.utils.seeding.np_random`` (sha512 ``hash_seed`` -> RandomState),
  * ``gym.envs.registration.register`` (records ids, no-op otherwise).
"""
from . import spaces, logger  # noqa: F401
from .core import Env, Wrapper, ObservationWrapper, ActionWrapper, RewardWrapper  # noqa: F401

__version__ = "0.21.0-shim"
