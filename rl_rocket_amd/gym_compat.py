"""The gym 0.21 pieces the reference env surface needs, without requiring gym.

If ``gym`` is importable its ``Env`` base class is used (so ``isinstance`` checks,
``gym.make`` and wrappers work); otherwise a minimal stand-in with the same
attribute protocol is provided.  ``Box`` always follows gym 0.21 semantics —
float32 bounds, sampling ``RandomState.uniform(low, high)`` into float64 and
casting to the space dtype, inclusive ``contains`` — with gym 0.21 seeding
(``seeding.np_random``: ``RandomState`` seeded by the little-endian uint32
words of the first 8 bytes of ``sha512(str(seed))``), so the single-env shims
reproduce the reference's reset stream exactly (gym 0.21 is pinned at the
reference's requirements.txt:29 but is absent from this image).
"""
import hashlib
import struct

import numpy as np

try:  # pragma: no cover - depends on the environment
    import gym as _gym

    EnvBase = _gym.Env
    HAVE_GYM = True
except Exception:  # gym is not installed in this image
    _gym = None
    HAVE_GYM = False

    class EnvBase:
        metadata = {"render.modes": []}
        reward_range = (-float("inf"), float("inf"))
        spec = None
        action_space = None
        observation_space = None

        def seed(self, seed=None):
            return [seed]

        def close(self):
            pass

        @property
        def unwrapped(self):
            return self


def _bigint_from_bytes(data):
    padding = 4 - len(data) % 4
    data += b"\0" * padding
    words = struct.unpack("%dI" % (len(data) // 4), data)
    return sum(w << (32 * i) for i, w in enumerate(words))


def _int_list_from_bigint(bigint):
    if bigint == 0:
        return [0]
    out = []
    while bigint > 0:
        bigint, mod = divmod(bigint, 2 ** 32)
        out.append(mod)
    return out


def np_random(seed=None):
    """gym 0.21 ``utils.seeding.np_random``."""
    if seed is None:
        seed = _bigint_from_bytes(np.random.bytes(8))
    if not (isinstance(seed, (int, np.integer)) and seed >= 0):
        raise ValueError("Seed must be a non-negative integer or omitted, not %r" % (seed,))
    seed = int(seed) % 2 ** 64
    h = _bigint_from_bytes(hashlib.sha512(str(seed).encode("utf8")).digest()[:8])
    rng = np.random.RandomState()
    rng.seed(_int_list_from_bigint(h))
    return rng, seed


class Box:
    """gym 0.21 ``spaces.Box`` (bounded float boxes are all this surface needs)."""

    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        self.dtype = np.dtype(dtype)
        if shape is None:
            shape = np.asarray(low).shape if not np.isscalar(low) else np.asarray(high).shape
        self.shape = tuple(shape)
        low = np.full(self.shape, low, dtype=self.dtype) if np.isscalar(low) else np.asarray(low)
        high = np.full(self.shape, high, dtype=self.dtype) if np.isscalar(high) else np.asarray(high)
        self.low = low.astype(self.dtype)
        self.high = high.astype(self.dtype)
        self._np_random = None
        if seed is not None:
            self.seed(seed)

    @property
    def np_random(self):
        if self._np_random is None:
            self.seed()
        return self._np_random

    def seed(self, seed=None):
        self._np_random, seed = np_random(seed)
        return [seed]

    def sample(self):
        s = np.empty(self.shape)
        s[...] = self.np_random.uniform(low=self.low, high=self.high, size=self.shape)
        return s.astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return bool(np.can_cast(x.dtype, self.dtype) and x.shape == self.shape
                    and np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return "Box(%s, %s, %s, %s)" % (self.low.min(), self.high.max(), self.shape, self.dtype)

    def to_gym(self):
        """The equivalent real gym Box, when gym is importable (for SB3 space checks)."""
        if not HAVE_GYM:
            return self
        return _gym.spaces.Box(low=self.low, high=self.high, dtype=self.dtype)


def register_ids():
    """Register the reference env ids (my_environment/__init__.py:4-12) with gym, if present."""
    if not HAVE_GYM:
        return False
    from gym.envs.registration import register, registry

    ids = {"my_environment/Falcon3DOF-v0": "rl_rocket_amd.envs:Rocket",
           "my_environment/Falcon6DOF-v0": "rl_rocket_amd.envs:Rocket6DOF"}
    existing = getattr(registry, "env_specs", registry)
    for env_id, entry in ids.items():
        if env_id not in existing:
            register(id=env_id, entry_point=entry)
    return True
