"""gym 0.21 ``spaces.Box`` / ``Discrete`` restated (fixture generation only).

Behaviour reproduced from gym 0.21.0 ``gym/spaces/box.py``:
  * bounds are cast to ``dtype`` (float32 by default) after shape inference;
  * ``sample()`` for a fully bounded box draws
    ``np_random.uniform(low, high, size)`` into a float64 array and casts it to
    ``dtype``;
  * ``contains(x)`` = ``np.can_cast(x.dtype, dtype) and shape matches and
    all(x >= low) and all(x <= high)`` (inclusive; NaN -> False).
"""
import numpy as np

from .utils import seeding


class Space:
    def __init__(self, shape=None, dtype=None, seed=None):
        self._shape = None if shape is None else tuple(shape)
        self.dtype = None if dtype is None else np.dtype(dtype)
        self._np_random = None
        if seed is not None:
            self.seed(seed)

    @property
    def np_random(self):
        if self._np_random is None:
            self.seed()
        return self._np_random

    @property
    def shape(self):
        return self._shape

    def seed(self, seed=None):
        self._np_random, seed = seeding.np_random(seed)
        return [seed]


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        self.dtype = np.dtype(dtype)
        if shape is not None:
            shape = tuple(shape)
        elif not np.isscalar(low):
            shape = np.asarray(low).shape
        elif not np.isscalar(high):
            shape = np.asarray(high).shape
        else:
            raise ValueError("shape must be provided or inferred")
        if np.isscalar(low):
            low = np.full(shape, low, dtype=dtype)
        if np.isscalar(high):
            high = np.full(shape, high, dtype=dtype)
        self.low = np.asarray(low).astype(self.dtype)
        self.high = np.asarray(high).astype(self.dtype)
        self.bounded_below = -np.inf < self.low
        self.bounded_above = np.inf > self.high
        super().__init__(shape, self.dtype, seed)

    def is_bounded(self, manner="both"):
        below = np.all(self.bounded_below)
        above = np.all(self.bounded_above)
        if manner == "both":
            return below and above
        if manner == "below":
            return below
        if manner == "above":
            return above
        raise ValueError(manner)

    def sample(self):
        high = self.high if self.dtype.kind == "f" else self.high.astype("int64") + 1
        sample = np.empty(self.shape)
        unbounded = ~self.bounded_below & ~self.bounded_above
        upp_bounded = ~self.bounded_below & self.bounded_above
        low_bounded = self.bounded_below & ~self.bounded_above
        bounded = self.bounded_below & self.bounded_above
        sample[unbounded] = self.np_random.normal(size=unbounded[unbounded].shape)
        sample[low_bounded] = (
            self.np_random.exponential(size=low_bounded[low_bounded].shape) + self.low[low_bounded]
        )
        sample[upp_bounded] = (
            -self.np_random.exponential(size=upp_bounded[upp_bounded].shape) + self.high[upp_bounded]
        )
        sample[bounded] = self.np_random.uniform(
            low=self.low[bounded], high=high[bounded], size=bounded[bounded].shape
        )
        if self.dtype.kind == "i":
            sample = np.floor(sample)
        return sample.astype(self.dtype)

    def contains(self, x):
        if not isinstance(x, np.ndarray):
            x = np.asarray(x, dtype=self.dtype)
        return bool(
            np.can_cast(x.dtype, self.dtype)
            and x.shape == self.shape
            and np.all(x >= self.low)
            and np.all(x <= self.high)
        )


class Discrete(Space):
    def __init__(self, n, seed=None):
        self.n = n
        super().__init__((), np.int64, seed)

    def sample(self):
        return int(self.np_random.randint(self.n))

    def contains(self, x):
        return 0 <= int(x) < self.n
