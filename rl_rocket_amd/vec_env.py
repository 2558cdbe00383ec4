"""``RocketVecEnv``: a stable-baselines3 ``VecEnv`` over N GPU-resident rocket envs.

Equivalent, for SB3's PPO, to ``DummyVecEnv([make_env] * N)`` with
``make_env`` = ``gym.make(id, **env_config)`` -> ``TimeLimit(max_episode_steps)``
-> ``Monitor`` (reference main_6DOF.py:18-24), but stepped by ONE launch of the
fused HIP kernel for all N envs:

  * on-device auto-reset; ``infos[i]["terminal_observation"]`` holds the final
    observation of a done env and ``infos[i]["TimeLimit.truncated"]`` is set on
    time-outs, exactly as SB3 1.6 DummyVecEnv + gym 0.21 TimeLimit do;
  * Monitor episode statistics ``infos[i]["episode"] = {"r", "l", "t"}`` for done envs;
  * ``infos`` is a lazy sequence: dicts are only materialised for done envs (and
    ``rewards_dict`` / ``bounds_violation`` only when ``info_terms=True``), so the
    host cost per step is O(#done), not O(N) dict building.

``device_outputs=True`` returns torch tensors that stay in HBM (no host copy);
otherwise numpy arrays as SB3 expects. Device outputs are double-buffered: the tensors
returned by step t (and reset) stay unchanged through step t + 1 and are overwritten by
step t + 2 — what SB3's collect_rollouts needs (it stores ``_last_obs`` from step t after
stepping t + 1). Their ``infos`` are built lazily from a per-step device snapshot (done /
truncated flags and the terminal rows of THAT step's done envs, copied device to device), so
reading them late still describes their own step. With ``monitor=True`` infos nobody reads are
built before their snapshot is reused, so every finished episode reaches the Monitor statistics
in step order; without it an unread snapshot is dropped unbuilt and nothing leaves HBM.

Late reads (device outputs, ``monitor=False``): the infos of step t must be read (indexed,
iterated or ``materialize()``-d) before step t + 2 — SB3's collect_rollouts reads them at once.
A wrapper or callback that keeps an unread infos object across two more steps gets a
RuntimeError on its first access, where DummyVecEnv's plain list would still answer; call
``materialize()`` on it before stepping on to keep it.
"""
import itertools
import time
from collections.abc import Sequence

import numpy as np

from . import _lib
from .batch import RocketBatch
from .gym_compat import Box
from .params import MAX_EPISODE_STEPS, parse_model

try:  # pragma: no cover - SB3 is optional (absent from this image)
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _VecEnvBase
except Exception:  # pragma: no cover
    _VecEnvBase = object


class _DoneRows:
    """The envs that finished at one step, as arrays (env index, terminal obs row, episode
    return / length, truncation flag); their info dicts are built on first access."""

    def __init__(self, idx, tobs, ret, ln, trunc, max_episode_steps, monitor, stamp):
        self.idx = np.asarray(idx)
        self._pos = None  # env index -> row, built on the first info() (most steps' infos are never read)
        self.tobs, self.ret, self.ln, self.trunc = tobs, ret, ln, trunc
        self.max_steps = max_episode_steps
        self.monitor = monitor
        self.stamp = stamp

    @property
    def pos(self):
        if self._pos is None:
            self._pos = dict(zip(self.idx.tolist(), range(len(self.idx))))
        return self._pos

    def info(self, i):
        """SB3 DummyVecEnv + gym TimeLimit + Monitor info of done env i (None if not done)."""
        k = self.pos.get(i)
        if k is None:
            return None
        return self._dict(k, self.tobs[k], bool(self.trunc[k]), float(self.ret[k]), int(self.ln[k]))

    def _dict(self, k, tobs, trunc, ret, ln):
        d = {"terminal_observation": tobs}
        if trunc:
            d["TimeLimit.truncated"] = True
        elif self.max_steps and ln >= self.max_steps:
            d["TimeLimit.truncated"] = False
        if self.monitor:
            d["episode"] = {"r": round(ret, 6), "l": ln, "t": self.stamp}
        return d

    def items(self):
        """(env index, info dict) of every done env, built in one pass over the arrays."""
        tobs = list(self.tobs)  # row views
        return [(i, self._dict(k, tobs[k], t, r, ln)) for k, (i, t, r, ln) in
                enumerate(zip(self.idx.tolist(), self.trunc.astype(bool).tolist(), self.ret.tolist(),
                              self.ln.tolist()))]


class LazyInfos(Sequence):
    """SB3 ``infos`` list whose dicts are built on access: {} for running envs (plus
    ``rewards_dict`` / ``bounds_violation`` with info_terms), the done envs' dicts from their
    arrays (``_DoneRows``).

    Indexing builds one dict (the done envs SB3 looks at cost O(#done)); iterating — what SB3
    1.6 ``collect_rollouts`` -> ``_update_info_buffer`` does with every step's infos — builds the
    whole list once, in one list comprehension with the done envs' dicts spliced in, and
    iterates that plain list (``Sequence.__iter__`` would call ``__getitem__`` N times, ~10x
    slower at N = 65 536). Every env's dict is its own object, as in DummyVecEnv, and indexing
    after iterating returns the same objects."""

    def __init__(self, n, done_rows=None, terms=None, term_names=None):
        self._n = n
        self._rows = done_rows          # _DoneRows or None
        self._terms = terms             # host [n_terms+2, N] array or None
        self._names = term_names
        self._cache = {}
        self._list = None               # the materialised list (first __iter__)

    def __len__(self):
        return self._n

    def _terms_of(self, i, d):
        t = self._terms
        d["rewards_dict"] = {k: float(t[j, i]) for j, k in enumerate(self._names)}
        d["bounds_violation"] = bool(t[len(self._names), i] > 0.5)
        return d

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(self._n))]
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError(i)
        if self._list is not None:
            return self._list[i]
        d = self._cache.get(i)
        if d is None:
            d = (self._rows.info(i) if self._rows is not None else None)
            if d is None:
                d = {}
            if self._terms is not None:
                self._terms_of(i, d)
            self._cache[i] = d
        return d

    def materialize(self):
        """The infos as a plain list of N dicts (built once; dicts already handed out by
        indexing are kept)."""
        if self._list is None:
            n = self._n
            if self._terms is None:
                lst = list(itertools.starmap(dict, itertools.repeat((), n)))  # N fresh dicts, ~25 % under a comprehension
            else:  # info_terms: every env's dict carries its reward terms (opt-in, O(N) by nature)
                lst = [self._terms_of(i, {}) for i in range(n)]
            if self._rows is not None:
                for i, d in self._rows.items():
                    if self._terms is not None:
                        d.update(lst[i])
                    lst[i] = d
            for i, d in self._cache.items():
                lst[i] = d
            self._list, self._cache = lst, {}
        return self._list

    def __iter__(self):
        return iter(self.materialize())

    def done_indices(self):
        return [] if self._rows is None else self._rows.idx.tolist()


class _DeviceInfos(LazyInfos):
    """infos of one device-output step, built on first access (or, with Monitor, before the
    step's snapshot is reused) from that step's own done / truncated flags and terminal rows."""

    def __init__(self, venv, slot, stamp):
        super().__init__(venv.num_envs)
        self._venv, self._slot = venv, slot
        self._stamp = stamp  # Monitor's episode "t" of this step (taken when the step ran)
        self._built = None

    def _build(self):
        if self._built is None:
            v = self._venv
            while v._pending and v._pending[0] is not self:  # earlier steps first (Monitor order)
                v._pending[0]._build()
            _, _, done, trunc = self._slot["out"]
            rows = v._gather_done(done, trunc, self._slot["term"], self._stamp)
            terms = self._slot["terms"]
            self._built = LazyInfos(v.num_envs, rows, None if terms is None else terms.cpu().numpy(),
                                    v.cfg.term_names)
            if v._pending and v._pending[0] is self:
                v._pending.pop(0)
            self._slot["infos"] = None
        return self._built

    def _drop(self):
        """Discard unbuilt: the snapshot is reused; reading these infos later raises."""
        v = self._venv
        if self in v._pending:
            v._pending.remove(self)
        self._slot["infos"] = None
        self._slot = None

    def __len__(self):
        return self._n

    def _live(self):
        if self._built is None and self._slot is None:
            raise RuntimeError("the infos of this step were read after their snapshot was reused (two steps "
                               "later); with monitor=False unread infos are not kept")
        return self._build()

    def __getitem__(self, i):
        return self._live()[i]

    def __iter__(self):
        return iter(self._live())

    def materialize(self):
        return self._live().materialize()

    def done_indices(self):
        if self._built is None and self._slot is None:
            raise RuntimeError("the infos of this step were read after their snapshot was reused")
        return self._build().done_indices()


class RocketVecEnv(_VecEnvBase):
    metadata = {"render.modes": []}

    def __init__(self, num_envs, model="6DOF", device=None, max_episode_steps=MAX_EPISODE_STEPS, monitor=True,
                 reward_annealing=False, integrator="rk4", info_terms=False, device_outputs=False,
                 env_id_offset=0, seed=None, **env_kwargs):
        self.model = parse_model(model)
        self.batch = RocketBatch(num_envs, model=self.model, device=device, max_episode_steps=max_episode_steps,
                                 auto_reset=True, episode_stats=monitor, reward_annealing=reward_annealing,
                                 integrator=integrator, env_id_offset=env_id_offset, compute_terms=info_terms,
                                 seed=seed, **env_kwargs)
        ns, na = self.batch.state_dim, self.batch.action_dim
        self.num_envs = int(num_envs)
        self.observation_space = Box(low=-1, high=1, shape=(ns,)).to_gym()
        self.action_space = Box(low=-1, high=1, shape=(na,)).to_gym()
        self.monitor = monitor
        self.info_terms = info_terms
        self.device_outputs = device_outputs
        self.max_episode_steps = max_episode_steps
        self._actions = None
        self._t_start = time.time()
        self.episode_returns = []
        self.episode_lengths = []
        self.episode_times = []
        self.total_steps = 0
        # cost split of step_wait (bench.py's SB3 legs): a dict the caller sets, accumulating
        # seconds per stage ("launch", "kernel", "d2h", "infos"); None = no timing
        self.timing = None
        self.cfg = self.batch.cfg
        self.state_names = self.batch.cfg.state_names if hasattr(self.batch.cfg, "state_names") else None
        if device_outputs:
            self._init_device_sets()

    # -- VecEnv API ------------------------------------------------------------------------------------------
    def reset(self):
        if self.device_outputs:
            self._flush_all()
            self._slot = 0
            return self.batch.reset(obs=self._sets[0]["out"][0])
        obs = self.batch.reset()
        return obs.cpu().numpy()

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self):
        self.total_steps += self.num_envs
        if self.device_outputs:
            return self._step_device()
        tm = self.timing
        if tm is not None:
            t0 = time.perf_counter()
        obs, rew, done, trunc = self.batch.step(self._actions)
        if tm is not None:  # the kernel's remaining device time, split from the copies
            t1 = time.perf_counter()
            self.batch.torch.cuda.synchronize(self.batch.device)
            t2 = time.perf_counter()
        # obs / reward / done / truncated as DMA copies into ONE fresh pinned block (PyTorch's
        # caching host allocator: after warm-up no pinning or page faults) and one synchronise;
        # the numpy arrays are views that keep the block alive, so every step's arrays are its own
        # (SB3 keeps _last_obs across the next step) and nothing is copied twice on the host
        obs_h, rew_h, done_h, trunc_h = self._to_host(obs, rew, done, trunc)
        if tm is not None:
            t3 = time.perf_counter()
        rows = None
        if done_h.any():
            idx, tobs, ret, ln = self.batch.fetch_done()
            rows = self._done_rows(idx, tobs, ret, ln, trunc_h[idx], self._now())
        infos = LazyInfos(self.num_envs, rows, self.batch.terms.cpu().numpy() if self.info_terms else None,
                          self.cfg.term_names)
        if tm is not None:
            t4 = time.perf_counter()
            for k, v in (("launch", t1 - t0), ("kernel", t2 - t1), ("d2h", t3 - t2), ("infos", t4 - t3)):
                tm[k] = tm.get(k, 0.0) + v
        return obs_h, rew_h, done_h, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def _to_host(self, obs, rew, done, trunc):
        """The four step outputs as numpy views of one fresh pinned block (obs [N][ns] f32,
        reward [N] f32, done [N] bool, truncated [N] u8), after one stream synchronise. The
        batch's outputs are views of one device block in the same layout (RocketBatch.alloc_outputs),
        so this is ONE DMA copy."""
        t, n, ns = self.batch.torch, self.num_envs, self.batch.state_dim
        o_b, r_b = 4 * n * ns, 4 * n
        blk = t.empty((o_b + r_b + 2 * n,), dtype=t.uint8, pin_memory=True)
        views = (blk[:o_b].view(t.float32).view(n, ns), blk[o_b:o_b + r_b].view(t.float32),
                 blk[o_b + r_b:o_b + r_b + n], blk[o_b + r_b + n:])
        src_blk = getattr(getattr(self.batch, "outputs", None), "block", None)
        if src_blk is not None and obs is self.batch.obs:
            blk.copy_(src_blk, non_blocking=True)
        else:
            for dst, src in zip(views, (obs, rew, done, trunc)):
                dst.copy_(src, non_blocking=True)
        t.cuda.current_stream(self.batch.device).synchronize()
        o, r, d, tr = (v.numpy() for v in views)
        return o, r, d.view(np.bool_), tr  # the kernel writes done as 0 / 1

    def _now(self):
        return round(time.time() - self._t_start, 6)

    def _done_rows(self, idx, tobs, ret, ln, trunc_k, now):
        """The done envs of a step (SB3 DummyVecEnv + TimeLimit + Monitor); Monitor statistics
        recorded here, vectorised (episode "t" = `now`, the time of the step that ended them)."""
        if self.monitor:
            self.episode_returns.extend(ret.tolist())
            self.episode_lengths.extend(ln.tolist())
            self.episode_times.extend([now] * len(idx))
        return _DoneRows(idx, tobs, ret, ln, trunc_k, self.max_episode_steps, self.monitor, now)

    # -- device outputs: double-buffered step outputs + per-step snapshots for the lazy infos ---------------
    def _init_device_sets(self):
        t = self.batch.torch
        n, ns, dev = self.num_envs, self.batch.state_dim, self.batch.device
        self._sets = []
        for _ in range(2):
            self._sets.append({
                "out": self.batch.alloc_outputs(),
                "term": (t.empty((n, ns), dtype=t.float32, device=dev), t.empty((n,), dtype=t.float32, device=dev),
                         t.empty((n,), dtype=t.int32, device=dev)),
                "terms": None if self.batch.terms is None else t.empty_like(self.batch.terms),
                "infos": None,
            })
        self._slot = 0
        self._pending = []  # unbuilt _DeviceInfos in step order
        self._gbuf = {}  # pinned host rows of _gather_done, allocated at its first use

    def _gather_done(self, done, trunc, term, stamp):
        """The done envs of a device-output step as host arrays: ONE library call (rr_gather_rows)
        reads that step's done flags, gathers the done rows of its snapshot (terminal obs, return,
        length, truncated) on the device into pinned host buffers and synchronises once."""
        import ctypes

        from .batch import HostArray

        n, ns = self.num_envs, self.batch.state_dim
        g = self._gbuf
        if g.get("rows") is None:
            g["rows"] = (HostArray((n,), np.int32), HostArray((n, ns), np.float32), HostArray((n,), np.float32),
                         HostArray((n,), np.int32), HostArray((n,), np.uint8))
        h = g["rows"]
        P = ctypes.c_void_p
        tobs, ret, ln = term
        c = self.batch.lib.rr_gather_rows(
            self.batch._h, P(done.data_ptr()), P(tobs.data_ptr()), P(ret.data_ptr()), P(ln.data_ptr()),
            P(trunc.data_ptr()), n, *(b.ptr for b in h), self.batch._stream())
        _lib.check(c, "rr_gather_rows")
        m = int(c)
        if not m:
            return None
        idx, tobs_h, ret_h, ln_h, tr_h = (b.array[:m].copy() for b in h)  # the pinned buffers are reused
        return self._done_rows(idx, tobs_h, ret_h, ln_h, tr_h, stamp)

    def _flush_all(self):
        while self._pending:
            self._pending[0]._build()

    def _step_device(self):
        tm = self.timing
        if tm is not None:
            t0 = time.perf_counter()
        self._slot ^= 1
        st = self._sets[self._slot]
        old = st["infos"]
        if old is not None:  # its snapshot is about to be reused
            if self.monitor:
                old._build()  # Monitor statistics are a side effect: every step's infos are built
            else:
                old._drop()  # nobody read them and building has no effect: drop unbuilt
        if tm is not None:
            t1 = time.perf_counter()
        obs, rew, done, trunc = self.batch.step(self._actions, out=st["out"])
        # this step's terminal rows, device to device: only the rows of the envs done now
        self.batch.copy_terminal(out=st["term"])
        if st["terms"] is not None:
            st["terms"].copy_(self.batch.terms)
        infos = _DeviceInfos(self, st, self._now())
        st["infos"] = infos
        self._pending.append(infos)
        if tm is not None:  # "infos": the Monitor build of step t - 2 (incl. its done-flag copy)
            t2 = time.perf_counter()
            for k, v in (("infos", t1 - t0), ("launch", t2 - t1)):
                tm[k] = tm.get(k, 0.0) + v
        return obs, rew, done.bool(), infos

    def close(self):
        if self.device_outputs and getattr(self, "_pending", None):
            self._flush_all()
        self.batch.close()
        for b in (getattr(self, "_gbuf", None) or {}).get("rows") or ():
            b.free()

    def seed(self, seed=None):
        if seed is None:
            seed = int(np.random.randint(0, 2 ** 31 - 1))
        self.batch.seed(seed)
        return [seed + i for i in range(self.num_envs)]

    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices

    def get_attr(self, attr_name, indices=None):
        value = getattr(self, attr_name, None)
        if value is None:
            value = getattr(self.batch.cfg, attr_name, None)
        if value is None and attr_name in self.batch.cfg.kwargs:
            value = self.batch.cfg.kwargs[attr_name]
        if value is None and attr_name == "reward_coefficients":
            value = self.batch.cfg.kwargs["reward_coeff"]
        return [value for _ in self._indices(indices)]

    def set_attr(self, attr_name, value, indices=None):
        raise AttributeError("RocketVecEnv envs share one device-resident config; %r cannot be set per env"
                             % attr_name)

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        raise AttributeError("RocketVecEnv has no per-env python objects (method %r)" % method_name)

    def env_is_wrapped(self, wrapper_class, indices=None):
        """True for the wrappers the fused step reproduces: SB3's ``Monitor`` (monitor=True; its
        ``info["episode"]`` is what SB3's evaluate_policy reads when this is True) and gym's
        ``TimeLimit`` (max_episode_steps > 0), as in main_6DOF.py:18-24's make_env."""
        name = getattr(wrapper_class, "__name__", "")
        wrapped = (name == "Monitor" and bool(self.monitor)) or (name == "TimeLimit" and bool(self.max_episode_steps))
        return [wrapped for _ in self._indices(indices)]

    def render(self, mode="human"):
        return None

    def get_images(self):
        return []

    @property
    def unwrapped(self):
        return self


class RocketVectorEnv(RocketVecEnv):
    """The same batched env with the ``gym.vector.VectorEnv`` surface of gym 0.21.0 — the
    version the reference pins (requirements.txt:29) — that the north star names:
    ``observation_space`` / ``action_space`` are the BATCHED Boxes (num_envs, dim) and
    ``single_observation_space`` / ``single_action_space`` the per-env ones; ``reset() -> obs``
    (no seed / options keywords, no info), ``step(actions) -> (obs, rewards, dones, infos)`` with
    ``infos`` a LIST of per-env dicts, as gym 0.21's ``SyncVectorEnv.step_wait`` returns, auto-reset
    of done envs and, as there, ``infos[i]["terminal_observation"]`` holding the last obs of a done
    env; ``reset_async`` / ``reset_wait`` / ``step_async`` / ``step_wait`` / ``close`` / ``seed``.
    It does NOT follow the later gym (>= 0.24) / gymnasium vector contract (5-tuple steps,
    dict-of-arrays infos, ``final_observation``). Stepping is the same fused kernel as
    ``RocketVecEnv``, whose SB3 ``VecEnv`` contract shares the list-of-dicts infos and the
    ``terminal_observation`` key."""

    def __init__(self, num_envs, model="6DOF", **kwargs):
        super().__init__(num_envs, model=model, **kwargs)
        ns, na = self.batch.state_dim, self.batch.action_dim
        self.single_observation_space = self.observation_space
        self.single_action_space = self.action_space
        self.observation_space = Box(low=-1, high=1, shape=(self.num_envs, ns)).to_gym()
        self.action_space = Box(low=-1, high=1, shape=(self.num_envs, na)).to_gym()
        self.is_vector_env = True

    def reset_async(self):
        pass

    def reset_wait(self, **kwargs):
        return self.reset()
