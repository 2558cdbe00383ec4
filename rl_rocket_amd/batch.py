"""``RocketBatch``: N rocket envs on one GPU behind the C-ABI, torch tensors in and out.

This is the device-resident core that both the SB3-style ``RocketVecEnv`` and the
single-env gym shims (``Rocket6DOF`` / ``Rocket``) sit on.  Every method launches
asynchronously on the current torch stream of the env's device; nothing here
synchronises except ``fetch_done``.
"""
import ctypes

import numpy as np

from . import _lib
from .params import lower, make_config


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _host_view(addr, shape, dtype):
    """numpy array over `addr` (memory the library owns; valid while it does)."""
    nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
    return np.frombuffer((ctypes.c_char * nbytes).from_address(addr), dtype=dtype).reshape(shape)


class HostArray:
    """A numpy array in pinned, GPU-coherent host memory (``rr_host_alloc``) that the kernels
    read and write directly: zero-copy step inputs / outputs for small N (``ptr`` is what the
    C-ABI takes). Freed by ``free()`` (or when collected); views of ``array`` must not outlive it."""

    def __init__(self, shape, dtype):
        self._lib = _lib.load()
        nbytes = max(1, int(np.prod(shape)) * np.dtype(dtype).itemsize)
        p = ctypes.c_void_p()
        _lib.check(self._lib.rr_host_alloc(ctypes.byref(p), nbytes), "rr_host_alloc")
        self.ptr = p
        self.array = _host_view(p.value, shape, dtype)

    def free(self):
        if getattr(self, "ptr", None) is not None and self.ptr.value:
            self.array = None
            self._lib.rr_host_free(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class OutputSet(tuple):
    """(obs, reward, done, truncated) device views of one contiguous block (`block`, uint8)."""

    def __new__(cls, views, block):
        self = super().__new__(cls, views)
        self.block = block
        return self


class RocketBatch:
    def __init__(self, num_envs, model="6DOF", device=None, max_episode_steps=0, auto_reset=True,
                 episode_stats=True, reward_annealing=False, integrator="rk4", env_id_offset=0,
                 compute_terms=False, seed=None, scipy_h0_clamp=False, action_soa=False, host_state=False,
                 **env_kwargs):
        import torch

        self.torch = torch
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device)
        if device.type != "cuda":
            raise ValueError("RocketBatch runs on a GPU (HIP) device; got %s — there is no CPU fallback" % device)
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.cfg = make_config(model, **env_kwargs)
        self.model = self.cfg.model
        self.num_envs = int(num_envs)
        self.state_dim = self.cfg.state_dim
        self.action_dim = self.cfg.action_dim
        self.n_terms = len(self.cfg.term_names)
        self.params = lower(self.cfg, max_episode_steps=max_episode_steps, auto_reset=auto_reset,
                            episode_stats=episode_stats, reward_annealing=reward_annealing, integrator=integrator,
                            scipy_h0_clamp=scipy_h0_clamp, action_soa=action_soa, host_state=host_state)
        # host_state: the state planes (+ v0, counter words, returns) in pinned host memory
        # (RR_FLAG_HOST_STATE), readable through host_state_arrays() after a stream synchronise
        self.host_state = bool(host_state)
        # action_soa: step() takes actions as [action_dim][N] planes (RR_FLAG_ACTION_SOA)
        self.action_soa = bool(action_soa)
        self.lib = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(self.lib.rr_create(ctypes.byref(h), ctypes.byref(self.params), self.num_envs, int(env_id_offset),
                                      device.index), "rr_create")
        self._h = h
        self.env_id_offset = int(env_id_offset)
        n = self.num_envs
        self.outputs = self.alloc_outputs()
        self.obs, self.reward, self.done, self.truncated = self.outputs
        self.terms = torch.empty((self.n_terms + 2, n), dtype=torch.float32, device=device) if compute_terms else None
        self.seed(self.cfg.kwargs["seed"] if seed is None else seed)

    # -- plumbing ---------------------------------------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def _upload(self, action):
        """Host (numpy) actions -> the device through a persistent pinned staging buffer and an
        asynchronous copy (pageable H2D goes through the runtime's bounce buffers, ~10x slower);
        an event guards the staging buffer against reuse before its previous copy has run."""
        t = self.torch
        a = np.asarray(action, dtype=np.float32)
        shape = (self.action_dim, self.num_envs) if self.action_soa else (self.num_envs, self.action_dim)
        if a.size != self.num_envs * self.action_dim:
            raise ValueError("expected %d actions, got shape %s" % (self.num_envs * self.action_dim, a.shape))
        # one (pinned, device) staging pair per stream: the device copy is only written and read in
        # the order of its own stream, so a step still reading it on stream A cannot be overwritten
        # by an upload issued on stream B
        stream = t.cuda.current_stream(self.device)
        stages = self.__dict__.setdefault("_stages", {})
        st = stages.get(stream.cuda_stream)
        if st is None:
            st = stages[stream.cuda_stream] = (t.empty(shape, dtype=t.float32, pin_memory=True),
                                               t.empty(shape, dtype=t.float32, device=self.device), t.cuda.Event())
        pin, dev, ev = st
        ev.synchronize()  # the previous upload has left the pinned buffer
        np.copyto(pin.numpy(), a.reshape(shape))
        dev.copy_(pin, non_blocking=True)
        ev.record(stream)
        return dev

    def _check_action(self, action):
        t = self.torch
        if not isinstance(action, t.Tensor):
            action = self._upload(action)
        if action.device != self.device:
            action = action.to(self.device, non_blocking=True)
        if action.dtype != t.float32:
            action = action.float()
        action = action.reshape((self.action_dim, self.num_envs) if self.action_soa else (self.num_envs, self.action_dim))
        if not action.is_contiguous():
            action = action.contiguous()
        return action

    # -- API --------------------------------------------------------------------------------------------------
    def seed(self, seed):
        _lib.check(self.lib.rr_seed(self._h, int(seed) & (2 ** 64 - 1), self._stream()), "rr_seed")

    def reset(self, mask=None, obs=None):
        """Fresh initial conditions for the envs where mask != 0 (all when None); writes the
        obs of every env into `obs` (default: the env's own obs tensor) and returns it."""
        m = None
        if mask is not None:
            m = self.torch.as_tensor(mask, device=self.device).to(self.torch.uint8).contiguous()
        obs = self.obs if obs is None else obs
        _lib.check(self.lib.rr_reset(self._h, _ptr(m), _ptr(obs), self._stream()), "rr_reset")
        return obs

    def alloc_outputs(self):
        """A fresh set of step output tensors (obs [N,ns] f32, reward [N] f32, done [N] u8, truncated
        [N] u8) for step(out=...): views of ONE contiguous device block in that order, so that a
        host copy of all four is one DMA (the returned tuple's `.block`)."""
        t = self.torch
        n, ns = self.num_envs, self.state_dim
        o_b, r_b = 4 * n * ns, 4 * n
        blk = t.empty((o_b + r_b + 2 * n,), dtype=t.uint8, device=self.device)
        return OutputSet((blk[:o_b].view(t.float32).view(n, ns), blk[o_b:o_b + r_b].view(t.float32),
                          blk[o_b + r_b:o_b + r_b + n], blk[o_b + r_b + n:]), blk)

    def step(self, action, out=None):
        """One env step for all envs. Returns the output tensors (obs [N,ns], reward [N], done
        [N] u8, truncated [N] u8): the env's own, reused by every step, or the set `out`
        (alloc_outputs(); e.g. double-buffered outputs that stay valid for one more step)."""
        action = self._check_action(action)
        self._last_action = action  # keep alive until the kernel has run
        obs, rew, done, trunc = out if out is not None else (self.obs, self.reward, self.done, self.truncated)
        _lib.check(self.lib.rr_step(self._h, _ptr(action), _ptr(obs), _ptr(rew), _ptr(done), _ptr(trunc),
                                    _ptr(self.terms), self._stream()), "rr_step")
        return obs, rew, done, trunc

    def step_rows(self, action, rows):
        """One env step writing obs, reward and done as rows [N, state_dim + 2] fp32 (obs,
        reward, done 0 / 1) into the device tensor `rows` (rr_step_rows; e.g. an all-gather
        send buffer). Returns `rows`; truncated / terms as step()."""
        t = self.torch
        if rows.shape != (self.num_envs, self.state_dim + 2) or rows.dtype != t.float32 or not rows.is_contiguous() \
                or rows.device != self.device:
            raise ValueError("rows must be a contiguous float32 [%d, %d] tensor on %s"
                             % (self.num_envs, self.state_dim + 2, self.device))
        action = self._check_action(action)
        self._last_action = action
        _lib.check(self.lib.rr_step_rows(self._h, _ptr(action), _ptr(rows), _ptr(self.truncated), _ptr(self.terms),
                                         self._stream()), "rr_step_rows")
        return rows

    def step_repeat(self, actions, n_steps):
        """`n_steps` consecutive steps, step t taking action batch t % len(actions) of the device
        tensor `actions` [B][N][action_dim] (rr_step_repeat: one host call, direct dispatch).
        Returns the output tensors of the last step."""
        t = self.torch
        if not isinstance(actions, t.Tensor) or actions.device != self.device or actions.dtype != t.float32:
            raise TypeError("actions must be a float32 tensor on %s" % self.device)
        shape = (self.action_dim, self.num_envs) if self.action_soa else (self.num_envs, self.action_dim)
        actions = actions.reshape((-1,) + shape).contiguous()
        self._last_action = actions
        _lib.check(self.lib.rr_step_repeat(self._h, _ptr(actions), actions.shape[0], int(n_steps), _ptr(self.obs),
                                           _ptr(self.reward), _ptr(self.done), _ptr(self.truncated), _ptr(self.terms),
                                           self._stream()), "rr_step_repeat")
        return self.obs, self.reward, self.done, self.truncated

    def set_state(self, state_soa, v0=None, elapsed=None):
        """Inject fp32 state planes [state_dim][N]; v0 [N] (kept when None); `elapsed` = counter
        words [N] (a plain step count below 2^counter_bits is episode 0 — build words for larger
        values with make_counter(), which range-checks them; None clears the steps and keeps the
        episode field). Zeroes the Monitor running return (restore() keeps it)."""
        t = self.torch
        st = t.as_tensor(state_soa, device=self.device, dtype=t.float32).reshape(self.state_dim, self.num_envs)
        st = st.contiguous()
        v = None if v0 is None else t.as_tensor(v0, device=self.device, dtype=t.float32).reshape(-1).contiguous()
        el = None if elapsed is None else t.as_tensor(elapsed, device=self.device, dtype=t.int32).reshape(-1).contiguous()
        self._keep = (st, v, el)
        _lib.check(self.lib.rr_set_state(self._h, _ptr(st), _ptr(v), _ptr(el), self._stream()), "rr_set_state")

    def get_state(self):
        t = self.torch
        st = t.empty((self.state_dim, self.num_envs), dtype=t.float32, device=self.device)
        v = t.empty((self.num_envs,), dtype=t.float32, device=self.device)
        el = t.empty((self.num_envs,), dtype=t.int32, device=self.device)
        _lib.check(self.lib.rr_get_state(self._h, _ptr(st), _ptr(v), _ptr(el), self._stream()), "rr_get_state")
        return st, v, el

    def host_state_arrays(self):
        """(state [state_dim][N] f32, v0 [N] f32, counter words [N] u32) as numpy views of the
        library's pinned host planes (host_state=True only). They reflect the last step once the
        stream has been synchronised; valid until close()."""
        if not self.host_state:
            raise ValueError("host_state_arrays() needs RocketBatch(host_state=True)")
        b = _lib.RrBuffers()
        _lib.check(self.lib.rr_get_buffers(self._h, ctypes.byref(b)), "rr_get_buffers")
        n, ns = self.num_envs, self.state_dim
        return (_host_view(b.state, (ns, n), np.float32), _host_view(b.v0, (n,), np.float32),
                _host_view(b.elapsed, (n,), np.uint32))

    # -- counter words and checkpoints ---------------------------------------------------------------------------
    @property
    def counter_bits(self):
        """Bits E of the elapsed-steps field of the counter word (episode number in bits E..31)."""
        return _lib.check(self.lib.rr_counter_bits(self._h), "rr_counter_bits")

    def split_counter(self, counter):
        """(elapsed steps, episode number) of counter words (tensor or array)."""
        e = self.counter_bits
        c = counter.to(self.torch.int64) & 0xFFFFFFFF if isinstance(counter, self.torch.Tensor) else \
            np.asarray(counter).astype(np.int64) & 0xFFFFFFFF
        return c & ((1 << e) - 1), c >> e

    def make_counter(self, elapsed, episode=0):
        """Counter words from elapsed steps and episode numbers (int32 view of the u32 word).
        Raises if an elapsed count does not fit the E-bit field (it would spill into the episode
        field, which keys the reset stream) or an episode number the 32 - E bits above it."""
        e = self.counter_bits
        el = np.asarray(elapsed, np.int64)
        ep = np.asarray(episode, np.int64)
        if (el < 0).any() or (el >= (1 << e)).any():
            raise ValueError("elapsed steps must be in [0, %d) (the counter word's %d-bit field)" % (1 << e, e))
        if (ep < 0).any() or (ep >= (1 << (32 - e))).any():
            raise ValueError("episode numbers must be in [0, 2^%d)" % (32 - e))
        w = (ep << e) | el
        return (w & 0xFFFFFFFF).astype(np.uint32).view(np.int32)

    def checkpoint(self):
        """Everything a restore needs, as device tensors: state planes, v0, raw counter words
        (TimeLimit steps | episode: keys the reset stream) and Monitor running returns."""
        t = self.torch
        st, v0, _ = self.get_state()
        cw = t.empty((self.num_envs,), dtype=t.int32, device=self.device)
        ret = t.empty((self.num_envs,), dtype=t.float32, device=self.device)
        _lib.check(self.lib.rr_get_aux(self._h, _ptr(cw), _ptr(ret), self._stream()), "rr_get_aux")
        return {"state": st, "v0": v0, "counter": cw, "ep_return": ret}

    def restore(self, ck):
        """Inverse of checkpoint(): the next steps are bitwise those of the checkpointed env."""
        self.set_state(ck["state"], v0=ck["v0"], elapsed=ck["counter"])
        cw, ret = ck["counter"].contiguous(), ck["ep_return"].contiguous()
        self._keep_aux = (cw, ret)
        _lib.check(self.lib.rr_set_aux(self._h, _ptr(cw), _ptr(ret), self._stream()), "rr_set_aux")

    def set_state64(self, state_soa, v0=None, elapsed=None):
        """fp64 state [state_dim][N] (the integrator's own state under integrator="dopri5";
        elapsed also sets the simulator clock t = steps * dt there)."""
        t = self.torch
        st = t.as_tensor(state_soa, device=self.device, dtype=t.float64).reshape(self.state_dim, self.num_envs)
        st = st.contiguous()
        v = None if v0 is None else t.as_tensor(v0, device=self.device, dtype=t.float32).reshape(-1).contiguous()
        el = None if elapsed is None else t.as_tensor(elapsed, device=self.device, dtype=t.int32).reshape(-1).contiguous()
        self._keep = (st, v, el)
        _lib.check(self.lib.rr_set_state64(self._h, _ptr(st), _ptr(v), _ptr(el), self._stream()), "rr_set_state64")

    def get_state64(self):
        t = self.torch
        st = t.empty((self.state_dim, self.num_envs), dtype=t.float64, device=self.device)
        v = t.empty((self.num_envs,), dtype=t.float32, device=self.device)
        el = t.empty((self.num_envs,), dtype=t.int32, device=self.device)
        _lib.check(self.lib.rr_get_state64(self._h, _ptr(st), _ptr(v), _ptr(el), self._stream()), "rr_get_state64")
        return st, v, el

    def fetch_done(self, capacity=None):
        """Done list of the last step on the host: (idx, terminal_obs, episode_return, episode_len),
        fresh arrays of the done rows. Synchronises the stream. The rows land in persistent pinned
        buffers (rr_host_alloc: the copies go straight to them instead of through the runtime's
        staging of pageable memory), sized to the largest done list seen (at least 4096 rows; a
        longer list grows them and is fetched again), and are copied out."""
        cap = self.num_envs if capacity is None else min(int(capacity), self.num_envs)
        rows = min(cap, max(4096, len(self._fetch[0].array) if getattr(self, "_fetch", None) else 0))
        while True:
            if getattr(self, "_fetch", None) is None or len(self._fetch[0].array) < rows:
                self._free_fetch()  # grown on demand (~1 % of the envs finish per step): not N rows up front
                ns = self.state_dim
                self._fetch = (HostArray((rows,), np.int32), HostArray((rows, ns), np.float32),
                               HostArray((rows,), np.float32), HostArray((rows,), np.int32))
            bufs = self._fetch
            c = self.lib.rr_fetch_done(self._h, min(cap, rows), *(b.ptr for b in bufs), self._stream())
            _lib.check(c, "rr_fetch_done")
            if int(c) <= rows or rows >= cap:
                break
            rows = min(cap, 1 << (int(c) - 1).bit_length())  # more done envs than rows: grow, fetch again
        m = min(int(c), cap)
        return tuple(b.array[:m].copy() for b in bufs)

    def _free_fetch(self):
        for b in getattr(self, "_fetch", None) or ():
            b.free()
        self._fetch = None

    def copy_terminal(self, out=None):
        """Device copies of the terminal rows of the envs done at the last step (rr_copy_terminal:
        only those rows are written). `out` = preallocated (obs [N,ns] f32, return [N] f32, len
        [N] i32), any may be None; by default fresh zero-filled tensors."""
        t = self.torch
        if out is None:
            out = (t.zeros((self.num_envs, self.state_dim), dtype=t.float32, device=self.device),
                   t.zeros((self.num_envs,), dtype=t.float32, device=self.device),
                   t.zeros((self.num_envs,), dtype=t.int32, device=self.device))
        tobs, ret, ln = out
        _lib.check(self.lib.rr_copy_terminal(self._h, _ptr(tobs), _ptr(ret), _ptr(ln), self._stream()),
                   "rr_copy_terminal")
        return tobs, ret, ln

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.torch.cuda.synchronize(self.device)
            self.lib.rr_destroy(self._h)
            self._h = ctypes.c_void_p()
        self._free_fetch()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
