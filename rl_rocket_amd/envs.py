"""Single-env gym shims with the reference's API, stepped by the HIP kernel (N = 1).

``Rocket6DOF`` / ``Rocket`` keep the constructor signature, attributes, ``reset`` /
``step`` return types and ``info`` keys of the reference classes
(my_environment/envs/rocket_env.py:505-719 / :19-175), so code written against the
reference (SB3 ``check_env``, ``RewardAnnealing``, ``EpisodeAnalyzer``-style readers of
``info["rewards_dict"]`` and the dataframe helpers) runs unchanged.

Reset draws the initial condition on the host with gym 0.21's ``Box.sample`` and seeding
(``gym_compat``), i.e. the reference's own reset stream, and uploads it with
``rr_set_state``; every ``step`` is one launch of the fused kernel and one stream synchronise:
the env's state lives in pinned host memory (``RR_FLAG_HOST_STATE``) and the action and outputs
in ``rr_host_alloc`` memory, so the kernel reads and writes them in place (no copy commands).  Rendering (pygame /
pyvista, rocket_env.py:249-383, 721-823) is out of scope and raises.
"""
import ctypes

import numpy as np

from . import _lib
from .batch import HostArray, RocketBatch
from .gym_compat import Box, EnvBase
from .params import (ACTION_NAMES_3DOF, ACTION_NAMES_6DOF, MAX_GIMBAL, MAX_THRUST, STATE_NAMES_3DOF,
                     STATE_NAMES_6DOF, config_3dof, config_6dof)


class _SimView:
    """The public surface of ``Simulator6DOF`` / ``Simulator3DOF`` that callers read
    (``states``, ``actions``, ``times``, ``state``, ``t``, ``timestep``; simulator.py:12-86, 179-257)."""

    def __init__(self, ic, dt, n_act):
        self.timestep = dt
        self.t = 0
        self.state = ic
        self.states = [ic]
        self.actions = [[0] * n_act]
        self.times = [0]


class _RocketBase(EnvBase):
    _model = 6

    def _init_common(self, cfg, device):
        kw = cfg.kwargs
        self.cfg = cfg
        self.ICMean = np.float32(kw["IC"])
        self.ICRange = np.float32(kw["ICRange"])
        self.timestep = kw["timestep"]
        self.metadata = dict(self.metadata)
        self.metadata["render_fps"] = 1 / self.timestep
        self.reward_coefficients = kw["reward_coeff"]
        self.init_space = Box(low=cfg.ic_low, high=cfg.ic_high)
        self.seed(kw["seed"])
        self.max_gimbal = MAX_GIMBAL
        self.max_thrust = MAX_THRUST
        self.state_normalizer = cfg.state_normalizer
        ns, na = cfg.state_dim, cfg.action_dim
        self.observation_space = Box(low=-1, high=1, shape=(ns,)).to_gym()
        self.action_space = Box(low=-1, high=1, shape=(na,)).to_gym()
        self.infos = []
        self.SIM = None
        # one step = one launch + one stream synchronise: the env's state planes live in pinned
        # host memory (RR_FLAG_HOST_STATE) and the action and every output in rr_host_alloc
        # memory, so the kernel reads and writes them directly and no copy command is queued
        self._batch = RocketBatch(1, model=cfg.model, device=device, max_episode_steps=0, auto_reset=False,
                                  episode_stats=False, compute_terms=True, host_state=True, **kw)
        nt = len(cfg.term_names)
        self._io = {k: HostArray(shape, dt) for k, shape, dt in (
            ("action", (1, na), np.float32), ("obs", (1, ns), np.float32), ("reward", (1,), np.float32),
            ("done", (1,), np.uint8), ("terms", (nt + 2, 1), np.float32))}
        self._state_h = self._batch.host_state_arrays()[0]
        self._torch = self._batch.torch

    # -- gym API ----------------------------------------------------------------------------------------------
    def seed(self, seed: int = 42):
        self.init_space.seed(seed)
        return [seed]

    def _upload(self, ic):
        import torch

        ns = self.cfg.state_dim
        v = ic[3:6] if self._model == 6 else ic[3:5]
        v0 = np.float32(np.linalg.norm(v.astype(np.float32)))
        self._batch.set_state(torch.from_numpy(ic.astype(np.float32).reshape(ns, 1).copy()),
                              v0=torch.tensor([v0], dtype=torch.float32))

    def _step_device(self, a):
        io, b = self._io, self._batch
        io["action"].array[0] = a
        stream = self._torch.cuda.current_stream(b.device)
        _lib.check(b.lib.rr_step(b._h, io["action"].ptr, io["obs"].ptr, io["reward"].ptr, io["done"].ptr, None,
                                 io["terms"].ptr, ctypes.c_void_p(stream.cuda_stream)), "rr_step")
        stream.synchronize()
        return (io["obs"].array[0].copy(), float(io["reward"].array[0]), bool(io["done"].array[0]),
                io["terms"].array[:, 0].copy(), self._state_h[:, 0].astype(np.float64))

    def render(self, mode="human"):
        raise NotImplementedError("rendering (pygame / pyvista) is out of scope of rl_rocket_amd")

    def close(self):
        if getattr(self, "_batch", None) is not None:
            self._batch.close()  # synchronises the device: no kernel still uses the host buffers
            self._batch = None
            self._state_h = None
            for h in self._io.values():
                h.free()

    def used_mass(self):
        return self.SIM.states[0][-1] - self.SIM.states[-1][-1]

    def states_to_dataframe(self):
        import pandas as pd

        return pd.DataFrame(self.SIM.states, columns=self.state_names)

    def actions_to_dataframe(self):
        import pandas as pd

        return pd.DataFrame(self.SIM.actions, columns=self.action_names)

    def _get_normalizer(self):
        return self.state_normalizer

    @property
    def vtarg_history(self):
        """v_targ of every step since the last reset. The reference appends it inside its reward
        (rocket_env.py:1012 / :245); the kernel computes it there too but does not return it, so
        here it is derived on access from the stored float32-cast states (``SIM.states``), the
        same values, and a step pays nothing for it."""
        sim = self.SIM
        return [] if sim is None else [self._compute_vtarg(np.asarray(s, np.float32)) for s in sim.states[1:]]


class Rocket6DOF(_RocketBase):
    """rocket_env.py:505 ``Rocket6DOF`` over the HIP step kernel."""

    metadata = {"render.modes": ["human", "rgb_array"], "render_fps": 30}
    _model = 6

    def __init__(self, IC=None, ICRange=None, timestep=0.1, seed=42, reward_coeff=None, trajectory_limits=None,
                 landing_params=None, device=None):
        kw = {k: v for k, v in dict(IC=IC, ICRange=ICRange, timestep=timestep, seed=seed,
                                     reward_coeff=reward_coeff, trajectory_limits=trajectory_limits,
                                     landing_params=landing_params).items() if v is not None}
        cfg = config_6dof(**kw)
        self.state_names = list(STATE_NAMES_6DOF)
        self.action_names = list(ACTION_NAMES_6DOF)
        self._init_common(cfg, device)
        e = cfg.extra
        self.position_bounds_space = Box(low=e["bounds_low"], high=e["bounds_high"], dtype=np.float32)
        self.state = None
        self.action = np.array([0.0, 0.0, 0.0])
        self.attitude_traj_limit = e["attitude_limit"]
        self.target_r = e["landing_radius"]
        self.maximum_v = e["maximum_velocity"]
        self.landing_target = [0, 0, 0]
        self.landing_attitude_limit = e["landing_attitude_limit"]
        self.omega_lim = np.array([0.2, 0.2, 0.2])
        self.waypoint = e["waypoint"]
        self.initial_condition = None

    def reset(self):
        """rocket_env.py:665-688"""
        ic = self.init_space.sample()
        ic[6:10] = ic[6:10] / np.linalg.norm(ic[6:10])
        self.initial_condition = ic
        self.state = ic
        self.SIM = _SimView(ic, self.timestep, 3)
        self._upload(ic)
        return self._get_obs()

    def step(self, normalized_action):
        """rocket_env.py:690-719"""
        a = np.asarray(normalized_action, dtype=np.float32).reshape(3)
        self.action = self._denormalize_action(a)
        obs, reward, done, terms, state = self._step_device(a)
        self.state = state
        self.SIM.state = state
        self.SIM.t = round(self.SIM.t + self.timestep, 3)
        self.SIM.times.append(self.SIM.t)
        self.SIM.states.append(state)
        self.SIM.actions.append(self.action)
        rewards_dict = {k: float(terms[j]) for j, k in enumerate(self.cfg.term_names)}
        info = {
            "rewards_dict": rewards_dict,
            "is_done": done,
            "state_history": self.SIM.states,
            "action_history": self.SIM.actions,
            "timesteps": self.SIM.times,
            "bounds_violation": bool(terms[len(self.cfg.term_names)] > 0.5),
        }
        return obs, reward, done, info

    def _denormalize_action(self, action):
        """rocket_env.py:969-981 (no clipping)"""
        gimbal_y = action[0] * self.max_gimbal
        gimbal_z = action[1] * self.max_gimbal
        thrust = (action[2] + 1) / 2.0 * self.max_thrust
        return np.float32([gimbal_y, gimbal_z, thrust])

    def _normalize_obs(self, obs):
        return (obs / self.state_normalizer).astype("float32")

    def _get_obs(self):
        return self._normalize_obs(self.state)

    def _compute_vtarg(self, state32):
        """rocket_env.py:986-1014 (host side, for vtarg_history only)."""
        r, v = state32[0:3].astype(np.float64), state32[3:6].astype(np.float64)
        v_0 = np.linalg.norm(np.asarray(self.SIM.states[0][3:6], dtype=np.float32))
        if r[0] > self.waypoint:
            r_hat = r - [self.waypoint, 0, 0]
            v_hat = v - [-2, 0, 0]
            tau = 20
        else:
            r_hat = np.array([r[0] + 1, 0, 0])
            v_hat = v - [-1, 0, 0]
            tau = 100
        t_go = np.linalg.norm(r_hat) / np.linalg.norm(v_hat)
        return -v_0 * (r_hat / max(1e-3, np.linalg.norm(r_hat))) * (1 - np.exp(-t_go / tau))

    def vtarg_to_dataframe(self):
        import pandas as pd

        return pd.DataFrame(self.vtarg_history, columns=["v_x", "v_y", "v_z"])

    # -- episode figures read by EpisodeAnalyzer (rocket_env.py:861-950) ------------------------------------
    # The reference's three figures (3D path with velocity cones over the landing pad, 3D path with the
    # target-velocity field and the landing target, the quaternion's components over time), built here by
    # one helper on plotly.graph_objects (imported lazily: plotting is off the step path).
    @staticmethod
    def _go():
        try:
            import plotly.graph_objects as go
        except ImportError as e:  # pragma: no cover - plotly ships with this image
            raise ImportError("the episode figures (get_trajectory_plotly & co.) need plotly") from e
        return go

    def _path_figure(self, arrows, pad=False, target=False):
        """The episode's 3D path (x altitude, y, z), `arrows` = (u, v, w) columns drawn as cones along
        it, optionally the landing pad (a disc of radius target_r in the x = 0 plane) and the target."""
        go = self._go()
        df = self.states_to_dataframe()
        u, v, w = (np.asarray(c, dtype=np.float64) for c in arrows)
        k = min(len(df), len(u))  # vtarg rows: one per step; state rows: one more (the IC)
        x, y, z = (df[c].to_numpy(dtype=np.float64) for c in ("x", "y", "z"))
        traces = [go.Scatter3d(x=x, y=y, z=z, mode="lines", name="trajectory"),
                  go.Cone(x=x[:k], y=y[:k], z=z[:k], u=u[:k], v=v[:k], w=w[:k], sizeref=3, showscale=False)]
        if pad:
            r = float(self.target_r)
            ax = np.linspace(-r, r, 100)
            zz, yy = np.meshgrid(ax, ax)
            disc = (zz * zz + yy * yy < r * r).astype(np.float64)
            traces.append(go.Surface(x=disc, y=yy, z=zz, surfacecolor=disc, showscale=False, name="landing pad"))
        fig = go.Figure(data=traces)
        if target:
            tx, ty, tz = (float(c) for c in self.landing_target)
            fig.add_trace(go.Scatter3d(x=[tx], y=[ty], z=[tz], mode="markers", name="target"))
            fig.update_layout(scene_camera={"up": {"x": 1, "y": 0, "z": 0}, "center": {"x": 0, "y": 0, "z": 0},
                                            "eye": {"x": 0.625, "y": 1.25, "z": 0.0}})
        fig.update_layout(scene_aspectmode="data")
        return fig

    def get_trajectory_plotly(self):
        df = self.states_to_dataframe()
        return self._path_figure((df["vx"], df["vy"], df["vz"]), pad=True)

    def get_vtarg_trajectory(self):
        vt = self.vtarg_to_dataframe()
        return self._path_figure((vt["v_x"], vt["v_y"], vt["v_z"]), target=True)

    def get_attitude_trajectory(self):
        go = self._go()
        df = self.states_to_dataframe()
        return go.Figure(data=[go.Scatter(x=df.index, y=df[c], mode="lines", name=c) for c in ("q0", "q1", "q2", "q3")])

    @property
    def rotation_obj(self):
        from scipy.spatial.transform import Rotation

        return Rotation.from_quat(np.roll(np.float32(self.state[6:10]), -1))


class Rocket(_RocketBase):
    """rocket_env.py:19 ``Rocket`` (3DOF) over the HIP step kernel."""

    metadata = {"render.modes": ["human", "rgb_array"], "render_fps": 10}
    _model = 3

    def __init__(self, IC=None, ICRange=None, timestep=0.1, seed=42, reward_coeff=None, device=None):
        kw = {k: v for k, v in dict(IC=IC, ICRange=ICRange, timestep=timestep, seed=seed,
                                     reward_coeff=reward_coeff).items() if v is not None}
        cfg = config_3dof(**kw)
        self.state_names = list(STATE_NAMES_3DOF)
        self.action_names = list(ACTION_NAMES_3DOF)
        self._init_common(cfg, device)
        e = cfg.extra
        self.x_bound_right = e["x_bound"]
        self.x_bound_left = -self.x_bound_right
        self.y_bound_up = e["z_bound"]
        self.y_bound_down = -30
        self.y = None
        self.action = np.array([0.0, 0.0])
        self.target_r = e["landing_radius"]
        self.waypoint = e["waypoint"]

    def reset(self):
        """rocket_env.py:137-148 (returns a float64 observation, like the reference)"""
        ic = self.init_space.sample()
        self.y = ic
        self.SIM = _SimView(ic, self.timestep, 2)
        self._upload(ic)
        return self._normalize_obs(self.y.astype(np.float32))

    def step(self, normalized_action):
        """rocket_env.py:150-175"""
        a = np.asarray(normalized_action, dtype=np.float32).reshape(2)
        self.action = self._denormalize_action(a)
        _, reward, done, terms, state = self._step_device(a)
        self.y = state
        self.SIM.state = state
        self.SIM.t = round(self.SIM.t + self.timestep, 3)
        self.SIM.times.append(self.SIM.t)
        self.SIM.states.append(state)
        self.SIM.actions.append(self.action)
        rewards_dict = {k: float(terms[j]) for j, k in enumerate(self.cfg.term_names)}
        info = {
            "rewards_dict": rewards_dict,
            "is_done": done,
            "state_history": self.SIM.states,
            "action_history": self.SIM.actions,
            "timesteps": self.SIM.times,
            "bounds_violation": bool(terms[len(self.cfg.term_names)] > 0.5),
        }
        return self._normalize_obs(state.astype(np.float32)), reward, done, info

    def _compute_vtarg(self, state32):
        """rocket_env.py:219-247 (host side, for vtarg_history only; z is the altitude, no +1)."""
        r, v = state32[0:2], state32[3:5]
        v_0 = np.linalg.norm(self.SIM.states[0][3:5])
        if r[1] > self.waypoint:
            r_hat = r - [0, self.waypoint]
            v_hat = v - [0, -2]
            tau = 20
        else:
            r_hat = [0, r[1]]
            v_hat = v - [0, -1]
            tau = 100
        t_go = np.linalg.norm(r_hat) / np.linalg.norm(v_hat)
        return -v_0 * (np.array(r_hat) / max(1e-3, np.linalg.norm(r_hat))) * (1 - np.exp(-t_go / tau))

    def vtarg_to_dataframe(self):
        import pandas as pd

        return pd.DataFrame(self.vtarg_history, columns=["v_x", "v_y"])

    def _denormalize_action(self, action):
        """rocket_env.py:395-406 (no clipping)"""
        gimbal = action[0] * self.max_gimbal
        thrust = (action[1] + 1) / 2.0 * self.max_thrust
        return np.float32([gimbal, thrust])

    def _normalize_obs(self, obs):
        return obs / self.state_normalizer

    def _get_obs(self):
        return self._normalize_obs(self.y)
