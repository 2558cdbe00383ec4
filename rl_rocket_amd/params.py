"""Lower the reference env constructor kwargs to the kernel's POD ``rr_params``.

Restates the derived constants of
  * ``Rocket6DOF.__init__`` — reference my_environment/envs/rocket_env.py:511-663
  * ``Rocket.__init__``     — rocket_env.py:27-135
and keeps the same keyword names, defaults and required keys, so that
``gym.make("my_environment/Falcon6DOF-v0", **env_config)`` style kwargs
(configuration_file.py:4-34) work unchanged.

``rr_params`` carries the reference's float64 values; the fp32 kernels round the
thresholds that the reference compares in float64 against float32 state values to the
float32 value that gives the same answer for every float32 input (``ceil_f``/``floor_f``,
restated in C++ in make_kparams), so they compare in fp32 exactly.
"""
import copy
import math

import numpy as np

from . import _lib

# Rocket6DOF.__init__ defaults, rocket_env.py:511-534
DEFAULTS_6DOF = dict(
    IC=[500, 100, 100, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 50e3],
    ICRange=[50, 10, 10, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 1e3],
    timestep=0.1,
    seed=42,
    reward_coeff={"alfa": -0.01, "beta": -1e-8, "eta": 2, "gamma": -10, "delta": -5, "kappa": 10, "xi": 0.004},
    trajectory_limits={"attitude_limit": [1.5, 1.5, 2 * np.pi]},
    landing_params={"waypoint": 50, "landing_radius": 30, "maximum_velocity": 10,
                    "landing_attitude_limit": [0.2, 0.2, 2 * np.pi], "omega_lim": [0.2, 0.2, 0.2]},
)

# Rocket.__init__ defaults, rocket_env.py:27-43
DEFAULTS_3DOF = dict(
    IC=[100, 500, np.pi / 2, -10, -50, 0, 50e3],
    ICRange=[10, 50, 0.1, 1, 10, 0.1, 1e3],
    timestep=0.1,
    seed=42,
    reward_coeff={"alfa": -0.01, "beta": -1e-8, "eta": 2, "gamma": -10, "delta": -5, "kappa": 10,
                  "waypoint": 50, "landing_radius": 30},
)

# configuration_file.py:4-34 (the benchmark env config of main_6DOF.py)
ENV_CONFIG_6DOF = dict(
    timestep=0.1,
    seed=42,
    IC=[500, 100, 100, -50, 0, 0, 1, 0, 0, 0, 0, 0, 0, 45e3],
    ICRange=[50, 10, 10, 10, 10, 10, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 1e3],
    reward_coeff={"alfa": -0.01, "beta": -1e-7, "delta": -5, "eta": 0.05, "gamma": -10, "kappa": 10, "xi": 0.004},
    trajectory_limits={"attitude_limit": [1.5, 1.5, 2 * np.pi]},
    landing_params={"waypoint": 50, "landing_radius": 30, "maximum_velocity": 10,
                    "landing_attitude_limit": [10 / 180 * np.pi, 10 / 180 * np.pi, 2 * np.pi],
                    "omega_lim": [0.2, 0.2, 0.2]},
)
MAX_EPISODE_STEPS = 800  # configuration_file.py:36-44: int(MAX_TIME / timestep)

STATE_NAMES_6DOF = ["x", "y", "z", "vx", "vy", "vz", "q0", "q1", "q2", "q3", "omega1", "omega2", "omega3", "mass"]
ACTION_NAMES_6DOF = ["gimbal_y", "gimbal_z", "thrust"]
STATE_NAMES_3DOF = ["x", "z", "theta", "vx", "vz", "omega", "mass"]
ACTION_NAMES_3DOF = ["gimbal", "thrust"]
TERM_NAMES_6DOF = ["velocity_tracking", "thrust_penalty", "eta", "attitude_constraint", "rew_goal"]
TERM_NAMES_3DOF = ["velocity_tracking", "thrust_penalty", "eta", "attitude_constraint", "attitude_hint", "rew_goal"]

MAX_GIMBAL = np.deg2rad(20)   # rocket_env.py:572
MAX_THRUST = 981e3            # rocket_env.py:573


def ceil_f(d):
    """Smallest float32 >= d: for float32 x, ``x < d`` <=> ``x < ceil_f(d)`` and ``x >= d`` <=> ``x >= ceil_f(d)``."""
    f = np.float32(d)
    if float(f) < d:
        f = np.nextafter(f, np.float32(np.inf))
    return float(f)


def floor_f(d):
    """Largest float32 <= d: ``x <= d`` <=> ``x <= floor_f(d)``, ``x > d`` <=> ``x > floor_f(d)``."""
    f = np.float32(d)
    if float(f) > d:
        f = np.nextafter(f, np.float32(-np.inf))
    return float(f)


class EnvConfig:
    """Host-side view of one env configuration (what the reference ctor derives)."""

    def __init__(self, model, kwargs, normalizer, ic_low, ic_high, extra):
        self.model = model
        self.kwargs = kwargs
        self.state_normalizer = normalizer      # float64, like the reference
        self.ic_low = ic_low                    # float32 Box bounds
        self.ic_high = ic_high
        self.extra = extra

    @property
    def state_dim(self):
        return 14 if self.model == 6 else 7

    @property
    def action_dim(self):
        return 3 if self.model == 6 else 2

    @property
    def term_names(self):
        return TERM_NAMES_6DOF if self.model == 6 else TERM_NAMES_3DOF


def _merge(defaults, kwargs):
    out = copy.deepcopy(defaults)
    for k, v in kwargs.items():
        if k not in defaults:
            raise TypeError("unexpected keyword argument %r" % k)
        out[k] = v
    return out


def config_6dof(**kwargs):
    """Rocket6DOF.__init__ derived constants (rocket_env.py:557-658)."""
    kw = _merge(DEFAULTS_6DOF, kwargs)
    ic_mean = np.float32(kw["IC"])
    ic_range = np.float32(kw["ICRange"])
    if ic_mean.shape != (14,) or ic_range.shape != (14,):
        raise AssertionError("The observation space has shape (14,) but the init_space has shape %s" % (ic_mean.shape,))
    ic_low = (ic_mean - ic_range / 2).astype(np.float32)
    ic_high = (ic_mean + ic_range / 2).astype(np.float32)
    m = ic_mean.astype(np.float64)
    r = ic_range.astype(np.float64)
    t_ff = (-m[3] + np.sqrt(m[3] ** 2 + 2 * 9.81 * m[0])) / 9.81
    omega_max = MAX_THRUST * np.sin(MAX_GIMBAL) * 15.0 / 6.04e6 * t_ff / 5.0
    v_max = 2 * 9.81 * t_ff
    norm = np.maximum(np.array([1.2 * abs(m[0]), 1.5 * abs(m[1]), 1.5 * abs(m[2]), v_max, v_max, v_max,
                                1.1, 1.1, 1.1, 1.1, omega_max, omega_max, omega_max, m[13] + r[13]]), 1)
    hi = (0.9 * np.maximum(norm[0:3], 100)).astype(np.float32)
    lo = np.insert(-0.9 * np.maximum(norm[1:3], 100), 0, -30).astype(np.float32)
    lp = kw["landing_params"]
    extra = dict(
        bounds_low=lo, bounds_high=hi,
        waypoint=lp["waypoint"], landing_radius=lp["landing_radius"], maximum_velocity=lp["maximum_velocity"],
        attitude_limit=list(kw["trajectory_limits"]["attitude_limit"]),
        landing_attitude_limit=list(lp["landing_attitude_limit"]),
        omega_lim=[0.2, 0.2, 0.2],  # hard-coded, rocket_env.py:656 (landing_params["omega_lim"] is ignored)
    )
    return EnvConfig(6, kw, norm, ic_low, ic_high, extra)


def config_3dof(**kwargs):
    """Rocket.__init__ derived constants (rocket_env.py:51-123)."""
    kw = _merge(DEFAULTS_3DOF, kwargs)
    ic_mean = np.float32(kw["IC"])
    ic_range = np.float32(kw["ICRange"])
    if ic_mean.shape != (7,) or ic_range.shape != (7,):
        raise AssertionError("The observation space has shape (7,) but the init_space has shape %s" % (ic_mean.shape,))
    rc = kw["reward_coeff"]
    for key in ("waypoint", "landing_radius"):
        if key not in rc:
            raise KeyError(key)  # rocket_env.py:122-123
    ic_low = (ic_mean - ic_range / 2).astype(np.float32)
    ic_high = (ic_mean + ic_range / 2).astype(np.float32)
    m = ic_mean.astype(np.float64)
    r = ic_range.astype(np.float64)
    t_ff = (-m[4] + np.sqrt(m[4] ** 2 + 2 * 9.81 * m[1])) / 9.81
    norm = np.maximum(np.array([1.5 * abs(m[0]), 1.5 * abs(m[1]), 2 * np.pi, 2 * 9.81 * t_ff, 2 * 9.81 * t_ff,
                                MAX_THRUST * np.sin(MAX_GIMBAL) * 30.0 / 6.04e6 * t_ff / 5.0, m[6] + r[6]]), 1)
    xb = 0.9 * np.maximum(norm[0], 100)
    zb = 0.9 * np.maximum(norm[1], 100)
    extra = dict(x_bound=float(xb), z_bound=float(zb), waypoint=rc["waypoint"], landing_radius=rc["landing_radius"])
    return EnvConfig(3, kw, norm, ic_low, ic_high, extra)


def make_config(model, **kwargs):
    model = parse_model(model)
    return config_6dof(**kwargs) if model == 6 else config_3dof(**kwargs)


def parse_model(model):
    if model in (6, "6", "6DOF", "6dof", "Falcon6DOF", "my_environment/Falcon6DOF-v0"):
        return 6
    if model in (3, "3", "3DOF", "3dof", "Falcon3DOF", "my_environment/Falcon3DOF-v0"):
        return 3
    raise ValueError("unknown model %r (expected '6DOF' or '3DOF')" % (model,))


INTEGRATORS = {"rk4": _lib.RR_INT_RK4, "euler": _lib.RR_INT_EULER, "dopri5": _lib.RR_INT_DOPRI5}


def lower(cfg, max_episode_steps=0, auto_reset=True, episode_stats=True, reward_annealing=False,
          integrator="rk4", action_soa=False, xi_default=0.01, scipy_h0_clamp=False, host_state=False):
    """EnvConfig -> ctypes rr_params. ``integrator``: "rk4" (fast parity mode), "euler"
    (non-parity speed mode) or "dopri5" (exact mode: fp64 scipy RK45 restatement);
    ``scipy_h0_clamp`` selects scipy >= 1.12's select_initial_step in dopri5 mode."""
    p = _lib.RrParams()
    p.model = cfg.model
    p.integrator = INTEGRATORS[integrator.lower()]
    p.max_episode_steps = int(max_episode_steps or 0)
    flags = 0
    if auto_reset:
        flags |= _lib.RR_FLAG_AUTO_RESET
    if episode_stats:
        flags |= _lib.RR_FLAG_EPISODE_STATS
    if reward_annealing:
        flags |= _lib.RR_FLAG_REWARD_ANNEALING
    if action_soa:
        flags |= _lib.RR_FLAG_ACTION_SOA
    if scipy_h0_clamp:
        flags |= _lib.RR_FLAG_SCIPY_H0_CLAMP
    if host_state:
        flags |= _lib.RR_FLAG_HOST_STATE
    p.flags = flags
    p.dt = float(cfg.kwargs["timestep"])
    ns = cfg.state_dim
    for j in range(_lib.RR_MAX_STATE):
        p.ic_low[j] = float(cfg.ic_low[j]) if j < ns else 0.0
        p.ic_high[j] = float(cfg.ic_high[j]) if j < ns else 0.0
        p.normalizer[j] = float(cfg.state_normalizer[j]) if j < ns else 1.0
    rc = cfg.kwargs["reward_coeff"]
    p.max_gimbal = float(MAX_GIMBAL)
    p.max_thrust = float(MAX_THRUST)
    for k in ("alfa", "beta", "eta", "gamma", "delta", "kappa"):
        setattr(p, k, float(rc.get(k, 0.0)))
    p.xi = float(rc.get("xi", xi_default))  # RewardAnnealing: reward_coefficients.get("xi", 0.01)
    e = cfg.extra
    if cfg.model == 6:
        for j in range(3):
            p.bounds_low[j] = float(e["bounds_low"][j])
            p.bounds_high[j] = float(e["bounds_high"][j])
            p.att_limit[j] = float(e["attitude_limit"][j])
            p.land_att_limit[j] = float(e["landing_attitude_limit"][j])
            p.omega_lim[j] = float(e["omega_lim"][j])
        p.waypoint = float(e["waypoint"])
        p.landing_radius = float(e["landing_radius"])
        p.max_velocity = float(e["maximum_velocity"])
    else:
        # _check_bounds: x <= -xb or x >= xb or z >= zb (rocket_env.py:441-445); the fp32
        # kernels round these with floor_f / ceil_f at rr_create
        p.bounds_low[0] = -float(e["x_bound"])
        p.bounds_high[0] = float(e["x_bound"])
        p.bounds_high[1] = float(e["z_bound"])
        p.waypoint = float(e["waypoint"])
        p.landing_radius = float(e["landing_radius"])
        p.max_velocity = 15.0  # v_lim, rocket_env.py:462
        for j in range(3):
            p.omega_lim[j] = 0.2
            p.att_limit[j] = 2 * math.pi
            p.land_att_limit[j] = 0.2
    return p
