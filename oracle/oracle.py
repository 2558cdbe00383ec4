"""TEST INFRASTRUCTURE ONLY — Python face of the CPU oracle (``librocket_oracle.so``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module; the product package ``rl_rocket_amd`` never does.

What it restates (reference = /root/reference, read-only):
  * ``Rocket6DOF.__init__`` derived constants, rocket_env.py:557-658
  * ``Rocket.__init__`` derived constants,     rocket_env.py:51-123
  * the per-step algorithm itself lives in ``rocket_oracle.c`` (see its header).

Parity of this oracle is pinned by ``tests/test_oracle_golden.py`` against the
reference's own outputs in ``tests/golden/rocket{6,3}dof_ref.npz``.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RO_LIB_PATH") or os.path.join(HERE, "librocket_oracle.so")  # override: sanitizer builds (tools/sanitize.sh)

# configuration_file.py:4-34 of the reference (the benchmark config), restated as data.
ENV_CONFIG_6DOF = {
    "timestep": 0.1,
    "seed": 42,
    "IC": [500, 100, 100, -50, 0, 0, 1, 0, 0, 0, 0, 0, 0, 45e3],
    "ICRange": [50, 10, 10, 10, 10, 10, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 1e3],
    "reward_coeff": {"alfa": -0.01, "beta": -1e-7, "delta": -5, "eta": 0.05, "gamma": -10,
                     "kappa": 10, "xi": 0.004},
    "trajectory_limits": {"attitude_limit": [1.5, 1.5, 2 * np.pi]},
    "landing_params": {"waypoint": 50, "landing_radius": 30, "maximum_velocity": 10,
                       "landing_attitude_limit": [10 / 180 * np.pi, 10 / 180 * np.pi, 2 * np.pi],
                       "omega_lim": [0.2, 0.2, 0.2]},
}

# Rocket.__init__ defaults, rocket_env.py:27-43
DEFAULTS_3DOF = {
    "IC": [100, 500, np.pi / 2, -10, -50, 0, 50e3],
    "ICRange": [10, 50, 0.1, 1, 10, 0.1, 1e3],
    "timestep": 0.1,
    "seed": 42,
    "reward_coeff": {"alfa": -0.01, "beta": -1e-8, "eta": 2, "gamma": -10, "delta": -5,
                     "kappa": 10, "waypoint": 50, "landing_radius": 30},
}

# Rocket6DOF.__init__ defaults, rocket_env.py:511-534
DEFAULTS_6DOF = {
    "IC": [500, 100, 100, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 50e3],
    "ICRange": [50, 10, 10, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 1e3],
    "timestep": 0.1,
    "seed": 42,
    "reward_coeff": {"alfa": -0.01, "beta": -1e-8, "eta": 2, "gamma": -10, "delta": -5,
                     "kappa": 10, "xi": 0.004},
    "trajectory_limits": {"attitude_limit": [1.5, 1.5, 2 * np.pi]},
    "landing_params": {"waypoint": 50, "landing_radius": 30, "maximum_velocity": 10,
                       "landing_attitude_limit": [0.2, 0.2, 2 * np.pi],
                       "omega_lim": [0.2, 0.2, 0.2]},
}


class RoCfg(ctypes.Structure):
    _fields_ = [
        ("model", ctypes.c_int32),
        ("scipy_clamp_h0", ctypes.c_int32),
        ("dt", ctypes.c_double),
        ("normalizer", ctypes.c_double * 14),
        ("bounds_lo", ctypes.c_float * 3),
        ("bounds_hi", ctypes.c_float * 3),
        ("x_bound", ctypes.c_double),
        ("z_bound", ctypes.c_double),
        ("max_gimbal", ctypes.c_double),
        ("max_thrust", ctypes.c_double),
        ("alfa", ctypes.c_double),
        ("beta", ctypes.c_double),
        ("eta", ctypes.c_double),
        ("gamma", ctypes.c_double),
        ("delta", ctypes.c_double),
        ("kappa", ctypes.c_double),
        ("waypoint", ctypes.c_double),
        ("landing_radius", ctypes.c_double),
        ("max_velocity", ctypes.c_double),
        ("att_limit", ctypes.c_double * 3),
        ("land_att_limit", ctypes.c_double * 3),
        ("omega_lim", ctypes.c_double * 3),
        ("integrator", ctypes.c_int32),
    ]


# RoCfg.integrator (rocket_oracle.h): the reference's scipy RK45 step, or the build's explicit-Euler
# speed mode (RR_INT_EULER, BASELINE.json configs[1])
INTEGRATORS = {"rk45": 0, "euler": 1}


def derived6(IC, ICRange, **_):
    """Rocket6DOF.__init__ derived constants (rocket_env.py:557-620), float32 inputs."""
    m = np.float32(IC).astype(np.float64)
    r = np.float32(ICRange).astype(np.float64)
    max_gimbal = np.deg2rad(20)
    max_thrust = 981e3
    t_ff = (-m[3] + np.sqrt(m[3] ** 2 + 2 * 9.81 * m[0])) / 9.81
    omega_max = max_thrust * np.sin(max_gimbal) * 15.0 / 6.04e6 * t_ff / 5.0
    v_max = 2 * 9.81 * t_ff
    norm = np.maximum(np.array([1.2 * abs(m[0]), 1.5 * abs(m[1]), 1.5 * abs(m[2]), v_max, v_max, v_max,
                                1.1, 1.1, 1.1, 1.1, omega_max, omega_max, omega_max, m[13] + r[13]]), 1)
    hi = 0.9 * np.maximum(norm[0:3], 100)
    lo = np.insert(-0.9 * np.maximum(norm[1:3], 100), 0, -30)
    return norm, lo.astype(np.float32), hi.astype(np.float32), max_gimbal, max_thrust


def derived3(IC, ICRange, **_):
    """Rocket.__init__ derived constants (rocket_env.py:66-100), float32 inputs."""
    m = np.float32(IC).astype(np.float64)
    r = np.float32(ICRange).astype(np.float64)
    max_gimbal = np.deg2rad(20)
    max_thrust = 981e3
    t_ff = (-m[4] + np.sqrt(m[4] ** 2 + 2 * 9.81 * m[1])) / 9.81
    norm = np.maximum(np.array([1.5 * abs(m[0]), 1.5 * abs(m[1]), 2 * np.pi, 2 * 9.81 * t_ff, 2 * 9.81 * t_ff,
                                max_thrust * np.sin(max_gimbal) * 30.0 / 6.04e6 * t_ff / 5.0, m[6] + r[6]]), 1)
    xb = 0.9 * np.maximum(norm[0], 100)
    zb = 0.9 * np.maximum(norm[1], 100)
    return norm, xb, zb, max_gimbal, max_thrust


def make_cfg(model, scipy_clamp_h0=False, integrator="rk45", **kw):
    c = RoCfg()
    c.model = model
    c.scipy_clamp_h0 = int(scipy_clamp_h0)
    c.integrator = INTEGRATORS[integrator]
    c.dt = float(kw.get("timestep", 0.1))
    rc = kw["reward_coeff"]
    norm = np.zeros(14)
    if model == 6:
        n, lo, hi, mg, mt = derived6(**kw)
        norm[:14] = n
        for i in range(3):
            c.bounds_lo[i] = float(lo[i])
            c.bounds_hi[i] = float(hi[i])
        lp = kw["landing_params"]
        c.waypoint = lp["waypoint"]
        c.landing_radius = lp["landing_radius"]
        c.max_velocity = lp["maximum_velocity"]
        for i in range(3):
            c.att_limit[i] = kw["trajectory_limits"]["attitude_limit"][i]
            c.land_att_limit[i] = lp["landing_attitude_limit"][i]
            c.omega_lim[i] = 0.2  # hard-coded, rocket_env.py:656
    else:
        n, xb, zb, mg, mt = derived3(**kw)
        norm[:7] = n
        c.x_bound, c.z_bound = float(xb), float(zb)
        c.waypoint = rc["waypoint"]
        c.landing_radius = rc["landing_radius"]
    for i in range(14):
        c.normalizer[i] = norm[i] if norm[i] != 0 else 1.0
    c.max_gimbal, c.max_thrust = float(mg), float(mt)
    for k in ("alfa", "beta", "eta", "gamma", "delta", "kappa"):
        setattr(c, k, float(rc.get(k, 0.0)))
    return c


_LIB = None


def load():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-C", HERE, "-s"])
        lib = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        lib.ro_step_batch.argtypes = [ctypes.POINTER(RoCfg), ctypes.c_int64, P, P, P, P, P, P, P, P, P, P, P, P,
                                      ctypes.c_int]
        lib.ro_step_batch.restype = None
        lib.ro_rhs.argtypes = [ctypes.POINTER(RoCfg), P, P, P]
        lib.ro_rhs.restype = None
        _LIB = lib
    return _LIB


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def step(cfg, ic, t_in, s_in, a, nthreads=1):
    """Batched reference step on injected rows. Shapes: ic [n,ns] f32, t_in [n] f64,
    s_in [n,ns] f64, a [n,na] f32. Returns a dict of numpy arrays."""
    lib = load()
    ns = 14 if cfg.model == 6 else 7
    nt = 5 if cfg.model == 6 else 6
    ic = np.ascontiguousarray(ic, np.float32).reshape(-1, ns)
    n = ic.shape[0]
    t_in = np.ascontiguousarray(np.broadcast_to(np.asarray(t_in, np.float64), (n,)))
    s_in = np.ascontiguousarray(s_in, np.float64).reshape(n, ns)
    a = np.ascontiguousarray(a, np.float32).reshape(n, -1)
    out = dict(state_out=np.empty((n, ns)), obs=np.empty((n, ns), np.float32), reward=np.empty(n),
               terms=np.empty((n, nt)), done=np.empty(n, np.int32), bounds_violation=np.empty(n, np.int32),
               status=np.empty(n, np.int32), nfev=np.empty(n, np.int32))
    lib.ro_step_batch(ctypes.byref(cfg), n, _ptr(ic), _ptr(t_in), _ptr(s_in), _ptr(a), _ptr(out["state_out"]),
                      _ptr(out["obs"]), _ptr(out["reward"]), _ptr(out["terms"]), _ptr(out["done"]),
                      _ptr(out["bounds_violation"]), _ptr(out["status"]), _ptr(out["nfev"]), int(nthreads))
    out["done"] = out["done"].astype(bool)
    out["bounds_violation"] = out["bounds_violation"].astype(bool)
    return out


def rhs(cfg, y, u):
    lib = load()
    ns = 14 if cfg.model == 6 else 7
    y = np.ascontiguousarray(y, np.float64).reshape(ns)
    u = np.ascontiguousarray(u, np.float32)
    dy = np.empty(ns)
    lib.ro_rhs(ctypes.byref(cfg), _ptr(y), _ptr(u), _ptr(dy))
    return dy


def floored_rel(a, b, normalizer):
    """|a-b| / max(|b|, normalizer_c) — SURVEY.md §8 parity metric."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b) / np.maximum(np.abs(b), np.asarray(normalizer, np.float64))
