"""TEST / BENCHMARK INFRASTRUCTURE ONLY — a single-env NumPy/SciPy restatement of the reference
step, written for this repo (not copied): the shape of the reference's own ``Rocket6DOF.step`` /
``Rocket.step`` — one env, a Python RHS called by ``scipy.integrate.solve_ivp`` (RK45, its
default rtol 1e-3 / atol 1e-6, a terminal ground event), then the reward, done and obs in
NumPy. Only ``tests/`` and ``bench.py``'s ``cpu_baseline`` leg use it: it is the node's own
timing of the reference algorithm in Python on one core, since the
reference itself cannot travel to the GPU box. Pinned to the reference's rows
(``tests/test_py_step.py``: <= 1e-8 floored-relative on the state against the fixtures the
reference produced on the same numpy 2.2 / scipy 1.15 stack, ``tests/golden/*_xstack.npz``).

What it restates (reference = /root/reference, read-only):
  * Simulator6DOF.step / RHS            simulator.py:227-294 (+ helpers :297-378)
  * Simulator3DOF.step / RHS / wrap     simulator.py:55-130, :150-163
  * Rocket6DOF.step post-processing     rocket_env.py:690-719, 825-859, 963-1061
  * Rocket.step post-processing         rocket_env.py:150-247, 395-476
The float32 points of the reference (float32 denormalised action, float32 cos/sin of the
gimbal and their products, the float32 state the reward reads) are kept; under numpy 2 the
6DOF mass rate is a float32 division (simulator.py:291-292).
"""
import math

import numpy as np
from scipy.integrate import solve_ivp

from . import oracle as O

G0 = 9.81
ISP = 360.0
J6 = np.array([75350.25, 6037675.13, 6037675.13])
JINV6 = 1.0 / J6
RT6 = np.array([-15.0, 0.0, 0.0])
I3, SREF3, CD3, RHO3 = 6.04e6, 10.5, 0.3, 1.225
XCG3, XCP3, XT3 = 10.0, 20.0, 40.0


def _dcm(q):
    """Rotation matrix of the scalar-first quaternion q, normalised first (scipy's from_quat)."""
    w, x, y, z = q / math.sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3])
    return np.array([[w * w + x * x - y * y - z * z, 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), w * w - x * x + y * y - z * z, 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), w * w - x * x - y * y + z * z]])


class PyEnv:
    """One env of `model` (6 or 3) with the config `kw` (oracle.ENV_CONFIG_6DOF / DEFAULTS_3DOF
    layout): step(ic, t, state, action) -> dict, the reference's step on an injected state."""

    def __init__(self, model, **kw):
        self.model = model
        self.cfg = O.make_cfg(model, **kw)
        c = self.cfg
        self.ns = 14 if model == 6 else 7
        self.norm = np.array(c.normalizer[:self.ns])
        self.dt = c.dt
        self.rc = {k: getattr(c, k) for k in ("alfa", "beta", "eta", "gamma", "delta", "kappa")}
        if model == 6:
            self.lo = np.array(c.bounds_lo[:], np.float32)
            self.hi = np.array(c.bounds_hi[:], np.float32)
            self.att_limit = np.array(c.att_limit[:])
            self.land_att = np.array(c.land_att_limit[:])

    # -- action and controls ------------------------------------------------------------------
    def _denorm(self, a):
        c = self.cfg
        a = a.astype(np.float64)
        if self.model == 6:
            return np.float32([a[0] * c.max_gimbal, a[1] * c.max_gimbal, (a[2] + 1) / 2 * c.max_thrust])
        return np.float32([a[0] * c.max_gimbal, (a[1] + 1) / 2 * c.max_thrust])

    def _rhs6(self, u):
        dy_, dz_, T = u
        cy, sy, cz, sz = np.cos(dy_), np.sin(dy_), np.cos(dz_), np.sin(dz_)  # float32
        tb = np.array([cy * cz, sy * cz, sz], np.float32).astype(np.float64) * np.float64(T)
        tau = np.cross(RT6, tb)
        dm = float(-T / np.float32(G0 * ISP))  # float32 under numpy 2

        def f(t, y):
            q = y[6:10]
            w = y[10:13]
            a = (1.0 / y[13]) * (_dcm(q) @ tb)
            a[0] -= G0
            w1, w2, w3 = w
            dq = 0.5 * np.array([-w1 * q[1] - w2 * q[2] - w3 * q[3], w1 * q[0] + w3 * q[2] - w2 * q[3],
                                 w2 * q[0] - w3 * q[1] + w1 * q[3], w3 * q[0] + w2 * q[1] - w1 * q[2]])
            dw = JINV6 * (tau - np.cross(w, J6 * w))
            return np.concatenate([y[3:6], a, dq, dw, [dm]])
        return f

    def _rhs3(self, u):
        d, T = float(u[0]), float(u[1])
        # numpy 2 (NEP 50): T * sin(delta) * (x_T - x_CG) stays float32 (the Python float is weak),
        # the mass rate -T / (Isp g0) too
        tsd = np.float32(u[1]) * np.sin(np.float32(u[0])) * np.float32(XT3 - XCG3)
        dom = (0.0 * (XCG3 - XCP3) - float(tsd)) / I3
        dm = float(-np.float32(u[1]) / np.float32(ISP * G0))

        def f(t, y):
            phi, vx, vz = y[2], y[3], y[4]
            A = CD3 * (0.5 * RHO3 * (vx * vx + vz * vz)) * SREF3
            return np.array([vx, vz, y[5], (T * math.cos(d + phi) - A * math.cos(phi)) / y[6],
                             (T * math.sin(d + phi) - A * math.cos(phi)) / y[6] - G0, dom, dm])
        return f

    # -- one step -------------------------------------------------------------------------------
    def step(self, ic, t, state, action):
        u = self._denorm(np.asarray(action, np.float32))
        ev_idx = 0 if self.model == 6 else 1

        def event(t_, y):
            return y[ev_idx]
        event.terminal = True
        f = self._rhs6(u) if self.model == 6 else self._rhs3(u)
        sol = solve_ivp(f, [t, t + self.dt], np.asarray(state, np.float64), events=event)
        y = sol.y[:, -1].copy()
        if self.model == 6:
            y[6:10] /= np.linalg.norm(y[6:10])
            out = self._finish6(np.asarray(ic, np.float32), u, sol.status, y)
        else:
            y[2] = math.fmod(math.fmod(y[2], 2 * math.pi) + 2 * math.pi, 2 * math.pi)
            out = self._finish3(np.asarray(ic, np.float32), u, sol.status, y)
        out.update(state_out=y, status=sol.status, t_out=round(t + self.dt, 3))
        return out

    def _finish6(self, ic, u, status, y):
        s = y.astype(np.float32)
        r = s[0:3]
        bv = not bool(np.all((r >= self.lo) & (r <= self.hi)))  # Box.contains, NaN outside
        v0 = float(np.linalg.norm(ic[3:6]))
        if s[0] > 50.0:
            rh = np.array([s[0] - 50.0, s[1], s[2]], np.float64)
            vh = np.array([s[3] + 2.0, s[4], s[5]], np.float64)
            tau = 20.0
        else:
            rh = np.array([s[0] + 1.0, 0.0, 0.0])
            vh = np.array([s[3] + 1.0, s[4], s[5]], np.float64)
            tau = 100.0
        nrh = np.linalg.norm(rh)
        vt = -v0 * rh / max(1e-3, nrh) * (1 - math.exp(-(nrh / np.linalg.norm(vh)) / tau))
        rc = self.rc
        vel = rc["alfa"] * np.linalg.norm(s[3:6] - vt)
        thr = rc["beta"] * float(u[2])
        R = _dcm(s[6:10].astype(np.float64))
        e = np.array([math.atan2(-R[0, 1], R[0, 0]), math.asin(min(1.0, max(-1.0, R[0, 2]))),
                      math.atan2(-R[1, 2], R[2, 2])])
        att = rc["gamma"] * float(np.any(np.abs(e) > self.att_limit))
        landing = (s[0] <= 1e-3 and np.linalg.norm(s[3:6]) < self.cfg.max_velocity and
                   np.linalg.norm(s[0:3]) < self.cfg.landing_radius and np.any(np.abs(e) < self.land_att) and
                   np.any(np.abs(s[10:13]) < 0.2))
        goal = rc["kappa"] * float(landing)
        terms = np.array([vel, thr, rc["eta"], att, goal])
        return dict(obs=(y / self.norm).astype(np.float32), reward=float(terms.sum()) + (-50.0 if bv else 0.0),
                    terms=terms, done=bool(status) or bv, bounds_violation=bv)

    def _finish3(self, ic, u, status, y):
        s = y.astype(np.float32)
        c = self.cfg
        bv = bool(s[0] <= -c.x_bound or s[0] >= c.x_bound or s[1] >= c.z_bound)
        v0 = float(np.linalg.norm(ic[3:5]))
        if s[1] > c.waypoint:
            rh = np.array([s[0], s[1] - c.waypoint], np.float64)
            vh = np.array([s[3], s[4] + 2.0], np.float64)
            tau = 20.0
        else:
            rh = np.array([0.0, s[1]], np.float64)
            vh = np.array([s[3], s[4] + 1.0], np.float64)
            tau = 100.0
        nrh = np.linalg.norm(rh)
        vt = -v0 * rh / max(1e-3, nrh) * (1 - math.exp(-(nrh / np.linalg.norm(vh)) / tau))
        rc = self.rc
        vel = rc["alfa"] * np.linalg.norm(s[3:5] - vt)
        thr = rc["beta"] * float(u[1])
        zeta = float(s[2]) - math.pi / 2
        att = rc["gamma"] * float(abs(zeta) > 2 * math.pi)
        hint = rc["delta"] * max(0.0, abs(zeta) - math.pi / 2)
        landing = (s[1] <= 1e-3 and np.linalg.norm(s[3:5]) < 15 and np.linalg.norm(s[0:2]) < c.landing_radius
                   and abs(zeta) < 0.2 and abs(s[5]) < 0.2)
        goal = rc["kappa"] * float(landing)
        terms = np.array([vel, thr, rc["eta"], att, hint, goal])
        return dict(obs=(s.astype(np.float64) / self.norm).astype(np.float32),
                    reward=float(terms.sum()) + (-50.0 if bv else 0.0), terms=terms, done=bool(status) or bv,
                    bounds_violation=bv)


def run_episodes(model, seconds, seed=0, max_episode_steps=800):
    """The CPU baseline leg: ONE env stepped by this restatement from a Python loop for about
    `seconds` (env_config / ctor-default ICs, U(-1,1) actions, reset on done or at the TimeLimit).
    Returns (env-steps, busy seconds)."""
    import time

    kw = O.ENV_CONFIG_6DOF if model == 6 else O.DEFAULTS_3DOF
    env = PyEnv(model, **kw)
    ns, na = (14, 3) if model == 6 else (7, 2)
    lo = np.float32(kw["IC"]) - np.float32(kw["ICRange"]) / 2
    hi = np.float32(kw["IC"]) + np.float32(kw["ICRange"]) / 2
    rng = np.random.default_rng(seed)

    def sample():
        ic = rng.uniform(lo, hi).astype(np.float32)
        if model == 6:
            ic[6:10] /= np.linalg.norm(ic[6:10])
        return ic

    ic = sample()
    s, t, el, steps = ic.astype(np.float64), 0.0, 0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        o = env.step(ic, t, s, rng.uniform(-1, 1, na).astype(np.float32))
        s, t, el, steps = o["state_out"], o["t_out"], el + 1, steps + 1
        if o["done"] or el >= max_episode_steps:
            ic = sample()
            s, t, el = ic.astype(np.float64), 0.0, 0
    return steps, time.perf_counter() - t0
