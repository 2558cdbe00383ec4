"""Generate the golden parity vectors from the REFERENCE's own CPU ``step()``.

Run in the survey container only (``/root/reference`` does not exist on the GPU
box; only the ``.npz`` files this script writes are committed and travel):

    # primary stack: python3.9 + numpy 1.26 (legacy scalar promotion, like the
    # pinned numpy 1.21.6) + scipy 1.7.1 (nearest the pinned scipy 1.7.3)
    PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 tests/golden/gen_golden.py generate
    # cross-check stack: python3.10 + numpy 2.2 (NEP 50) + scipy 1.15.3,
    # replaying the primary inputs
    PYTHONDONTWRITEBYTECODE=1 python3 tests/golden/gen_golden.py replay

How the reference is reached: ``/root/reference`` is put on ``sys.path`` and
``my_environment.envs.rocket_env`` / ``my_environment.utils.simulator`` are
imported as they are.  gym 0.21 (pinned, absent from the image) is replaced by
the restatement in ``tests/golden/_shim/gym`` and the render-only imports
``pyvista`` / ``pygame`` by empty modules; nothing on the ``step()`` path is
replaced.  The reference is executed with bytecode writing disabled.

Row injection: build ``SimulatorXDOF(IC, dt)``, overwrite its
fp64 ``state`` and ``t``, attach it as ``env.SIM`` and call ``env.step(a)``.
``SIM.RHS`` is wrapped to count evaluations and ``SIM.step`` to capture the
``solve_ivp`` status, which ``env.step`` discards.

Row groups:
  G1 random-policy rows from env-config ICs (auto-reset on done)
  G2 ground-event rows (descending states close to the ground)
  G3 crafted landing-success rows (rew_goal = kappa)
  G4 attitude-limit and near-gimbal-lock attitudes
  G5 bounds faces, incl. exact-boundary values
  G6 3DOF analogues (incl. theta near the 0/2pi wrap)
  G7 fixed-action multi-step trajectories
  G8 derived constants, reset IC streams
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(HERE, "_shim"))

import warnings  # noqa: E402

warnings.filterwarnings("ignore")

from scipy.spatial.transform import Rotation  # noqa: E402

from my_environment.envs.rocket_env import Rocket, Rocket6DOF  # noqa: E402
from my_environment.utils.simulator import Simulator3DOF, Simulator6DOF  # noqa: E402
import configuration_file as refcfg  # noqa: E402

TERMS6 = ["velocity_tracking", "thrust_penalty", "eta", "attitude_constraint", "rew_goal"]
TERMS3 = ["velocity_tracking", "thrust_penalty", "eta", "attitude_constraint", "attitude_hint", "rew_goal"]

STACK = "np%s_scipy%s" % (np.__version__, __import__("scipy").__version__)


# ----------------------------------------------------------------------------
# instrumented single step on an injected state
# ----------------------------------------------------------------------------
class _Probe:
    def __init__(self, sim):
        self.nfev = 0
        self.status = None
        rhs, step = sim.RHS, sim.step

        def rhs_counted(t, y, u):
            self.nfev += 1
            return rhs(t, y, u)

        def step_captured(u):
            out = step(u)
            self.status = int(out[1])
            return out

        sim.RHS = rhs_counted
        sim.step = step_captured


def inject_step(env, model, ic, state_in, t_in, action):
    """Run the reference env.step(action) from an injected (ic, state, t)."""
    ic = np.asarray(ic, dtype=np.float32)
    if model == 6:
        sim = Simulator6DOF(ic, env.timestep)
    else:
        sim = Simulator3DOF(ic, env.timestep)
    sim.state = np.array(state_in, dtype=np.float64)
    sim.t = float(t_in)
    env.SIM = sim
    env.vtarg_history = []
    if model == 6:
        q = np.float32(state_in[6:10])
        env.rotation_obj = Rotation.from_quat(np.roll(q, -1))
    probe = _Probe(sim)
    obs, reward, done, info = env.step(np.asarray(action, dtype=np.float32))
    return _pack(model, obs, reward, done, info, env.SIM.state, probe)


def _pack(model, obs, reward, done, info, state_out, probe):
    terms = TERMS6 if model == 6 else TERMS3
    rd = info["rewards_dict"]
    return dict(
        state_out=np.array(state_out, dtype=np.float64),
        obs=np.array(obs, dtype=np.float64),
        reward=float(reward),
        terms=np.array([float(rd[k]) for k in terms], dtype=np.float64),
        done=bool(done),
        bounds_violation=bool(info["bounds_violation"]),
        status=int(probe.status),
        nfev=int(probe.nfev),
    )


class Rows:
    def __init__(self):
        self.cols = {k: [] for k in ("group", "ic", "t_in", "state_in", "action")}
        self.out = {}

    def add(self, group, ic, t_in, state_in, action, res):
        self.cols["group"].append(group)
        self.cols["ic"].append(np.asarray(ic, np.float32))
        self.cols["t_in"].append(float(t_in))
        self.cols["state_in"].append(np.asarray(state_in, np.float64))
        self.cols["action"].append(np.asarray(action, np.float32))
        for k, v in res.items():
            self.out.setdefault(k, []).append(v)

    def arrays(self):
        d = {k: np.array(v) for k, v in self.cols.items()}
        d["group"] = d["group"].astype(np.int8)
        for k, v in self.out.items():
            d[k] = np.array(v)
        d["done"] = d["done"].astype(np.bool_)
        d["bounds_violation"] = d["bounds_violation"].astype(np.bool_)
        d["status"] = d["status"].astype(np.int8)
        d["nfev"] = d["nfev"].astype(np.int16)
        d["obs"] = d["obs"].astype(np.float32)
        return d


def _quat_from_euler_zyx(a, b, c):
    q = Rotation.from_euler("zyx", [a, b, c]).as_quat()  # scalar-last
    return np.roll(q, 1)  # scalar-first


# ----------------------------------------------------------------------------
# 6DOF
# ----------------------------------------------------------------------------
def gen6(rows_per_random=2000, seed=1234):
    cfg = refcfg.env_config
    env = Rocket6DOF(**cfg)
    rng = np.random.default_rng(seed)
    rows = Rows()

    # G1 random-policy rows (the env's own reset stream, seed 42 via the ctor)
    env.reset()
    ic = env.initial_condition.copy()
    while len(rows.cols["group"]) < rows_per_random:
        a = rng.uniform(-1, 1, 3).astype(np.float32)
        s_in, t_in = np.array(env.SIM.state, np.float64), env.SIM.t
        probe = _Probe(env.SIM)
        obs, reward, done, info = env.step(a)
        rows.add(1, ic, t_in, s_in, a, _pack(6, obs, reward, done, info, env.SIM.state, probe))
        if done:
            env.reset()
            ic = env.initial_condition.copy()

    base_ic = np.float32(cfg["IC"])

    def upright(n):
        q = np.zeros((n, 4))
        q[:, 0] = 1.0
        return q

    # G2 ground events: descending from 0.2..6 m
    for i in range(200):
        s = np.zeros(14)
        s[0] = rng.uniform(0.05, 6.0)
        s[1:3] = rng.uniform(-40, 40, 2)
        s[3] = rng.uniform(-70, -2)
        s[4:6] = rng.uniform(-5, 5, 2)
        q = _quat_from_euler_zyx(*rng.uniform(-0.3, 0.3, 3))
        s[6:10] = q
        s[10:13] = rng.uniform(-0.3, 0.3, 3)
        s[13] = rng.uniform(30e3, 46e3)
        a = rng.uniform(-1, 1, 3).astype(np.float32)
        t_in = rng.integers(0, 600) / 10
        rows.add(2, base_ic, t_in, s, a, inject_step(env, 6, base_ic, s, t_in, a))
    # G2b: exactly at the ground (x0 == 0 -> event at t0) and ascending from below
    for x0, vx in ((0.0, -5.0), (0.0, 3.0), (-0.5, 8.0), (-2.0, -1.0)):
        s = np.zeros(14)
        s[0], s[3] = x0, vx
        s[6] = 1.0
        s[13] = 40e3
        a = np.float32([0.1, -0.1, 0.2])
        rows.add(2, base_ic, 1.0, s, a, inject_step(env, 6, base_ic, s, 1.0, a))

    # G3 landing success (close to the ground, slow, inside the radius, upright)
    for i in range(120):
        s = np.zeros(14)
        s[0] = rng.uniform(0.01, 0.4)
        s[1:3] = rng.uniform(-20, 20, 2)
        s[3] = rng.uniform(-8, -1.0)
        s[4:6] = rng.uniform(-2, 2, 2)
        s[6:10] = _quat_from_euler_zyx(*rng.uniform(-0.1, 0.1, 3))
        s[10:13] = rng.uniform(-0.15, 0.15, 3)
        s[13] = rng.uniform(30e3, 46e3)
        a = rng.uniform(-1, 1, 3).astype(np.float32)
        t_in = rng.integers(0, 800) / 10
        rows.add(3, base_ic, t_in, s, a, inject_step(env, 6, base_ic, s, t_in, a))

    # G4 attitude limits and gimbal lock
    for i in range(200):
        s = np.zeros(14)
        s[0] = rng.uniform(50, 500)
        s[1:3] = rng.uniform(-100, 100, 2)
        s[3:6] = rng.uniform(-60, 10, 3)
        if i < 60:
            ang = rng.uniform(-np.pi, np.pi, 3)
        elif i < 120:
            ang = rng.uniform(-1.6, 1.6, 3)
            ang[rng.integers(0, 2)] = rng.choice([-1, 1]) * rng.uniform(1.45, 1.55)
        else:  # near pitch = +-pi/2 (gimbal lock of the zyx sequence)
            ang = rng.uniform(-2, 2, 3)
            ang[1] = rng.choice([-1, 1]) * (np.pi / 2 - 10 ** rng.uniform(-7, -2))
        s[6:10] = _quat_from_euler_zyx(*ang) * rng.uniform(0.95, 1.05)  # slightly non-unit too
        s[10:13] = rng.uniform(-1.0, 1.0, 3)
        s[13] = rng.uniform(30e3, 46e3)
        a = rng.uniform(-1, 1, 3).astype(np.float32)
        rows.add(4, base_ic, 3.0, s, a, inject_step(env, 6, base_ic, s, 3.0, a))

    # G5 bounds faces: exact faces with zero lateral motion (y/z stay exact),
    # just outside, and a crossing of the upper x face.
    lo = env.position_bounds_space.low.astype(np.float64)
    hi = env.position_bounds_space.high.astype(np.float64)
    faces = []
    for ax in (1, 2):
        for val in (lo[ax], hi[ax]):
            for eps in (0.0, 1e-3, -1e-3, 0.5, -0.5):
                faces.append((ax, val + eps))
    for (ax, val) in faces:
        s = np.zeros(14)
        s[0] = 300.0
        s[ax] = val
        s[3] = -20.0
        s[6] = 1.0
        s[13] = 40e3
        a = np.float32([0.0, 0.0, 0.4])
        rows.add(5, base_ic, 2.0, s, a, inject_step(env, 6, base_ic, s, 2.0, a))
    for x0 in (539.0, 539.9, 540.5, 541.0):
        s = np.zeros(14)
        s[0] = x0
        s[3] = 10.0
        s[6] = 1.0
        s[13] = 40e3
        a = np.float32([0.0, 0.0, 1.0])
        rows.add(5, base_ic, 2.0, s, a, inject_step(env, 6, base_ic, s, 2.0, a))
    # (a NaN state is out of contract: the reference raises ValueError inside
    #  Rotation.from_quat during the RK stages, simulator.py:346)

    # G8 derived constants + reset stream
    resets = []
    env2 = Rocket6DOF(**cfg)
    for _ in range(32):
        env2.reset()
        resets.append(env2.initial_condition.copy())
    envd = Rocket6DOF()
    resets_default = []
    for _ in range(8):
        envd.reset()
        resets_default.append(envd.initial_condition.copy())

    d = rows.arrays()
    d.update(
        normalizer=np.asarray(env.state_normalizer, np.float64),
        bounds_low=env.position_bounds_space.low,
        bounds_high=env.position_bounds_space.high,
        normalizer_default=np.asarray(envd.state_normalizer, np.float64),
        bounds_low_default=envd.position_bounds_space.low,
        bounds_high_default=envd.position_bounds_space.high,
        resets_seed42=np.array(resets),
        resets_default_seed42=np.array(resets_default),
    )

    # G7: fixed-action trajectories from the first reset IC (50 steps each)
    traj_actions = np.float32([[0, 0, 0.2], [0.3, -0.2, 0.5], [-0.5, 0.5, 1.0], [0.0, 0.0, -1.0]])
    trajs = []
    for a in traj_actions:
        e = Rocket6DOF(**cfg)
        e.reset()
        ic7 = e.initial_condition.copy()
        st = [np.array(e.SIM.state, np.float64)]
        for _ in range(50):
            _, _, done, _ = e.step(a)
            st.append(np.array(e.SIM.state, np.float64))
            if done:
                break
        while len(st) < 51:
            st.append(np.full(14, np.nan))
        trajs.append(np.array(st))
        d.setdefault("traj_ic", []).append(ic7)
    d["traj_ic"] = np.array(d["traj_ic"])
    d["traj_actions"] = traj_actions
    d["traj_states"] = np.array(trajs)
    return d


# ----------------------------------------------------------------------------
# 3DOF
# ----------------------------------------------------------------------------
def gen3(rows_per_random=1500, seed=4321):
    env = Rocket()
    rng = np.random.default_rng(seed)
    rows = Rows()
    env.reset()
    ic = np.array(env.SIM.states[0], np.float32)
    while len(rows.cols["group"]) < rows_per_random:
        a = rng.uniform(-1, 1, 2).astype(np.float32)
        s_in, t_in = np.array(env.SIM.state, np.float64), env.SIM.t
        probe = _Probe(env.SIM)
        obs, reward, done, info = env.step(a)
        rows.add(1, ic, t_in, s_in, a, _pack(3, obs, reward, done, info, env.SIM.state, probe))
        if done:
            env.reset()
            ic = np.array(env.SIM.states[0], np.float32)

    base_ic = np.float32([100, 500, np.pi / 2, -10, -50, 0, 50e3])

    def s3(x, z, th, vx, vz, om, m):
        return np.array([x, z, th, vx, vz, om, m], np.float64)

    # G2 ground events
    for i in range(200):
        s = s3(rng.uniform(-40, 40), rng.uniform(0.05, 6.0), np.pi / 2 + rng.uniform(-0.3, 0.3),
               rng.uniform(-5, 5), rng.uniform(-70, -2), rng.uniform(-0.3, 0.3), rng.uniform(30e3, 50e3))
        a = rng.uniform(-1, 1, 2).astype(np.float32)
        rows.add(2, base_ic, 4.0, s, a, inject_step(env, 3, base_ic, s, 4.0, a))
    for z0, vz in ((0.0, -5.0), (0.0, 3.0), (-0.5, 8.0)):
        s = s3(0, z0, np.pi / 2, 0, vz, 0, 40e3)
        a = np.float32([0.1, 0.2])
        rows.add(2, base_ic, 1.0, s, a, inject_step(env, 3, base_ic, s, 1.0, a))
    # G3 landing success
    for i in range(120):
        s = s3(rng.uniform(-20, 20), rng.uniform(0.01, 0.4), np.pi / 2 + rng.uniform(-0.1, 0.1),
               rng.uniform(-2, 2), rng.uniform(-10, -1), rng.uniform(-0.15, 0.15), rng.uniform(30e3, 50e3))
        a = rng.uniform(-1, 1, 2).astype(np.float32)
        rows.add(3, base_ic, 2.0, s, a, inject_step(env, 3, base_ic, s, 2.0, a))
    # G6 theta near the 0 / 2pi wrap, attitude hint, large theta
    for i in range(200):
        if i < 100:
            th = rng.choice([0.0, 2 * np.pi]) + rng.uniform(-0.05, 0.05)
        else:
            th = rng.uniform(-7, 14)
        s = s3(rng.uniform(-100, 100), rng.uniform(50, 600), th, rng.uniform(-20, 20),
               rng.uniform(-60, 10), rng.uniform(-1, 1), rng.uniform(30e3, 50e3))
        a = rng.uniform(-1, 1, 2).astype(np.float32)
        rows.add(6, base_ic, 2.0, s, a, inject_step(env, 3, base_ic, s, 2.0, a))
    # G5 bounds
    xb, zb = env.x_bound_right, env.y_bound_up
    for x0 in (xb - 0.5, xb + 0.5, -xb + 0.5, -xb - 0.5, xb, -xb):
        s = s3(x0, 300, np.pi / 2, 0, -10, 0, 40e3)
        a = np.float32([0.0, 0.0])
        rows.add(5, base_ic, 2.0, s, a, inject_step(env, 3, base_ic, s, 2.0, a))
    for z0 in (zb - 0.5, zb + 0.5, zb - 3.0):
        s = s3(0, z0, np.pi / 2, 0, 20, 0, 40e3)
        a = np.float32([0.0, 1.0])
        rows.add(5, base_ic, 2.0, s, a, inject_step(env, 3, base_ic, s, 2.0, a))

    d = rows.arrays()
    resets = []
    e2 = Rocket()
    for _ in range(32):
        e2.reset()
        resets.append(np.array(e2.SIM.states[0], np.float32))
    d.update(
        normalizer=np.asarray(env.state_normalizer, np.float64),
        x_bound=np.float64(env.x_bound_right),
        z_bound=np.float64(env.y_bound_up),
        resets_seed42=np.array(resets),
    )
    traj_actions = np.float32([[0, 0.0], [0.3, 0.5], [-0.5, 1.0], [0.0, -1.0]])
    trajs, tics = [], []
    for a in traj_actions:
        e = Rocket()
        e.reset()
        tics.append(np.array(e.SIM.states[0], np.float32))
        st = [np.array(e.SIM.state, np.float64)]
        for _ in range(50):
            _, _, done, _ = e.step(a)
            st.append(np.array(e.SIM.state, np.float64))
            if done:
                break
        while len(st) < 51:
            st.append(np.full(7, np.nan))
        trajs.append(np.array(st))
    d["traj_ic"] = np.array(tics)
    d["traj_actions"] = traj_actions
    d["traj_states"] = np.array(trajs)
    return d


# ----------------------------------------------------------------------------
def replay(src, model):
    """Re-run the primary inputs on this interpreter's numpy/scipy stack."""
    d = dict(np.load(src))
    env = Rocket6DOF(**refcfg.env_config) if model == 6 else Rocket()
    out = {}
    for i in range(len(d["group"])):
        r = inject_step(env, model, d["ic"][i], d["state_in"][i], d["t_in"][i], d["action"][i])
        for k, v in r.items():
            out.setdefault(k, []).append(v)
    res = {k: np.array(v) for k, v in out.items()}
    res["obs"] = res["obs"].astype(np.float32)
    return res


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "generate"
    if mode == "generate":
        d6 = gen6()
        d6["stack"] = np.array(STACK)
        np.savez_compressed(os.path.join(HERE, "rocket6dof_ref.npz"), **d6)
        d3 = gen3()
        d3["stack"] = np.array(STACK)
        np.savez_compressed(os.path.join(HERE, "rocket3dof_ref.npz"), **d3)
        print("wrote", len(d6["group"]), "6DOF rows and", len(d3["group"]), "3DOF rows with", STACK)
    elif mode == "replay":
        for model, name in ((6, "rocket6dof"), (3, "rocket3dof")):
            r = replay(os.path.join(HERE, name + "_ref.npz"), model)
            r["stack"] = np.array(STACK)
            np.savez_compressed(os.path.join(HERE, name + "_ref_xstack.npz"), **r)
            print("replayed", name, "with", STACK)
    else:
        raise SystemExit("usage: gen_golden.py [generate|replay]")


if __name__ == "__main__":
    main()
