"""GPU parity: the HIP step kernel (through the C-ABI) against the reference's own
outputs (golden rows from /root/reference, tests/golden/gen_golden.py) and against
the CPU oracle on larger seeded inputs."""
import numpy as np
import pytest

from gpu_util import TOL_REWARD, TOL_STATE, floored_rel, run_rows

pytestmark = pytest.mark.gpu

ENV6 = None


def _env6():
    from rl_rocket_amd.params import ENV_CONFIG_6DOF
    return ENV_CONFIG_6DOF


def _state_err(model, a, b, norm, circ_theta=False):
    """Per-component floored-relative state error. circ_theta (3DOF): theta compared on the circle,
    so that a value within rounding of the 0 / 2pi wrap point (fp32 vs fp64 wrapping it to opposite
    ends) is not a 2pi error."""
    e = floored_rel(a, b, norm)
    if model == 3 and circ_theta:
        d = np.abs(np.asarray(a, np.float64)[:, 2] - np.asarray(b, np.float64)[:, 2])
        e[:, 2] = np.minimum(d, 2 * np.pi - d) / np.maximum(np.abs(b[:, 2]), norm[2])
    return e


def _check_rows(model, g, out, label, tol_state=TOL_STATE, tol_reward=TOL_REWARD, circ_theta=False):
    ns = 14 if model == 6 else 7
    norm = g["normalizer"][:ns]
    e_state = _state_err(model, out["state_out"], g["state_out"], norm, circ_theta).max(1)
    e_obs = floored_rel(out["obs"], g["obs"], 1.0).max(1)
    e_rew = floored_rel(out["reward"], g["reward"], 1.0)
    e_terms = floored_rel(out["terms"], g["terms"], 1.0).max(1)
    done_eq = out["done"] == g["done"]
    bv_eq = out["bounds_violation"] == g["bounds_violation"]
    ev_eq = out["event"] == (g["status"] == 1)
    msg = "%s: max state %.3g obs %.3g reward %.3g terms %.3g; done mismatches %d, bv %d, event %d" % (
        label, e_state.max(), e_obs.max(), e_rew.max(), e_terms.max(), (~done_eq).sum(), (~bv_eq).sum(),
        (~ev_eq).sum())
    print(msg)
    e_comp = _state_err(model, out["state_out"], g["state_out"], norm, circ_theta)
    worst = np.argmax(e_comp, axis=0)
    print("  per-component max:", " ".join("%d:%.2g(row %d g%d)" % (j, e_comp[worst[j], j], worst[j],
                                                                     g["group"][worst[j]]) for j in range(ns)))
    if model == 3 and circ_theta:  # obs[2] = theta / 2pi: the same circle, period 1
        d = np.abs(out["obs"][:, 2].astype(np.float64) - g["obs"][:, 2])
        e_obs = np.maximum(floored_rel(np.delete(out["obs"], 2, 1), np.delete(g["obs"], 2, 1), 1.0).max(1),
                           np.minimum(d, 1.0 - d))
    bad = np.where((e_state > tol_state) | (e_obs > tol_state) | (e_rew > tol_reward) | (e_terms > tol_reward)
                   | ~done_eq | ~bv_eq | ~ev_eq)[0]
    for i in bad[:10]:
        print("  row", i, "group", g["group"][i], "state_err", e_state[i], "rew", out["reward"][i], g["reward"][i],
              "done", out["done"][i], g["done"][i], "terms", out["terms"][i], g["terms"][i])
    assert len(bad) == 0, msg


def test_golden6_single_step(golden6):
    out = run_rows(6, golden6, **_env6())
    _check_rows(6, golden6, out, "6DOF golden")


def test_golden3_single_step(golden3):
    out = run_rows(3, golden3)
    _check_rows(3, golden3, out, "3DOF golden")


@pytest.mark.parametrize("model", [6, 3])
def test_golden_trajectories(model, golden6, golden3):
    """G7: 50-step fixed-action trajectories chained on the GPU (fp32 state carried
    across steps) stay within the north star's 1e-5 floored-relative of the fp64 reference's
    own trajectory at every step."""
    import torch
    from rl_rocket_amd.batch import RocketBatch

    g = golden6 if model == 6 else golden3
    kw = _env6() if model == 6 else {}
    ns = 14 if model == 6 else 7
    traj = g["traj_states"]  # [k, 51, ns]
    k = traj.shape[0]
    b = RocketBatch(k, model=model, device="cuda:0", auto_reset=False, episode_stats=False, **kw)
    ic = g["traj_ic"].astype(np.float32)
    v0 = np.sqrt((ic[:, 3:6 if model == 6 else 5] ** 2).sum(1, dtype=np.float32)).astype(np.float32)
    b.set_state(torch.from_numpy(traj[:, 0, :].astype(np.float32).T.copy()), v0=torch.from_numpy(v0))
    act = torch.from_numpy(g["traj_actions"].astype(np.float32)).cuda()
    worst = 0.0
    alive = np.ones(k, bool)
    for t in range(1, traj.shape[1]):
        _, _, done, _ = b.step(act)
        st = b.get_state()[0].cpu().numpy().T
        ref = traj[:, t, :]
        ok = alive & ~np.isnan(ref).any(1)
        if ok.any():
            e = floored_rel(st[ok], ref[ok], g["normalizer"][:ns]).max()
            worst = max(worst, e)
        alive &= ~done.cpu().numpy().astype(bool)
    b.close()
    print("model", model, "50-step drift", worst)
    assert worst < TOL_STATE  # the north star's 1e-5 after 50 chained fp32 steps (measured 2.4e-6)


def _random_states6(n, seed=0):
    """Seeded 6DOF states spanning the descent envelope (incl. near-ground rows)."""
    rng = np.random.default_rng(seed)
    s = np.zeros((n, 14))
    s[:, 0] = np.where(rng.random(n) < 0.1, rng.uniform(0.01, 5, n), rng.uniform(5, 560, n))
    s[:, 1:3] = rng.uniform(-140, 140, (n, 2))
    s[:, 3] = rng.uniform(-80, 20, n)
    s[:, 4:6] = rng.uniform(-20, 20, (n, 2))
    q = rng.normal(size=(n, 4))
    q[:, 0] += 3.0
    s[:, 6:10] = q / np.linalg.norm(q, axis=1, keepdims=True)
    s[:, 10:13] = rng.uniform(-0.5, 0.5, (n, 3))
    s[:, 13] = rng.uniform(30e3, 46e3, n)
    ic = np.tile(np.float32([500, 100, 100, -50, 0, 0, 1, 0, 0, 0, 0, 0, 0, 45e3]), (n, 1))
    ic[:, 3:6] = rng.uniform(-55, 5, (n, 3)).astype(np.float32)
    a = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    return ic, s.astype(np.float32).astype(np.float64), a


def _quat_from_zyx(a, b, c):
    """q = (w, x, y, z) whose rotation gives the env's zyx angles a = atan2(-R01, R00),
    b = asin(R02), c = atan2(-R12, R22) (rocket_env.py:852-855): q = qx(c) qy(b) qz(a)."""
    def qa(axis, t):
        q = np.zeros((len(t), 4))
        q[:, 0] = np.cos(t / 2)
        q[:, 1 + axis] = np.sin(t / 2)
        return q

    def mul(p, q):
        w1, x1, y1, z1 = p.T
        w2, x2, y2, z2 = q.T
        return np.stack([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                         w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2], axis=1)
    return mul(mul(qa(0, c), qa(1, b)), qa(2, a))


def _zyx_of(q):
    w, x, y, z = (q / np.linalg.norm(q, axis=1, keepdims=True)).T
    a = np.arctan2(-2 * (x * y - z * w), w * w + x * x - y * y - z * z)
    b = np.arcsin(np.clip(2 * (x * z + y * w), -1, 1))
    c = np.arctan2(-2 * (y * z - x * w), w * w - x * x - y * y + z * z)
    return np.stack([a, b, c], axis=1)


def _near_limit_rows6(n, seed, lo, hi, limit=1.5):
    """6DOF rows whose attitude sits just inside or just outside the attitude limit on axis 0
    (atan2) or axis 1 (asin): angle = +-(limit + d), |d| = 10^U(lo, hi) of either sign; omega = 0 and
    zero gimbal, so the step leaves the attitude as it is (up to renormalisation). Returns (ic,
    state, action, axis, d)."""
    rng = np.random.default_rng(seed)
    axis = rng.integers(0, 2, n)
    d = rng.choice([-1.0, 1.0], n) * 10.0 ** rng.uniform(lo, hi, n)
    ang = rng.choice([-1.0, 1.0], n) * (limit + d)
    a = np.where(axis == 0, ang, rng.uniform(-0.5, 0.5, n))
    b = np.where(axis == 1, ang, rng.uniform(-0.5, 0.5, n))
    c = rng.uniform(-3.0, 3.0, n)
    s = np.zeros((n, 14))
    s[:, 0] = rng.uniform(200, 500, n)
    s[:, 1:3] = rng.uniform(-100, 100, (n, 2))
    s[:, 3] = rng.uniform(-60, 0, n)
    s[:, 4:6] = rng.uniform(-10, 10, (n, 2))
    s[:, 6:10] = _quat_from_zyx(a, b, c)
    s[:, 13] = rng.uniform(35e3, 45e3, n)
    ic = np.tile(np.float32([500, 100, 100, -50, 0, 0, 1, 0, 0, 0, 0, 0, 0, 45e3]), (n, 1))
    act = np.zeros((n, 3), np.float32)
    act[:, 2] = rng.uniform(-1, 1, n).astype(np.float32)
    return ic, s, act, axis, d


def test_attitude_tests_at_the_limits_fast(oracle_mod):
    """The fast kernel's attitude tests run without inverse trig (X < r cos L, |sin b| > sin L):
    against the oracle's atan2 / asin on rows 1e-5 .. 1e-3 rad inside and outside the 1.5 rad
    limit of both tested axes (beyond the fp32 attitude's rounding), the penalty term agrees row for
    row and both sides of the limit are present."""
    n = 8192
    ic, s, a, axis, d = _near_limit_rows6(n, 3, -5.0, -3.0)
    s = s.astype(np.float32).astype(np.float64)
    rows = dict(group=np.zeros(n, np.int8), ic=ic, state_in=s, action=a)
    out = run_rows(6, rows, **_env6())
    cfg = oracle_mod.make_cfg(6, **oracle_mod.ENV_CONFIG_6DOF)
    ref = oracle_mod.step(cfg, ic, 0.0, s, a, nthreads=8)
    e = _zyx_of(ref["state_out"][:, 6:10].astype(np.float32).astype(np.float64))  # reward reads the fp32 attitude
    side = np.abs(e[np.arange(n), axis]) > 1.5
    assert np.array_equal(side, d > 0)  # the rows sit where they were put, after the step
    assert 0.3 < side.mean() < 0.7
    att_ref = ref["terms"][:, 3] != 0
    att = out["terms"][:, 3] != 0
    assert np.array_equal(att_ref, side)
    assert np.array_equal(att, att_ref), np.flatnonzero(att != att_ref)[:10]


LAND_LIMIT = (0.2, 0.25, 0.3)  # all below pi / 2: the landing test's any() hinges on each axis


def _env6_land():
    import copy
    from rl_rocket_amd.params import ENV_CONFIG_6DOF
    kw = copy.deepcopy(ENV_CONFIG_6DOF)
    kw["landing_params"]["landing_attitude_limit"] = list(LAND_LIMIT)
    return kw


def _near_limit_landing_rows6(n, seed, lo, hi):
    """6DOF rows that touch down in the step (0.05 m, descending 2 m/s, minimum thrust, omega 0)
    with two zyx angles clearly beyond their landing limits (LAND_LIMIT) and the third, on a random
    axis, at +-(limit + d), |d| = 10^U(lo, hi) of either sign: the landing's attitude test
    (any(|angle| < limit), rocket_env.py:1036-1061) then depends on that axis alone. Returns (ic,
    state, action, axis, d)."""
    rng = np.random.default_rng(seed)
    L = np.array(LAND_LIMIT)
    axis = rng.integers(0, 3, n)
    d = rng.choice([-1.0, 1.0], n) * 10.0 ** rng.uniform(lo, hi, n)
    ang = (L + 0.05 + rng.uniform(0, 0.1, (n, 3))) * rng.choice([-1.0, 1.0], (n, 3))
    ang[np.arange(n), axis] = rng.choice([-1.0, 1.0], n) * (L[axis] + d)
    s = np.zeros((n, 14))
    s[:, 0] = 0.05
    s[:, 1:3] = rng.uniform(-5, 5, (n, 2))
    s[:, 3] = -2.0
    s[:, 4:6] = rng.uniform(-0.5, 0.5, (n, 2))
    s[:, 6:10] = _quat_from_zyx(ang[:, 0], ang[:, 1], ang[:, 2])
    s[:, 13] = 40e3
    ic = np.tile(np.float32([500, 100, 100, -50, 0, 0, 1, 0, 0, 0, 0, 0, 0, 45e3]), (n, 1))
    act = np.zeros((n, 3), np.float32)
    act[:, 2] = -1.0
    return ic, s, act, axis, d


def test_landing_attitude_test_at_the_limits_fast(oracle_mod):
    """The landing's attitude test without inverse trig, at rows 1e-5 .. 1e-3 rad inside and
    outside a landing limit on each of the three axes: every row touches down, and the landing
    bonus (terms[4]) agrees with the oracle's row for row, both sides present."""
    import copy
    n = 8192
    ic, s, a, axis, d = _near_limit_landing_rows6(n, 4, -5.0, -3.0)
    s = s.astype(np.float32).astype(np.float64)
    rows = dict(group=np.zeros(n, np.int8), ic=ic, state_in=s, action=a)
    out = run_rows(6, rows, **_env6_land())
    kw = copy.deepcopy(oracle_mod.ENV_CONFIG_6DOF)
    kw["landing_params"]["landing_attitude_limit"] = list(LAND_LIMIT)
    ref = oracle_mod.step(oracle_mod.make_cfg(6, **kw), ic, 0.0, s, a, nthreads=8)
    assert (ref["status"] == 1).all() and out["event"].all()
    e = _zyx_of(ref["state_out"][:, 6:10].astype(np.float32).astype(np.float64))
    inside = np.abs(e[np.arange(n), axis]) < np.array(LAND_LIMIT)[axis]
    assert np.array_equal(inside, d < 0) and 0.3 < inside.mean() < 0.7
    assert np.array_equal(ref["terms"][:, 4] != 0, inside)
    assert np.array_equal(out["terms"][:, 4] != 0, inside), np.flatnonzero((out["terms"][:, 4] != 0) != inside)[:10]


def test_oracle_parity_6dof_65536(oracle_mod):
    """N = 65536 seeded rows: GPU step vs the CPU oracle (faithful scipy RK45 + event)."""
    n = 65536
    ic, s, a = _random_states6(n, seed=7)
    rows = dict(group=np.zeros(n, np.int8), ic=ic, state_in=s, action=a)
    out = run_rows(6, rows, **_env6())
    cfg = oracle_mod.make_cfg(6, **oracle_mod.ENV_CONFIG_6DOF)
    ref = oracle_mod.step(cfg, ic, 0.0, s, a, nthreads=8)
    ref["event"] = ref["status"] == 1
    g = dict(ref)
    g["group"] = rows["group"]
    g["normalizer"] = np.array(cfg.normalizer[:14])
    _check_rows(6, g, out, "6DOF oracle N=65536")


def _random_states3(n, seed=0):
    """Seeded 3DOF states [x, z, theta, vx, vz, omega, m] spanning the golden rows' envelope: 10 %
    near the ground (z in [0.01, 5] m, descending: ground events), 10 % with theta within 0.03 rad
    of the 0 / 2pi wrap point (omega up to 1 rad/s carries them across it), the bounds faces
    (|x| up to 140 > x_bound 135)."""
    rng = np.random.default_rng(seed)
    s = np.zeros((n, 7))
    s[:, 0] = rng.uniform(-140, 140, n)
    s[:, 1] = np.where(rng.random(n) < 0.1, rng.uniform(0.01, 5, n), rng.uniform(5, 680, n))
    w = rng.random(n)
    s[:, 2] = np.where(w < 0.05, rng.uniform(0, 0.03, n),
                       np.where(w < 0.1, rng.uniform(2 * np.pi - 0.03, 2 * np.pi, n),
                                rng.uniform(np.pi / 2 - 1.2, np.pi / 2 + 1.2, n)))
    s[:, 3] = rng.uniform(-40, 40, n)
    s[:, 4] = rng.uniform(-100, 20, n)
    s[:, 5] = rng.uniform(-1, 1, n)
    s[:, 6] = rng.uniform(30e3, 51e3, n)
    ic = np.tile(np.float32([100, 500, np.pi / 2, -10, -50, 0, 50e3]), (n, 1))
    ic[:, 3] = rng.uniform(-11, -9, n).astype(np.float32)
    ic[:, 4] = rng.uniform(-55, -45, n).astype(np.float32)
    a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
    return ic, s.astype(np.float32).astype(np.float64), a


def _oracle_rows(oracle_mod, model, n, seed, integrator="rk45"):
    ic, s, a = _random_states6(n, seed) if model == 6 else _random_states3(n, seed)
    rows = dict(group=np.zeros(n, np.int8), ic=ic, state_in=s, action=a)
    kw = oracle_mod.ENV_CONFIG_6DOF if model == 6 else oracle_mod.DEFAULTS_3DOF
    cfg = oracle_mod.make_cfg(model, integrator=integrator, **kw)
    ref = oracle_mod.step(cfg, ic, 0.0, s, a, nthreads=8)
    ref["event"] = ref["status"] == 1
    g = dict(ref)
    g["group"] = rows["group"]
    g["normalizer"] = np.array(cfg.normalizer[:14 if model == 6 else 7])
    return rows, g


def test_oracle_parity_3dof_65536(oracle_mod):
    """N = 65536 seeded 3DOF rows (ground events, theta across the 0 / 2pi wrap, bounds faces):
    GPU RK4 step vs the CPU oracle (scipy RK45 + event) within the north star's 1e-5; done,
    bounds and event flags identical on every row."""
    n = 65536
    rows, g = _oracle_rows(oracle_mod, 3, n, seed=11)
    th0, th1 = rows["state_in"][:, 2], g["state_out"][:, 2]
    wrapped = np.abs(th1 - th0) > np.pi
    assert wrapped.sum() > 500 and g["event"].sum() > 1000 and g["bounds_violation"].sum() > 100
    out = run_rows(3, rows)
    _check_rows(3, g, out, "3DOF oracle N=65536", circ_theta=True)


@pytest.mark.parametrize("model,n", [(3, 4096), (6, 4096), (3, 65536 + 17)])
def test_euler_vs_oracle_euler(oracle_mod, model, n):
    """BASELINE configs[1] ("3DOF N=4096 fp32, Euler"): the GPU's RR_INT_EULER step is explicit
    Euler of the reference RHS (simulator.py:88-130 / :259-294) with the event root on Euler's
    line (oracle/rocket_oracle.c euler_step) — within 1e-6 floored-relative of the fp64 oracle on
    state, obs, reward and terms, flags identical, ground events and theta wraps included."""
    rows, g = _oracle_rows(oracle_mod, model, n, seed=23 + model, integrator="euler")
    assert g["event"].sum() > n // 40
    out = run_rows(model, rows, integrator="euler", **(_env6() if model == 6 else {}))
    _check_rows(model, g, out, "%dDOF Euler vs oracle Euler N=%d" % (model, n), tol_state=1e-6, tol_reward=1e-6,
                circ_theta=True)


def test_full_size_properties_6dof():
    """Size-independent properties at the benchmark size N = 524288 with auto-reset:
    determinism, done-list == done mask, reset ICs inside init_space, unit quaternions,
    obs == state / normalizer for non-done envs."""
    import torch
    from rl_rocket_amd.batch import RocketBatch

    n = 524288
    kw = _env6()

    def run(steps):
        b = RocketBatch(n, model=6, device="cuda:0", max_episode_steps=800, **kw)
        b.reset()
        gen = torch.Generator(device="cuda:0")
        gen.manual_seed(123)
        hist = []
        for _ in range(steps):
            a = torch.rand((n, 3), device="cuda:0", generator=gen) * 2 - 1
            obs, rew, done, trunc = b.step(a)
            idx, tobs, ret, ln = b.fetch_done()
            d = done.cpu().numpy().astype(bool)
            assert np.array_equal(np.sort(idx), np.nonzero(d)[0])
            hist.append((obs.clone(), rew.clone(), done.clone()))
        st = b.get_state()[0]
        torch.cuda.synchronize()
        b.close()
        return hist, st

    h1, st1 = run(30)
    h2, st2 = run(30)
    for (o1, r1, d1), (o2, r2, d2) in zip(h1, h2):
        assert torch.equal(o1, o2) and torch.equal(r1, r2) and torch.equal(d1, d2)
    assert torch.equal(st1, st2)
    st = st1.cpu().numpy()
    qn = np.linalg.norm(st[6:10], axis=0)
    assert np.abs(qn - 1).max() < 1e-5
    from rl_rocket_amd.params import config_6dof
    cfg = config_6dof(**kw)
    obs = h1[-1][0].cpu().numpy()
    np.testing.assert_allclose(obs, (st.T / cfg.state_normalizer).astype(np.float32), rtol=2e-6, atol=1e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("model", [6, 3])
@pytest.mark.parametrize("n,auto_reset", [(65536 + 300, True), (4096 + 37, True), (65536 + 300, False)])
def test_helper_wave_launch_is_bitwise_equal(model, n, auto_reset, monkeypatch):
    """At small N the step kernel runs with helper waves that draw the auto-reset candidates
    (step_kernel<..., HELP = true, WPB>, rr_create reads RR_HELP_MAX_N). Outputs, reward
    terms, terminal rows, Monitor returns and state must be bitwise those of the single-role
    kernel, over steps with many resets. Ragged last workgroup; N = 4096 + 37 runs one main
    wave per workgroup (WPB = 1); without auto-reset both launches are the single-role kernel
    (a check of the test itself)."""
    import torch
    from rl_rocket_amd.batch import RocketBatch

    kw = _env6() if model == 6 else {}

    def run(help_max_n):
        monkeypatch.setenv("RR_HELP_MAX_N", str(help_max_n))
        b = RocketBatch(n, model=model, device="cuda:0", max_episode_steps=40, auto_reset=auto_reset,
                        compute_terms=True, **kw)
        b.reset()
        gen = torch.Generator(device="cuda:0")
        gen.manual_seed(7)
        out, resets = [], 0
        for _ in range(60):
            a = torch.rand((n, b.action_dim), device="cuda:0", generator=gen) * 2 - 1
            obs, rew, done, trunc = b.step(a)
            idx, tobs, ret, ln = b.fetch_done()
            resets += len(idx)
            out.append((obs.clone(), rew.clone(), done.clone(), trunc.clone(), b.terms.clone(),
                        torch.as_tensor(tobs).clone(), torch.as_tensor(ret).clone(), torch.as_tensor(ln).clone()))
            if not auto_reset and len(idx):
                b.reset(done)
        st = b.get_state()
        torch.cuda.synchronize()
        b.close()
        return out, st, resets

    h_help, st_help, resets = run(1 << 40)
    h_plain, st_plain, _ = run(0)
    assert resets >= n  # TimeLimit 40 over 60 steps: every env done at least once
    for x, y in zip(h_help, h_plain):
        for u, v in zip(x, y):
            assert torch.equal(u, v)
    for u, v in zip(st_help, st_plain):
        assert torch.equal(torch.as_tensor(u), torch.as_tensor(v))


@pytest.mark.gpu
@pytest.mark.parametrize("model", [6, 3])
@pytest.mark.parametrize("integrator", ["rk4", "dopri5"])
def test_action_soa_layout_is_bitwise_equal(model, integrator, golden6, golden3):
    """RR_FLAG_ACTION_SOA ([action_dim][N] action planes, a template parameter of the step
    kernel) gives bitwise the outputs of the [N][action_dim] row layout."""
    import torch
    from rl_rocket_amd.batch import RocketBatch

    g = golden6 if model == 6 else golden3
    kw = _env6() if model == 6 else {}
    n = len(g["group"])
    ic = g["ic"].astype(np.float32)
    v0 = np.sqrt((ic[:, 3:6 if model == 6 else 5] ** 2).sum(1, dtype=np.float32)).astype(np.float32)
    outs = []
    for soa in (False, True):
        b = RocketBatch(n, model=model, device="cuda:0", max_episode_steps=0, auto_reset=False, episode_stats=False,
                        compute_terms=True, integrator=integrator, action_soa=soa, **kw)
        st = torch.from_numpy(g["state_in"].astype(np.float32).T.copy())
        if integrator == "dopri5":
            b.set_state64(torch.from_numpy(g["state_in"].T.copy()), v0=torch.from_numpy(v0))
        else:
            b.set_state(st, v0=torch.from_numpy(v0))
        a = torch.from_numpy(g["action"].astype(np.float32))
        obs, rew, done, trunc = b.step(a.T.contiguous() if soa else a)
        outs.append([x.clone() for x in (obs, rew, done, b.terms)] + [b.get_state()[0].clone()])
        torch.cuda.synchronize()
        b.close()
    for u, v in zip(*outs):
        assert torch.equal(u, v)


@pytest.mark.gpu
@pytest.mark.parametrize("model", [6, 3])
@pytest.mark.parametrize("n", [1, 2, 63, 65, 255, 257])
def test_small_and_ragged_batches(model, n, golden6, golden3):
    """Batches that fill no wave or leave a ragged last wave / workgroup: every row still
    matches the reference within the north-star tolerance, and the row of env k does not
    depend on which other envs share its wave (bitwise equal to the same row stepped in the
    full golden batch)."""
    g = golden6 if model == 6 else golden3
    kw = _env6() if model == 6 else {}
    N = len(g["group"])
    sel = np.linspace(0, N - 1, n).astype(np.int64)
    rows = {k: v[sel] for k, v in g.items() if getattr(v, "ndim", 0) >= 1 and len(v) == N}
    out = run_rows(model, rows, **kw)
    full = run_rows(model, {k: v for k, v in g.items() if getattr(v, "ndim", 0) >= 1 and len(v) == N}, **kw)
    e = floored_rel(out["state_out"], rows["state_out"], g["normalizer"]).max()
    assert e < TOL_STATE, e
    assert np.array_equal(out["done"], rows["done"])
    for k in ("state_out", "obs", "reward", "terms"):
        assert np.array_equal(out[k], full[k][sel]), k


NEG_ATT = (-0.1, -0.2, 1.0)   # attitude penalty limits below 0: |angle| > limit holds for every row
NEG_LAND = (-0.1, 0.0, 0.3)   # landing limits <= 0 never admit; the landing's any() hinges on axis 2


def _negative_limit_rows(oracle_mod, n, seed):
    """Rows that touch down (_near_limit_landing_rows6), with attitude / landing limits outside the
    angles' range (NEG_ATT, NEG_LAND; rocket_env.py:852-855, 1040-1061 compare |angle| with the
    configured limit, whatever its sign), and the oracle's step of them."""
    import copy
    ic, s, a, axis, d = _near_limit_landing_rows6(n, seed, -3.0, -1.0)
    s = s.astype(np.float32).astype(np.float64)
    kw = copy.deepcopy(oracle_mod.ENV_CONFIG_6DOF)
    kw["trajectory_limits"]["attitude_limit"] = list(NEG_ATT)
    kw["landing_params"]["landing_attitude_limit"] = list(NEG_LAND)
    ref = oracle_mod.step(oracle_mod.make_cfg(6, **kw), ic, 0.0, s, a, nthreads=8)
    assert (ref["terms"][:, 3] != 0).all()  # the penalty on every row
    landed = ref["terms"][:, 4] != 0
    assert 0.05 < landed.mean() < 0.5 and not landed[axis != 2].any()
    return ic, s, a, kw, ref


def test_negative_attitude_limits_fast(oracle_mod):
    """Limits outside the angles' range make the attitude tests constant (make_kparams' thresholds):
    the attitude penalty and the landing bonus agree with the oracle's atan2 / asin row for row."""
    n = 4096
    ic, s, a, kw, ref = _negative_limit_rows(oracle_mod, n, 8)
    out = run_rows(6, dict(group=np.zeros(n, np.int8), ic=ic, state_in=s, action=a), **kw)
    assert np.array_equal(out["terms"][:, 3] != 0, ref["terms"][:, 3] != 0)
    assert np.array_equal(out["terms"][:, 4] != 0, ref["terms"][:, 4] != 0)
