"""The CPU oracle (oracle/rocket_oracle.c, a restatement of the reference step incl.
scipy RK45 + terminal event) against the reference's own outputs.

Primary fixtures: reference run on python3.9 / numpy 1.26 / scipy 1.7.1 (nearest the
reference's pins numpy 1.21.6 / scipy 1.7.3). Cross-stack fixtures: the same inputs
replayed on python3.10 / numpy 2.2 / scipy 1.15.3 (select_initial_step gained a
t_bound clamp after 1.7: oracle flag scipy_clamp_h0)."""
import numpy as np
import pytest

STATE_TOL = 1e-8      # floored-relative; measured <= 4.3e-9 (float32 sin/cos ulp differences)
REWARD_TOL = 1e-7


def _run(oracle_mod, model, g, clamp):
    kw = oracle_mod.ENV_CONFIG_6DOF if model == 6 else oracle_mod.DEFAULTS_3DOF
    cfg = oracle_mod.make_cfg(model, scipy_clamp_h0=clamp, **kw)
    return cfg, oracle_mod.step(cfg, g["ic"], g["t_in"], g["state_in"], g["action"])


@pytest.mark.parametrize("model", [6, 3])
def test_oracle_vs_reference_primary(oracle_mod, model, golden6, golden3):
    g = golden6 if model == 6 else golden3
    cfg, o = _run(oracle_mod, model, g, clamp=False)
    e = oracle_mod.floored_rel(o["state_out"], g["state_out"], g["normalizer"])
    assert e.max() < STATE_TOL, e.max()
    assert np.array_equal(o["status"], g["status"])
    assert np.array_equal(o["nfev"], g["nfev"]), "adaptive step sequence differs from scipy's"
    assert np.array_equal(o["done"], g["done"])
    assert np.array_equal(o["bounds_violation"], g["bounds_violation"])
    assert np.abs(o["reward"] - g["reward"]).max() < REWARD_TOL
    assert np.abs(o["terms"][:, :g["terms"].shape[1]] - g["terms"]).max() < REWARD_TOL
    assert np.abs(o["obs"] - g["obs"]).max() < 1e-7


@pytest.mark.parametrize("model", [6, 3])
def test_oracle_vs_reference_cross_stack(oracle_mod, model, golden6, golden3, golden6_x, golden3_x):
    g = golden6 if model == 6 else golden3
    x = golden6_x if model == 6 else golden3_x
    cfg, o = _run(oracle_mod, model, g, clamp=True)
    e = oracle_mod.floored_rel(o["state_out"], x["state_out"], g["normalizer"])
    assert e.max() < STATE_TOL, e.max()
    assert np.array_equal(o["status"], x["status"])
    assert np.array_equal(o["nfev"], x["nfev"])
    assert np.array_equal(o["done"], x["done"])
    # numpy 2 computes the 3DOF attitude_hint in float32 (NEP 50); the oracle follows the pins
    assert np.abs(o["reward"] - x["reward"]).max() < (1e-7 if model == 6 else 5e-6)


def test_golden_coverage(golden6, golden3):
    """The fixtures exercise every branch the kernel has: ground events, landings,
    attitude violations, bounds faces, theta wrap, multi-attempt RK45 steps."""
    for g in (golden6, golden3):
        assert (g["status"] == 1).sum() > 100
        assert (g["terms"][:, -1] > 0).sum() > 50          # rew_goal = kappa
        assert g["bounds_violation"].sum() > 5
        assert (g["nfev"] > 8).sum() > 100                  # rejected steps
    assert (golden6["terms"][:, 3] != 0).sum() > 50          # attitude constraint
    th = golden3["state_out"][:, 2]
    assert th.min() >= 0 and th.max() < 2 * np.pi


def test_oracle_rhs_matches_reference_formulas(oracle_mod):
    """Spot-check the restated RHS against closed forms (simulator.py:259-294)."""
    cfg = oracle_mod.make_cfg(6, **oracle_mod.ENV_CONFIG_6DOF)
    y = np.zeros(14)
    y[6] = 1.0
    y[13] = 40e3
    u = np.float32([0.0, 0.0, 500e3])
    dy = oracle_mod.rhs(cfg, y, u)
    assert dy[3] == pytest.approx(500e3 / 40e3 - 9.81)
    assert np.all(dy[[4, 5, 10, 11, 12]] == 0)
    assert dy[13] == pytest.approx(-500e3 / (9.81 * 360))


@pytest.mark.parametrize("model", [6, 3])
def test_euler_oracle_is_one_rhs_evaluation(oracle_mod, model, golden6, golden3):
    """RO_INT_EULER (the restatement behind the GPU's RR_INT_EULER, BASELINE configs[1]): on the
    golden inputs, rows without a ground event are y0 + dt f(y0) with f the oracle's reference RHS
    (one evaluation, nfev 1), then renormalised / wrapped; rows with an event end on Euler's line
    with the altitude at 0; status 1 exactly where the altitude changes sign over the step."""
    g = golden6 if model == 6 else golden3
    kw = oracle_mod.ENV_CONFIG_6DOF if model == 6 else oracle_mod.DEFAULTS_3DOF
    cfg = oracle_mod.make_cfg(model, integrator="euler", **kw)
    o = oracle_mod.step(cfg, g["ic"], g["t_in"], g["state_in"], g["action"])
    ev = 0 if model == 6 else 1
    assert (o["nfev"] == 1).all()
    mg, mt = cfg.max_gimbal, cfg.max_thrust
    checked = events = 0
    for i in range(0, len(g["group"]), 7):
        a = g["action"][i].astype(np.float64)
        u = np.float32([a[0] * mg, a[1] * mg, (a[2] + 1) / 2.0 * mt]) if model == 6 else \
            np.float32([a[0] * mg, (a[1] + 1) / 2.0 * mt])
        y0 = g["state_in"][i]
        f0 = oracle_mod.rhs(cfg, y0, u)
        y1 = y0 + cfg.dt * f0
        crosses = (y0[ev] <= 0 <= y1[ev]) or (y0[ev] >= 0 >= y1[ev])
        assert o["status"][i] == (1 if crosses else 0), i
        if crosses and y1[ev] != 0:
            s = y0[ev] / (y0[ev] - y1[ev])
            y1 = y0 + (s * cfg.dt) * f0
            assert abs(y1[ev]) < 1e-9
            events += 1
        if model == 6:
            y1[6:10] /= np.linalg.norm(y1[6:10])
        else:
            y1[2] = np.fmod(np.fmod(y1[2], 2 * np.pi) + 2 * np.pi, 2 * np.pi)
        np.testing.assert_allclose(o["state_out"][i], y1, rtol=1e-13, atol=1e-11)
        checked += 1
    assert checked > 250 and events > 10


@pytest.mark.parametrize("model", [6, 3])
def test_euler_oracle_converges_to_the_reference_step(oracle_mod, model, golden6, golden3):
    """Consistency of the Euler restatement with the reference's RK45 step: over a step of
    dt = 1e-4 the two agree to O(dt^2) (floored-relative < 1e-6 on rows without an event)."""
    g = golden6 if model == 6 else golden3
    kw = dict(oracle_mod.ENV_CONFIG_6DOF if model == 6 else oracle_mod.DEFAULTS_3DOF, timestep=1e-4)
    eu = oracle_mod.step(oracle_mod.make_cfg(model, integrator="euler", **kw), g["ic"], g["t_in"], g["state_in"],
                         g["action"])
    rk = oracle_mod.step(oracle_mod.make_cfg(model, **kw), g["ic"], g["t_in"], g["state_in"], g["action"])
    ok = (eu["status"] == 0) & (rk["status"] == 0)
    assert ok.sum() > 0.8 * len(ok)
    e = oracle_mod.floored_rel(eu["state_out"][ok], rk["state_out"][ok], g["normalizer"])
    assert e.max() < 1e-6, e.max()
