"""oracle/py_step.py (the single-env NumPy/SciPy restatement bench.py times as the node's own
Python-on-one-core baseline) against the reference's own rows. It runs on this image's numpy 2.2 /
scipy 1.15, so it is pinned to the fixtures the reference produced on that same stack
(tests/golden/*_xstack.npz, made by tests/golden/gen_golden.py): state <= 1e-8 floored-relative,
identical solve_ivp status, done and bounds flags, reward within 1e-7 (6DOF) / 5e-6 (3DOF,
float32 terms of the reference)."""
import numpy as np
import pytest


@pytest.mark.parametrize("model", [6, 3])
def test_py_step_vs_reference(model, golden6, golden3, golden6_x, golden3_x):
    from oracle import oracle as O
    from oracle.py_step import PyEnv

    g = golden6 if model == 6 else golden3
    x = golden6_x if model == 6 else golden3_x
    env = PyEnv(model, **(O.ENV_CONFIG_6DOF if model == 6 else O.DEFAULTS_3DOF))
    rows = np.arange(0, len(g["group"]), 3)  # every third row: ~1 s of Python per model
    worst, wr = 0.0, 0.0
    for i in rows:
        o = env.step(g["ic"][i], g["t_in"][i], g["state_in"][i], g["action"][i])
        worst = max(worst, float(O.floored_rel(o["state_out"], x["state_out"][i], g["normalizer"]).max()))
        assert o["status"] == x["status"][i], i
        assert o["done"] == x["done"][i] and o["bounds_violation"] == x["bounds_violation"][i], i
        wr = max(wr, abs(o["reward"] - x["reward"][i]))
        assert np.abs(o["obs"] - x["obs"][i]).max() < 1e-7, i
    print("model", model, "rows", len(rows), "state", worst, "reward", wr)
    assert worst < 1e-8
    assert wr < (1e-7 if model == 6 else 5e-6)


def test_run_episodes_counts_steps():
    from oracle.py_step import run_episodes

    steps, busy = run_episodes(6, 0.3)
    assert steps > 10 and busy >= 0.3
