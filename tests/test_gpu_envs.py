"""GPU: the gym / SB3 surfaces over the HIP kernel (single-env shims and RocketVecEnv)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_rocket6dof_shim_reset_and_step(golden6, oracle_mod):
    from rl_rocket_amd.envs import Rocket6DOF
    from rl_rocket_amd.params import ENV_CONFIG_6DOF

    env = Rocket6DOF(**ENV_CONFIG_6DOF)
    obs = env.reset()
    # the reference's own reset stream (gym 0.21 seeding, seed 42)
    np.testing.assert_array_equal(env.initial_condition, golden6["resets_seed42"][0])
    assert obs.dtype == np.float32 and obs.shape == (14,)
    np.testing.assert_array_equal(obs, (golden6["resets_seed42"][0] / env.state_normalizer).astype(np.float32))
    a = np.float32([0.2, -0.1, 0.5])
    obs, reward, done, info = env.step(a)
    assert isinstance(reward, float) and isinstance(done, bool)
    assert set(info) == {"rewards_dict", "is_done", "state_history", "action_history", "timesteps",
                         "bounds_violation"}
    assert set(info["rewards_dict"]) == {"velocity_tracking", "thrust_penalty", "eta", "attitude_constraint",
                                         "rew_goal"}
    cfg = oracle_mod.make_cfg(6, **oracle_mod.ENV_CONFIG_6DOF)
    ic = golden6["resets_seed42"][0]
    ref = oracle_mod.step(cfg, ic[None], 0.0, ic[None].astype(np.float64), a[None])
    e = oracle_mod.floored_rel(env.state, ref["state_out"][0], cfg.normalizer[:14]).max()
    assert e < 1e-5
    assert abs(reward - ref["reward"][0]) < 1e-5 * max(1, abs(ref["reward"][0]))
    assert len(env.SIM.states) == 2 and env.SIM.times == [0, 0.1]
    assert env.states_to_dataframe().shape == (2, 14)
    assert env.vtarg_to_dataframe().shape == (1, 3)
    for _ in range(200):
        obs, reward, done, info = env.step(np.float32([0, 0, -1]))  # free fall -> ground event
        if done:
            break
    assert done and abs(env.state[0]) < 1e-3
    env.close()


def test_rocket3dof_shim(golden3):
    from rl_rocket_amd.envs import Rocket

    env = Rocket()
    obs = env.reset()
    assert obs.dtype == np.float64 and obs.shape == (7,)  # the reference's 3DOF obs is float64
    np.testing.assert_array_equal(env.SIM.states[0], golden3["resets_seed42"][0])
    obs, reward, done, info = env.step(np.float32([0.1, 0.3]))
    assert "attitude_hint" in info["rewards_dict"]
    env.close()


def test_vec_env_sb3_semantics():
    from rl_rocket_amd.params import ENV_CONFIG_6DOF
    from rl_rocket_amd.vec_env import RocketVecEnv

    n = 4096
    env = RocketVecEnv(n, model="6DOF", device="cuda:0", max_episode_steps=5, monitor=True, **ENV_CONFIG_6DOF)
    obs = env.reset()
    assert obs.shape == (n, 14) and obs.dtype == np.float32
    rng = np.random.default_rng(0)
    seen_trunc = False
    for k in range(12):
        obs, rew, done, infos = env.step(rng.uniform(-1, 1, (n, 3)).astype(np.float32))
        assert rew.shape == (n,) and done.dtype == bool and len(infos) == n
        idx = np.nonzero(done)[0]
        assert infos.done_indices() == idx.tolist()
        for i in idx[:50]:
            d = infos[i]
            assert d["terminal_observation"].shape == (14,)
            assert "episode" in d and d["episode"]["l"] <= 5
            if d.get("TimeLimit.truncated"):
                seen_trunc = True
                assert d["episode"]["l"] == 5
        if k == 4:  # every env has either ended before or hits the limit now
            assert done.all() or env.episode_lengths
    assert seen_trunc
    assert np.all(np.abs(obs) < 10)
    env.close()
