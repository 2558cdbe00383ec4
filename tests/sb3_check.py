"""Test helper: the assertions of stable-baselines3 1.6 ``common.env_checker.check_env``
restated (SB3 is not installed here). The reference's only API-contract test runs
``check_env(Rocket6DOF(**env_config), skip_render_check=False)``
(test_6DOF_sb_integration.py:15-18); ``check_env`` below applies the same checks, in the
same order, to any object with the gym 0.21 ``Env`` surface:

  _check_spaces           observation_space / action_space exist and are Box spaces
  _check_box_obs / action finite bounds; action Box symmetric, normalised to [-1, 1], float32
  _check_returned_values  reset() -> ndarray obs in observation_space; step(sample) -> 4-tuple
                          (obs in observation_space, float/int reward, bool done, dict info)
  _check_render           every mode in metadata["render.modes"] renders (none declared here)
  _check_nan              10 random steps through a DummyVecEnv-style auto-reset loop with no
                          NaN / inf in obs or rewards (VecCheckNan)

It raises AssertionError with SB3's messages; warnings SB3 would print are returned.
"""
import numpy as np


def _box(space):
    return all(hasattr(space, a) for a in ("low", "high", "shape", "dtype", "contains", "sample"))


def _check_obs(obs, space, method):
    assert not isinstance(obs, tuple), "The observation returned by the `%s()` method should be a single value, " \
                                       "not a tuple" % method
    assert isinstance(obs, np.ndarray), "The observation returned by `%s()` method must be a numpy array" % method
    assert space.contains(obs), "The observation returned by the `%s()` method does not match the given " \
                                "observation space" % method


def check_env(env, skip_render_check=True):
    warns = []
    # _check_spaces
    assert hasattr(env, "observation_space"), "You must specify an observation space (cf gym.spaces)"
    assert hasattr(env, "action_space"), "You must specify an action space (cf gym.spaces)"
    obs_space, act_space = env.observation_space, env.action_space
    assert _box(obs_space), "The observation space must inherit from gym.spaces"
    assert _box(act_space), "The action space must inherit from gym.spaces"
    # _check_box_obs
    if np.any(np.equal(obs_space.low, -np.inf)) or np.any(np.equal(obs_space.high, np.inf)):
        warns.append("unbounded observation space")
    # action space checks
    low, high = np.asarray(act_space.low), np.asarray(act_space.high)
    if np.any(np.abs(low) != np.abs(high)) or np.any(low != -1) or np.any(high != 1):
        warns.append("action space not symmetric / normalised")
    assert np.all(np.isfinite(np.array([low, high]))), "Continuous action space must have a finite lower and upper bound"
    if np.dtype(act_space.dtype) != np.dtype(np.float32):
        warns.append("action space is not float32")
    # _check_returned_values
    obs = env.reset()
    _check_obs(obs, obs_space, "reset")
    data = env.step(act_space.sample())
    assert len(data) == 4, "The `step()` method must return four values: obs, reward, done, info"
    obs, reward, done, info = data
    _check_obs(obs, obs_space, "step")
    assert isinstance(reward, (float, int)), "The reward returned by `step()` must be a float"
    assert isinstance(done, bool), "The `done` signal must be a boolean"
    assert isinstance(info, dict), "The `info` returned by `step()` must be a python dictionary"
    # _check_render
    if not skip_render_check:
        modes = getattr(env, "metadata", {}).get("render.modes")
        if modes is None:
            warns.append("no render modes declared")
        for mode in modes or []:
            env.render(mode=mode)
    # _check_nan (VecCheckNan over DummyVecEnv: auto-reset on done)
    env.reset()
    for _ in range(10):
        obs, reward, done, _ = env.step(act_space.sample())
        assert np.all(np.isfinite(obs)), "VecCheckNan: found NaN / inf in the observations"
        assert np.isfinite(reward), "VecCheckNan: found NaN / inf in the rewards"
        if done:
            env.reset()
    return warns
