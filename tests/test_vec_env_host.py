"""Host logic of RocketVecEnv (SB3 VecEnv semantics) with a stand-in batch: the info
dicts SB3 1.6 DummyVecEnv + gym TimeLimit + Monitor would produce for done envs."""
import numpy as np

from rl_rocket_amd.vec_env import LazyInfos, RocketVecEnv


class _FakeBatch:
    def __init__(self, n):
        self.num_envs = n
        self.terms = None

    def fetch_done(self):
        idx = np.array([1, 3], np.int32)
        tobs = np.arange(2 * 14, dtype=np.float32).reshape(2, 14)
        return idx, tobs, np.float32([-12.5, 3.25]), np.int32([800, 42])


def _env(n=5):
    env = RocketVecEnv.__new__(RocketVecEnv)
    env.num_envs = n
    env.batch = _FakeBatch(n)
    env.monitor = True
    env.info_terms = False
    env.max_episode_steps = 800
    env.episode_returns, env.episode_lengths, env.episode_times = [], [], []
    env._t_start = 0.0

    class _Cfg:
        term_names = ["a"]

    env.cfg = _Cfg()
    return env


def test_done_infos_match_sb3_semantics():
    env = _env()
    trunc = np.array([0, 1, 0, 0, 0], np.uint8)
    idx, tobs, ret, ln = env.batch.fetch_done()
    rows = env._done_rows(idx, tobs, ret, ln, trunc[idx], 1.5)
    assert rows._pos is None  # the env -> row map is built on the first infos access, not per step
    infos = LazyInfos(5, rows, None, ["a"])
    assert len(infos) == 5
    assert infos[0] == {} and infos[2] == {} and infos[4] == {}
    assert infos[1]["TimeLimit.truncated"] is True
    assert "TimeLimit.truncated" not in infos[3]
    np.testing.assert_array_equal(infos[3]["terminal_observation"], np.arange(14, 28, dtype=np.float32))
    assert infos[1]["episode"]["r"] == -12.5 and infos[1]["episode"]["l"] == 800 and infos[1]["episode"]["t"] == 1.5
    assert infos[3]["episode"]["l"] == 42
    assert infos.done_indices() == [1, 3]
    assert env.episode_lengths == [800, 42] and env.episode_returns == [-12.5, 3.25] and env.episode_times == [1.5] * 2
    # SB3 VecNormalize mutates done infos in place: the mutation must persist
    infos[1]["terminal_observation"] = "x"
    assert infos[1]["terminal_observation"] == "x"
    assert infos[-1] == {} and len(infos[1:3]) == 2


def test_lazy_infos_terms():
    terms = np.array([[1.0, 2.0], [0.0, 1.0], [0.0, 0.0]])
    li = LazyInfos(2, None, terms, ["velocity_tracking"])
    assert li[0] == {"rewards_dict": {"velocity_tracking": 1.0}, "bounds_violation": False}
    assert li[1]["bounds_violation"] is True
