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


def test_iteration_matches_indexing_and_keeps_handed_out_dicts():
    env = _env()
    trunc = np.array([0, 1, 0, 0, 0], np.uint8)
    idx, tobs, ret, ln = env.batch.fetch_done()
    infos = LazyInfos(5, env._done_rows(idx, tobs, ret, ln, trunc[idx], 1.5), None, ["a"])
    d3 = infos[3]
    d3["mark"] = 1  # a dict handed out before iterating stays the env's dict
    lst = list(infos)
    assert len(lst) == 5 and lst[3] is d3 and lst[3]["mark"] == 1
    assert lst[1]["TimeLimit.truncated"] is True and lst[1]["episode"]["l"] == 800
    assert lst[0] == {} and lst[2] == {} and lst[4] == {}
    assert len({id(d) for d in lst}) == 5  # every env its own dict, as DummyVecEnv's list
    assert infos[1] is lst[1] and infos[-1] is lst[4]
    # SB3 1.6 _update_info_buffer over every env
    eps = [i.get("episode") for i in infos if i.get("episode") is not None]
    assert [e["l"] for e in eps] == [800, 42]


def test_iteration_with_terms_carries_terms_and_done_rows():
    env = _env(2)
    idx, tobs, ret, ln = np.array([1], np.int32), np.ones((1, 14), np.float32), np.float32([2.0]), np.int32([5])
    terms = np.array([[1.0, 2.0], [0.0, 1.0], [0.0, 0.0]])
    infos = LazyInfos(2, env._done_rows(idx, tobs, ret, ln, np.uint8([0]), 0.0), terms, ["velocity_tracking"])
    lst = list(infos)
    assert lst[0] == {"rewards_dict": {"velocity_tracking": 1.0}, "bounds_violation": False}
    assert lst[1]["rewards_dict"] == {"velocity_tracking": 2.0} and lst[1]["bounds_violation"] is True
    assert lst[1]["episode"]["l"] == 5


def test_iteration_is_no_slower_than_a_plain_list():
    """SB3's per-step loop over all infos (collect_rollouts -> _update_info_buffer) at
    N = 65 536: iterating the lazy infos (building the list included) costs no more than
    iterating a plain list of N dicts that was built the same way (the
    Sequence.__iter__ fallback was ~10x slower)."""
    import time

    n = 65536
    idx = np.arange(0, n, 70, dtype=np.int32)
    env = _env(n)
    rows = env._done_rows(idx, np.zeros((len(idx), 14), np.float32), np.zeros(len(idx), np.float32),
                          np.full(len(idx), 7, np.int32), np.zeros(len(idx), np.uint8), 0.0)

    def consume(infos):
        k = 0
        for i, info in enumerate(infos):
            if info.get("episode") is not None:
                k += 1
            info.get("is_success")
        return k

    def best(make):
        t = []
        for _ in range(15):
            x = make()
            t0 = time.perf_counter()
            k = consume(x)
            t.append(time.perf_counter() - t0)
        return min(t), k

    t_lazy, k = best(lambda: LazyInfos(n, rows, None, ["a"]))
    assert k == len(idx)

    def plain():  # DummyVecEnv's list: N dicts built in step_wait, then the same loop
        t0 = time.perf_counter()
        lst = [{} for _ in range(n)]
        for i in idx.tolist():
            lst[i] = {"episode": {"r": 0.0, "l": 7, "t": 0.0}, "terminal_observation": None}
        return time.perf_counter() - t0, lst

    t_plain = []
    for _ in range(15):
        tb, lst = plain()
        t0 = time.perf_counter()
        consume(lst)
        t_plain.append(tb + time.perf_counter() - t0)
    t_plain = min(t_plain)
    print("lazy %.2f ms, plain list build + iterate %.2f ms" % (t_lazy * 1e3, t_plain * 1e3))
    # best of 15 each; the bar catches the ~10x regression, not scheduler noise
    assert t_lazy <= 1.5 * t_plain + 0.002


def test_env_is_wrapped_reports_monitor_and_time_limit():
    env = _env()

    class Monitor:
        pass

    class TimeLimit:
        pass

    class Other:
        pass

    env._indices = RocketVecEnv._indices.__get__(env)
    assert env.env_is_wrapped(Monitor) == [True] * 5
    assert env.env_is_wrapped(TimeLimit, indices=[0, 1]) == [True, True]
    assert env.env_is_wrapped(Other) == [False] * 5
    env.monitor = False
    env.max_episode_steps = 0
    assert env.env_is_wrapped(Monitor) == [False] * 5 and env.env_is_wrapped(TimeLimit) == [False] * 5
