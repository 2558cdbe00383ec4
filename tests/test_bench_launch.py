"""bench.py's multi-rank launch contract and the EpisodeAnalyzer host logic
(no GPU needed)."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launch_plan():
    from bench import launch_plan

    assert launch_plan(1, {}) == ("run", None)
    assert launch_plan(2, {}) == ("spawn", None)
    assert launch_plan(8, {}) == ("spawn", None)
    assert launch_plan(2, {"WORLD_SIZE": "2"}) == ("run", None)
    assert launch_plan(1, {"WORLD_SIZE": "1"}) == ("run", None)
    plan, msg = launch_plan(8, {"WORLD_SIZE": "1"})
    assert plan == "error" and "WORLD_SIZE" in msg
    assert launch_plan(0, {})[0] == "error"


def _run(args, **env):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, capture_output=True,
                          text=True, timeout=300)


def test_bench_gpus_fails_loudly_without_enough_gpus():
    """--gpus N > visible GPUs: non-zero exit and a message, never a silent one-GPU line. (On a
    box with >= 2 GPUs this would start ranks; the test only runs where fewer are visible.)"""
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("this host has >= 2 GPUs")
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "1"])
    assert r.returncode != 0 and "needs 2 visible GPU" in r.stderr
    assert '"metric"' not in r.stdout


def test_bench_gpus_must_match_world_size():
    r = _run(["--gpus", "8"], WORLD_SIZE="1")
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr


def _stub_env(T=6):
    from rl_rocket_amd.envs import Rocket6DOF
    from rl_rocket_amd.params import STATE_NAMES_6DOF

    u = object.__new__(Rocket6DOF)
    u.state_names = list(STATE_NAMES_6DOF)
    u.action_names = ["gimbal_y", "gimbal_z", "thrust"]
    u.target_r = 30
    u.landing_target = [0, 0, 0]
    rng = np.random.default_rng(0)
    states = [rng.normal(size=14) for _ in range(T + 1)]

    class SIM:
        pass

    u.SIM = SIM()
    u.SIM.states, u.SIM.actions = states, [[0, 0, 0]] + [list(rng.normal(size=3)) for _ in range(T)]
    u.waypoint = 50.0  # vtarg_history is derived from SIM.states (envs._RocketBase.vtarg_history)
    u.observation_space = u.action_space = None
    return u


def test_episode_analyzer_statistics_host():
    sys.path.insert(0, os.path.join(ROOT, "compat"))
    from my_environment.wrappers import EpisodeAnalyzer

    u = _stub_env()
    script = [({"rew_goal": 0.0, "attitude_constraint": 0.0}, False)] * 5 + [({"rew_goal": 10.0,
                                                                                "attitude_constraint": 0.0}, True)]
    it = iter(script)

    def step(a):
        rd, done = next(it)
        return np.zeros(14, np.float32), 1.0, done, {"rewards_dict": rd}

    u.step = step
    env = EpisodeAnalyzer(u)
    for _ in range(6):
        env.step(np.zeros(3))
    st = env.last_episode["stats"]
    assert st["ep_statistic/landing_success"] == 10.0
    np.testing.assert_allclose(st["ep_statistic/used_mass"], u.SIM.states[0][-1] - u.SIM.states[-1][-1])
    np.testing.assert_allclose(st["final_errors/vx"], abs(u.SIM.states[-1][3]))
    assert len(env.last_episode["rewards"]) == 6 and env.rewards_info == []
    # the shim's figures (plotly is in this image)
    import plotly.graph_objects as go

    f = u.get_trajectory_plotly()
    assert isinstance(f, go.Figure) and [t.type for t in f.data] == ["scatter3d", "cone", "surface"]
    assert len(f.data[0].x) == len(u.SIM.states) and len(f.data[1].u) == len(u.SIM.states)
    f = u.get_vtarg_trajectory()
    assert [t.type for t in f.data] == ["scatter3d", "cone", "scatter3d"]
    assert len(f.data[1].u) == len(u.SIM.states) - 1  # one target velocity per step
    f = u.get_attitude_trajectory()
    assert [t.name for t in f.data] == ["q0", "q1", "q2", "q3"]


def test_host_cores_uses_the_affinity_mask_narrowed_by_quota_and_omp(monkeypatch):
    """cpu_baseline's all-cores leg: the affinity count, narrowed by the cgroup CPU quota and
    OMP_NUM_THREADS when set (no fixed cap), with where the count came from."""
    import bench

    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(40)))
    monkeypatch.setattr(bench, "_cgroup_cpus", lambda: None)
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    assert bench.host_cores() == (40, {"affinity": 40})
    monkeypatch.setattr(bench, "_cgroup_cpus", lambda: 24)
    assert bench.host_cores() == (24, {"affinity": 40, "cgroup_quota": 24})
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    assert bench.host_cores() == (16, {"affinity": 40, "cgroup_quota": 24, "OMP_NUM_THREADS": 16})


def test_rollout_roofline_counts():
    """The configs[4] roofline's algorithmic counts: SB3 MlpPolicy (64x64) towers' GEMM FLOPs per
    env-step and the collect's HBM bytes per env-step."""
    import bench

    # pi: 14*64 + 64*64 + 64*3 MACs, vf: 14*64 + 64*64 + 64*1 MACs, 2 FLOP each
    assert bench.rollout_flops_per_env_step(14, 3) == 2 * (896 + 4096 + 192) + 2 * (896 + 4096 + 64) == 20480
    assert bench.rollout_flops_per_env_step(7, 2) == 2 * (448 + 4096 + 128) + 2 * (448 + 4096 + 64)
    # buffer slices per step: obs 56 + action 12 + value / log-prob / start / reward / adv / ret 24
    b16 = bench.rollout_bytes_per_env_step(14, 3, 16)
    assert bench.rollout_bytes_per_env_step(14, 3, 10 ** 9) == pytest.approx(92.0)
    assert 92.0 < b16 < 110.0


def test_committed_traces_quote_the_upper_median_of_this_machine_code(tmp_path, monkeypatch):
    """bench.py quotes, of the committed traces measured on the running kernel's machine code,
    the upper median (re-runs on other boxes scatter; never the best of two) and lists them;
    traces of other code are ignored."""
    import json

    import bench

    name = "void step_kernel<6, 0, false, true, 4, false>(...)"
    for tag, mean, isa in (("a", 4800.0, "h1"), ("b", 4300.0, "h1"), ("c", 4000.0, "old"), ("d", 4700.0, "h1")):
        d = tmp_path / "profiles" / "r9" / tag
        d.mkdir(parents=True)
        (d / "rocprof_step_k20_n64.json").write_text(json.dumps(
            {"kernel": "step_kernel<6,RK4>", "kernel_name": name, "isa_hash": isa, "mean_ns": mean}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "_isa_hashes", lambda: {name: "h1"})
    d, src = bench.stored_rocprof(6, 64, 20)
    assert d["mean_ns"] == 4700.0 and src.endswith("r9/d/rocprof_step_k20_n64.json")  # of 4300 / 4700 / 4800
    assert d["median_of"].startswith("3 files")
    monkeypatch.setattr(bench, "_isa_hashes", lambda: {name: "other"})
    d, why = bench.stored_rocprof(6, 64, 20)
    assert d is None and "no file" in why


def test_committed_traces_of_another_launch_mode_are_not_quoted(tmp_path, monkeypatch):
    """the line's frac quotes only traces recorded with the running command's launch
    mode (graph replays at K >= 8): of three graph traces and two direct ones of the same code, the
    upper median of the graph ones; with no graph trace, none (the reason names the other mode).
    PMC traffic takes the lower median (a larger byte count would raise a bandwidth: ADVICE r4)."""
    import json

    import bench

    name = "void step_kernel<6, 0, false, true, 4, false>(...)"
    for tag, mean, launch in (("a", 4800.0, "graph"), ("b", 4300.0, "direct: tools/libbench_timed.so"),
                              ("c", 4500.0, "graph"), ("d", 4000.0, "direct: x"), ("e", 4900.0, "graph")):
        d = tmp_path / "profiles" / "r9" / tag
        d.mkdir(parents=True)
        (d / "rocprof_step_k20_n64.json").write_text(json.dumps(
            {"kernel": "step_kernel<6,RK4>", "kernel_name": name, "isa_hash": "h1", "mean_ns": mean,
             "launch": launch}))
        (d / "pmc_traffic_n64.json").write_text(json.dumps(
            {"kernel": "step_kernel<6,RK4>", "kernel_name": name, "isa_hash": "h1", "traffic_bytes": mean * 1000}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "_isa_hashes", lambda: {name: "h1"})
    d, src = bench.stored_rocprof(6, 64, 20, launch="graph")
    assert d["mean_ns"] == 4800.0 and d["median_of"].startswith("3 files") and "graph launches only" in d["selection"]
    d, src = bench.stored_rocprof(6, 64, 20, launch="direct")
    assert d["mean_ns"] == 4300.0  # upper median of 4000 / 4300
    d, why = bench.stored_rocprof(6, 64, 20, launch="eager")
    assert d is None and "other launch mode" in why
    traffic, src = bench.stored_traffic(6, 64)
    assert traffic == 4500.0 * 1000  # lower median of five
    assert bench.launch_kind("graph") == "graph" and bench.launch_kind("direct: tools/x") == "direct"
    assert bench.launch_kind("rr_step per step") == "eager"
