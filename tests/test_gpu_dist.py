"""configs[3]'s multi-process path in the GPU suite: 2 ranks started as child
processes (each a fresh interpreter: nothing is inherited from this process's GPU context), both
on cuda:0 over gloo (RCCL refuses two ranks on one GPU), 20 003 envs in uneven shards, TimeLimit
15 so that every env ends episodes (auto-reset and truncation inside the run). The gathered obs /
reward / done rows (ShardGather.step -> rr_step_rows + all_gather) and the done lists (terminal
rows, returns, lengths) must be bitwise ONE 20 003-env batch's at every step (tests/dist_worker.py).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, extra=(), timeout=100):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), WORLD_SIZE=str(world),
               HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "dist_worker.py")] + list(extra),
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return [p.returncode for p in procs], outs


@pytest.mark.gpu
def test_two_ranks_step_bitwise_one_batch():
    rcs, outs = _run(2)
    line = [x for x in outs[0][0].splitlines() if x.startswith("{")]
    assert rcs == [0, 0], (rcs, [o[1][-2000:] for o in outs])
    res = json.loads(line[-1])
    print(res)
    assert res["ok"] and res["world_size"] == 2 and res["shards"] == [10002, 10001]
    assert res["done_total"] > 20003 and res["truncated_total"] > 0  # every env reset, time-outs included


@pytest.mark.gpu
def test_four_ranks_at_configs3_global_size_step_bitwise_one_batch():
    """configs[3]'s workload as far as one GPU goes. Its global size, 524 288 envs,
    + 3 so the shards are uneven (131 073 x 3 + 131 072: the first three ranks run the plain step
    kernel, the last the helper-wave kernel, the one-batch twin the plain kernel), over 4 ranks
    (separate processes, all on cuda:0, gloo). TimeLimit 15 over 40 steps: every env resets twice
    (all 524 291 at once at steps 15 and 30, besides the physics ends). At every step the gathered
    rows and the done lists (global ids, terminal rows, returns, lengths) are bitwise ONE
    524 291-env batch's."""
    g = 524288 + 3
    rcs, outs = _run(4, ["--global-envs", str(g), "--steps", "40", "--max-episode-steps", "15"], timeout=240)
    line = [x for x in outs[0][0].splitlines() if x.startswith("{")]
    assert rcs == [0, 0, 0, 0], (rcs, [o[1][-2000:] for o in outs])
    res = json.loads(line[-1])
    print(res)
    assert res["ok"] and res["world_size"] == 4 and res["global_envs"] == g
    assert res["shards"] == [131073, 131073, 131073, 131072]
    assert res["done_total"] >= 2 * g and res["truncated_total"] > g
