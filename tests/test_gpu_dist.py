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


def _run(world, extra=()):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), WORLD_SIZE=str(world),
               HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "dist_worker.py")] + list(extra),
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=100))
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
