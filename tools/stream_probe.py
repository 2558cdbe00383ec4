"""Concurrent env shards on one GPU: S ``RocketBatch`` shards of N/S envs stepped on S
streams from one hipGraph (S independent chains of back-to-back step launches), against
one batch of N envs on one stream: does one chain's per-launch boundary (launch, barrier,
end-of-kernel cache actions) hide under another chain's kernels?

    python tools/stream_probe.py [--n 65536] [--streams 1,2,4] [--steps 4096] [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(n, S, steps, gs=64):
    import torch

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF

    dev = torch.device("cuda", 0)
    m = n // S
    envs = [RocketBatch(m, model=6, device=dev, max_episode_steps=800, auto_reset=True, episode_stats=False,
                        env_id_offset=k * m, **ENV_CONFIG_6DOF) for k in range(S)]
    for e in envs:
        e.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    pool = torch.rand((8, n, 3), device=dev, generator=g) * 2 - 1
    pools = [pool[:, k * m:(k + 1) * m].contiguous() for k in range(S)]
    for k in range(30):
        for j, e in enumerate(envs):
            e.step(pools[j][k % 8])
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    cap.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.graph(graph, stream=cap):
        for st in streams:
            st.wait_stream(cap)
        for j, (e, st) in enumerate(zip(envs, streams)):
            with torch.cuda.stream(st):
                for k in range(gs):
                    e.step(pools[j][k % 8])
        for st in streams:
            cap.wait_stream(st)
    torch.cuda.current_stream(dev).wait_stream(cap)
    graph.replay()
    torch.cuda.synchronize()
    reps = max(2, steps // gs)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cur = torch.cuda.current_stream(dev)
    e0.record(cur)
    for _ in range(reps):
        graph.replay()
    e1.record(cur)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (reps * gs)
    for e in envs:
        e.close()
    return us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--streams", default="1,2,4")
    ap.add_argument("--steps", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    res = {}
    for _ in range(a.rounds):
        for S in [int(x) for x in a.streams.split(",")]:
            res.setdefault(S, []).append(run(a.n, S, a.steps))
    out = {"n": a.n, "us_per_step": {S: statistics.median(v) for S, v in res.items()},
           "G_env_steps_per_s": {S: a.n / statistics.median(v) / 1e3 for S, v in res.items()}, "runs": res}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
