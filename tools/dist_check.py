"""Multi-rank check of the sharded step + all_gather, run under torchrun:

    RR_BENCH_ONE_DEVICE=1 RR_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 tools/dist_check.py [--global-envs 20003]

Every rank steps its shard of G envs (rl_rocket_amd.dist.shard: uneven shards, global env ids)
with the same seeded global action sequence and gathers the step rows of all ranks with
ShardGather.step (rr_step_rows + one all_gather). Rank 0 also steps ONE batch of all G envs
with the same actions and requires the gathered obs / reward / done to be bitwise equal to it
at every step (auto-resets and TimeLimit inside the run). Prints one JSON line on rank 0 and
exits non-zero on a mismatch. Same knobs as bench.py: RR_BENCH_ONE_DEVICE=1 puts every rank on
cuda:0, RR_BENCH_BACKEND (default nccl).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--global-envs", type=int, default=20003)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--max-episode-steps", type=int, default=15)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.dist import ShardGather, shard
    from rl_rocket_amd.params import ENV_CONFIG_6DOF

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = 0 if os.environ.get("RR_BENCH_ONE_DEVICE") == "1" else int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("RR_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(backend)
    G = a.global_envs
    n_local, off = shard(G, world, rank)
    env = RocketBatch(n_local, model=6, device=dev, max_episode_steps=a.max_episode_steps, env_id_offset=off,
                      **ENV_CONFIG_6DOF)
    env.reset()
    g = ShardGather(n_local, env.state_dim, dev, global_envs=G)
    ref = None
    if rank == 0:
        ref = RocketBatch(G, model=6, device=dev, max_episode_steps=a.max_episode_steps, **ENV_CONFIG_6DOF)
        ref.reset()
    gen = torch.Generator(device=dev).manual_seed(1234)
    worst, n_done = 0, 0
    for t in range(a.steps):
        act = torch.rand((G, 3), device=dev, generator=gen) * 2 - 1  # identical on every rank
        obs, rew, done = g.step(env, act[off:off + n_local].contiguous())
        if ref is not None:
            o, r, d, _ = ref.step(act)
            bad = int((obs != o).any(1).sum() + (rew != r).sum() + (done != d.float()).sum())
            worst = max(worst, bad)
            n_done += int(d.sum())
    torch.cuda.synchronize(dev)
    if rank == 0:
        print(json.dumps({"check": "sharded step + all_gather == one batch (bitwise)", "ok": worst == 0,
                          "mismatching_rows_worst_step": worst, "world_size": dist.get_world_size(),
                          "backend": dist.get_backend(), "global_envs": G, "steps": a.steps,
                          "shards": [shard(G, world, r)[0] for r in range(world)], "done_total": n_done,
                          "max_episode_steps": a.max_episode_steps}), flush=True)
    env.close()
    if ref is not None:
        ref.close()
    dist.destroy_process_group()
    if rank == 0 and worst:
        sys.exit(1)


if __name__ == "__main__":
    main()
