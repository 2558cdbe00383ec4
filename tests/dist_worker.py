"""One rank of tests/test_gpu_dist.py (started as a child process by the test; not a test module).

Every rank steps its shard of G envs (rl_rocket_amd.dist.shard: uneven shards, global env ids)
on cuda:0 with the same seeded global action sequence, and gathers the step rows of all ranks
with ShardGather.step (rr_step_rows into the send rows + one all_gather over gloo). Each rank
also sends its done list (global env ids, terminal obs rows, episode returns and lengths, from
rr_fetch_done) to rank 0. Rank 0 steps ONE batch of all G envs with the same actions and counts,
at every step, the rows where the gathered obs / reward / done or the done lists differ (bitwise).
Rank 0 prints one JSON line; exit status 1 on any mismatch.

Environment: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT (the test sets them).
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
    import datetime

    import numpy as np
    import torch
    import torch.distributed as dist

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.dist import ShardGather, shard
    from rl_rocket_amd.params import ENV_CONFIG_6DOF

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)  # every rank on the box's one GPU
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=90))
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
    bad_rows, bad_done, n_done, n_trunc = 0, 0, 0, 0
    for t in range(a.steps):
        act = torch.rand((G, 3), device=dev, generator=gen) * 2 - 1  # identical on every rank
        obs, rew, done = g.step(env, act[off:off + n_local].contiguous())
        idx, tobs, ret, ln = env.fetch_done()
        lists = [None] * world if rank == 0 else None
        dist.gather_object((idx.astype(np.int64) + off, tobs, ret, ln), lists, dst=0)
        if ref is not None:
            o, r, d, tr = ref.step(act)
            bad_rows = max(bad_rows, int((obs != o).any(1).sum() + (rew != r).sum() + (done != d.float()).sum()))
            ri, rt, rr, rl = ref.fetch_done()
            gi = np.concatenate([x[0] for x in lists])
            same = (np.array_equal(gi, ri.astype(np.int64)) and
                    np.array_equal(np.concatenate([x[1] for x in lists]), rt) and
                    np.array_equal(np.concatenate([x[2] for x in lists]), rr) and
                    np.array_equal(np.concatenate([x[3] for x in lists]), rl))
            bad_done += 0 if same else 1
            n_done += len(ri)
            n_trunc += int(tr.sum())
    torch.cuda.synchronize(dev)
    ok = True
    if rank == 0:
        ok = bad_rows == 0 and bad_done == 0
        print(json.dumps({"check": "sharded step + all_gather (rr_step_rows) == one batch, bitwise", "ok": ok,
                          "mismatching_rows_worst_step": bad_rows, "steps_with_done_list_mismatch": bad_done,
                          "world_size": dist.get_world_size(), "backend": dist.get_backend(), "global_envs": G,
                          "steps": a.steps, "shards": [shard(G, world, r)[0] for r in range(world)],
                          "done_total": n_done, "truncated_total": n_trunc,
                          "max_episode_steps": a.max_episode_steps}), flush=True)
    env.close()
    if ref is not None:
        ref.close()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
