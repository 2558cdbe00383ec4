"""world_size-2 gloo test of the multi-GPU path's host logic: shard layout and the
all_gather reassembly of per-shard step outputs in global env order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rl_rocket_amd.dist import ShardGather, shard


def test_shard_partition():
    for g, w in ((524288, 8), (10, 3), (7, 4), (65536, 1)):
        parts = [shard(g, w, r) for r in range(w)]
        assert sum(n for n, _ in parts) == g
        off = 0
        for n, o in parts:
            assert o == off
            off += n
    with pytest.raises(ValueError):
        shard(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_local, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _, off = shard(n_local * world, world, rank)
    gid = torch.arange(off, off + n_local, dtype=torch.float32)
    obs = gid[:, None].repeat(1, 14) + torch.arange(14, dtype=torch.float32) * 1e-3
    rew = -gid
    done = (gid.long() % 3 == 0).to(torch.uint8)
    g = ShardGather(n_local, 14, "cpu")
    o, r, d = g(obs, rew, done)
    q.put((rank, o.numpy().copy(), r.numpy().copy(), d.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_world2_gloo():
    world, n_local = 2, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_local, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    gid = np.arange(world * n_local, dtype=np.float32)
    for _, o, r, d in res:
        np.testing.assert_array_equal(o[:, 0], gid)
        np.testing.assert_array_equal(r, -gid)
        np.testing.assert_array_equal(d, (gid.astype(int) % 3 == 0).astype(np.uint8))
