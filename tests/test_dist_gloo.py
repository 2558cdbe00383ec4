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


def _worker(rank, world, port, global_envs, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_local, off = shard(global_envs, world, rank)
    gid = torch.arange(off, off + n_local, dtype=torch.float32)
    g = ShardGather(n_local, 14, "cpu", global_envs=global_envs)
    # the rows the step kernel writes (rr_step_rows): obs[14], reward, done 0 / 1
    rows = g.local_rows
    rows[:, :14] = gid[:, None] + torch.arange(14, dtype=torch.float32) * 1e-3
    rows[:, 14] = -gid
    rows[:, 15] = (gid.long() % 3 == 0).float()
    o, r, d = g.gather()
    res = [o.numpy().copy(), r.numpy().copy(), d.numpy().copy()]
    # the legacy entry point: outputs produced elsewhere, copied into the send rows
    o2, r2, d2 = g(rows[:, :14].clone() + 1, rows[:, 14].clone() - 1, (gid.long() % 2 == 0).to(torch.uint8))
    res += [o2.numpy().copy(), r2.numpy().copy(), d2.numpy().copy()]
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("global_envs", [12, 13])
def test_gather_world2_gloo(global_envs):
    """Equal (12 = 6 + 6) and padded uneven (13 = 7 + 6) shards reassemble in global env order."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, global_envs, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    gid = np.arange(global_envs, dtype=np.float32)
    for _, (o, r, d, o2, r2, d2) in res:
        assert o.shape == (global_envs, 14)
        np.testing.assert_array_equal(o[:, 0], gid)
        np.testing.assert_array_equal(o[:, 13], gid + np.float32(13e-3))
        np.testing.assert_array_equal(r, -gid)
        np.testing.assert_array_equal(d, (gid.astype(int) % 3 == 0).astype(np.float32))
        np.testing.assert_array_equal(o2[:, 0], gid + 1)
        np.testing.assert_array_equal(r2, -gid - 1)
        np.testing.assert_array_equal(d2, (gid.astype(int) % 2 == 0).astype(np.float32))


def test_gather_rejects_wrong_shard_size():
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        with pytest.raises(ValueError):
            ShardGather(5, 14, "cpu", global_envs=6)
    finally:
        dist.destroy_process_group()


class _FakeRollout:
    """The fields ppo_update reads from a DeviceRollout, on the host."""

    def __init__(self, seed, n_steps=4, n_envs=32, ns=14, na=3):
        g = torch.Generator().manual_seed(seed)

        class _Env:
            num_envs = n_envs

        self.env, self.n_steps = _Env(), n_steps
        self.obs = torch.randn((n_steps, n_envs, ns), generator=g)
        self.actions = torch.randn((n_steps, n_envs, na), generator=g)
        self.log_probs = torch.randn((n_steps, n_envs), generator=g) - 3.0
        self.advantages = torch.randn((n_steps, n_envs), generator=g)
        self.returns = torch.randn((n_steps, n_envs), generator=g)


def _ppo_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rl_rocket_amd.rollout import MlpActorCritic, ppo_update

    torch.manual_seed(0)  # replicas start equal
    pol = MlpActorCritic(14, 3)
    opt = torch.optim.Adam(pol.parameters(), lr=3e-4, eps=1e-5)
    ro = _FakeRollout(seed=100 + rank)  # each rank's own env shard
    ppo_update(pol, opt, ro, n_epochs=1, batch_size=ro.n_steps * ro.env.num_envs, group=dist.group.WORLD)
    q.put((rank, [p.detach().numpy().copy() for p in pol.parameters()]))  # numpy: no shared-memory handles
    dist.barrier()
    dist.destroy_process_group()


def test_ppo_replicas_allreduce_world2_gloo():
    """One policy replica per rank: after an update on different local
    rollouts the replicas are identical, and equal to one optimizer step on the average of
    the two ranks' gradients."""
    from rl_rocket_amd.rollout import MlpActorCritic

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ppo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for a, b in zip(res[0], res[1]):
        np.testing.assert_array_equal(a, b)
    # reference: the same minibatch loss on each rank's data, gradients averaged, one step
    torch.manual_seed(0)
    ref = MlpActorCritic(14, 3)
    grads = []
    for rank in range(world):
        ro = _FakeRollout(seed=100 + rank)
        n = ro.n_steps * ro.env.num_envs
        ref.zero_grad(set_to_none=True)
        mean, value = ref(ro.obs.reshape(n, -1))
        lp = ref.log_prob(mean, ro.actions.reshape(n, -1))
        adv = ro.advantages.reshape(n)
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
        ratio = torch.exp(lp - ro.log_probs.reshape(n))
        pg = -torch.min(adv * ratio, adv * torch.clamp(ratio, 0.8, 1.2)).mean()
        vf = torch.nn.functional.mse_loss(ro.returns.reshape(n), value)
        loss = pg + 0.01 * (-ref.entropy(n).mean()) + 0.5 * vf
        loss.backward()
        grads.append([p.grad.clone() for p in ref.parameters()])
    for p, g0, g1 in zip(ref.parameters(), *grads):
        p.grad = (g0 + g1) / 2
    torch.nn.utils.clip_grad_norm_(ref.parameters(), 0.5)
    torch.optim.Adam(ref.parameters(), lr=3e-4, eps=1e-5).step()
    for a, b in zip(res[0], ref.parameters()):
        np.testing.assert_allclose(a, b.detach().numpy(), atol=1e-6, rtol=1e-5)


def _rank_rows_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import per_rank_rows

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["LOCAL_RANK"] = str(rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = per_rank_rows(dist, 0.1 * (rank + 1), 0.004 * (rank + 1), 20)  # rank r: (r + 1) x the wall / device time
    q.put((rank, rows))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_per_rank_rows_world4_gloo():
    """at world > 1 the bench line carries every rank's own wall time and events
    figure (one all_gather_object), not only rank 0's and the max; a 4-rank rehearsal shows four
    entries, in rank order, identical on every rank."""
    world = 4
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_rows_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        rows = got[r]
        assert [x["rank"] for x in rows] == list(range(world)) and rows == got[0]
        for k, x in enumerate(rows):
            assert abs(x["wall_ms_per_step"] - 5.0 * (k + 1)) < 1e-9
            assert abs(x["kernel_us"] - 4.0 * (k + 1)) < 1e-9 and x["local_rank"] == k
