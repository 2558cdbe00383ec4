"""Multi-GPU: one process per GPU, envs sharded by contiguous global id ranges.

Stepping needs no communication (envs are independent). The only
collective is optional: reassembling the per-step outputs of all shards on every rank
(``all_gather`` over RCCL/xGMI with the "nccl" backend), for a learner that wants the
global batch. Ranks own envs [offset, offset + n_local); the reset stream is keyed on
global ids, so results do not depend on the shard layout.
"""


def shard(global_envs, world_size, rank):
    """(n_local, offset) of `rank` when `global_envs` are split over `world_size` ranks
    (the first `global_envs % world_size` ranks get one extra env)."""
    if world_size <= 0 or not 0 <= rank < world_size:
        raise ValueError("bad rank/world_size")
    base, extra = divmod(int(global_envs), int(world_size))
    n_local = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return n_local, offset


class ShardGather:
    """all_gather of equal-size per-rank step outputs into preallocated global tensors."""

    def __init__(self, n_local, state_dim, device, group=None):
        import torch
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        n = n_local * self.world
        self.obs = torch.empty((n, state_dim), dtype=torch.float32, device=device)
        self.reward = torch.empty((n,), dtype=torch.float32, device=device)
        self.done = torch.empty((n,), dtype=torch.uint8, device=device)
        self._into = dist.get_backend(group) != "gloo"

    def _gather(self, out, t):
        if self._into:
            self.dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        elif out.is_cuda:  # gloo moves host tensors only: stage through the host (CPU rehearsal path)
            host = out.cpu()
            self.dist.all_gather(list(host.chunk(self.world)), t.cpu().contiguous(), group=self.group)
            out.copy_(host)
        else:
            self.dist.all_gather(list(out.chunk(self.world)), t.contiguous(), group=self.group)

    def __call__(self, obs, reward, done):
        self._gather(self.obs, obs)
        self._gather(self.reward, reward)
        self._gather(self.done, done)
        return self.obs, self.reward, self.done
