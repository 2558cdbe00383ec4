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
    """One all_gather per step of the per-rank step outputs into global tensors: obs
    [n][state_dim], reward [n] and done [n] are packed as one fp32 row of state_dim + 2
    values per env (done as 0 / 1), gathered with a single collective (RCCL over xGMI with
    the "nccl" backend; SURVEY.md §8e: one large message per step instead of three), and
    exposed as views / conversions of the gathered block in global env order."""

    def __init__(self, n_local, state_dim, device, group=None):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.ns = state_dim
        n = n_local * self.world
        self._send = torch.empty((n_local, state_dim + 2), dtype=torch.float32, device=device)
        self._recv = torch.empty((n, state_dim + 2), dtype=torch.float32, device=device)
        self.obs = self._recv[:, :state_dim]            # view (row stride state_dim + 2)
        self.reward = self._recv[:, state_dim]          # view
        self.done = torch.empty((n,), dtype=torch.uint8, device=device)
        self._into = dist.get_backend(group) != "gloo"

    def _gather(self):
        if self._into:
            self.dist.all_gather_into_tensor(self._recv, self._send, group=self.group)
        elif self._recv.is_cuda:  # gloo moves host tensors only: stage through the host (CPU rehearsal path)
            host = self._recv.cpu()
            self.dist.all_gather(list(host.chunk(self.world)), self._send.cpu(), group=self.group)
            self._recv.copy_(host)
        else:
            self.dist.all_gather(list(self._recv.chunk(self.world)), self._send, group=self.group)

    def __call__(self, obs, reward, done):
        ns = self.ns
        self._send[:, :ns].copy_(obs)
        self._send[:, ns].copy_(reward)
        self._send[:, ns + 1].copy_(done)
        self._gather()
        self.done.copy_(self._recv[:, ns + 1])
        return self.obs, self.reward, self.done
