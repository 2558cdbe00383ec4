"""Multi-GPU: one process per GPU, envs sharded by contiguous global id ranges.

Stepping needs no communication (envs are independent). The only
collective is optional: reassembling the per-step outputs of all shards on every rank
(``all_gather`` over RCCL/xGMI with the "nccl" backend), for a learner that wants the
global batch. Ranks own envs [offset, offset + n_local); the reset stream is keyed on
global ids, so results do not depend on the shard layout
(tests/test_gpu_state.py::test_sharded_stepping_is_bitwise_one_batch; multi-rank:
tests/test_gpu_dist.py: two ranks as separate processes, bitwise one batch).
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
    """One all_gather per step of every rank's step outputs into global tensors.

    Each rank's outputs are ONE block of rows [n_pad][state_dim + 2] fp32 — obs, reward,
    done as 0 / 1 — which the step kernel writes itself (``step(env, action)`` ->
    ``RocketBatch.step_rows`` / ``rr_step_rows``), so nothing runs between the step and the
    collective: one ``all_gather_into_tensor`` of equal blocks (RCCL over xGMI with the
    "nccl" backend; xGMI is point-to-point, so one large message per step rather than three
    small ones). Uneven shards (``shard()`` gives the first
    ``global % world`` ranks one extra env) are padded to n_pad = ceil(global / world) rows,
    and the global tensors are then gathered back into global env order (one index_select);
    with equal shards they are views of the received block. step() is a fixed sequence of
    device launches, so it can be captured in a hipGraph with the nccl backend.

    ``obs`` [global][state_dim], ``reward`` [global], ``done`` [global] (float 0 / 1) are
    refreshed in place by every call."""

    def __init__(self, n_local, state_dim, device, group=None, global_envs=None):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.ns = state_dim
        self.n_local = int(n_local)
        if global_envs is None:
            global_envs = self.n_local * self.world
        self.global_envs = int(global_envs)
        sizes = [shard(self.global_envs, self.world, r)[0] for r in range(self.world)]
        if sizes[self.rank] != self.n_local:
            raise ValueError("rank %d holds %d envs, shard(%d, %d) gives %d" % (self.rank, self.n_local,
                                                                             self.global_envs, self.world,
                                                                             sizes[self.rank]))
        self.n_pad = max(sizes)
        w = state_dim + 2
        self.send = torch.zeros((self.n_pad, w), dtype=torch.float32, device=device)
        self._recv = torch.empty((self.n_pad * self.world, w), dtype=torch.float32, device=device)
        self.even = all(s == self.n_pad for s in sizes)
        if self.even:
            self.rows = self._recv
            self._index = None
        else:  # global env g of rank r sits at row r * n_pad + (g - offset_r)
            idx = torch.cat([torch.arange(s, dtype=torch.int64) + r * self.n_pad for r, s in enumerate(sizes)])
            self._index = idx.to(device)
            self.rows = torch.empty((self.global_envs, w), dtype=torch.float32, device=device)
        self.obs = self.rows[:, :state_dim]      # views (row stride state_dim + 2)
        self.reward = self.rows[:, state_dim]
        self.done = self.rows[:, state_dim + 1]
        self._into = dist.get_backend(group) != "gloo"

    @property
    def local_rows(self):
        """This rank's send rows [n_local][state_dim + 2] (contiguous)."""
        return self.send[:self.n_local]

    def gather(self):
        """Gather every rank's send block; returns (obs, reward, done) global views."""
        if self._into:
            self.dist.all_gather_into_tensor(self._recv, self.send, group=self.group)
        elif self._recv.is_cuda:  # gloo moves host tensors only: stage through the host (CPU rehearsal path)
            host = self._recv.cpu()
            self.dist.all_gather(list(host.chunk(self.world)), self.send.cpu(), group=self.group)
            self._recv.copy_(host)
        else:
            self.dist.all_gather(list(self._recv.chunk(self.world)), self.send, group=self.group)
        if self._index is not None:
            self.torch.index_select(self._recv, 0, self._index, out=self.rows)
        return self.obs, self.reward, self.done

    def step(self, env, action):
        """One env step of this rank's shard written straight into the send rows
        (RocketBatch.step_rows), then the all-gather."""
        env.step_rows(action, self.local_rows)
        return self.gather()

    def __call__(self, obs, reward, done):
        """Gather outputs produced elsewhere (copies them into the send rows first)."""
        ns, m = self.ns, self.n_local
        self.send[:m, :ns].copy_(obs)
        self.send[:m, ns].copy_(reward)
        self.send[:m, ns + 1].copy_(done)
        return self.gather()
