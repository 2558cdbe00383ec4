"""On-device PPO rollouts: policy inference, env step and rollout buffer all in HBM.

SURVEY.md §8(f) rank 2 / BASELINE.json configs[4]: stock SB3 1.6 copies every observation
batch to a NumPy ``RolloutBuffer`` on the host; here the PyTorch policy consumes the obs
tensor the step kernel wrote, the sampled actions go straight back into ``rr_step``, and
the buffer, GAE and the PPO update stay on the GPU. One ``collect`` (n_steps × [policy
forward + sample + env step + buffer writes]) can be captured into a hipGraph.

``MlpActorCritic`` mirrors SB3 1.6 ``ActorCriticPolicy`` defaults for PPO with
``"MlpPolicy"`` (the reference's ``sb3_config["policy_type"]``, configuration_file.py:41):
separate pi / vf MLPs [64, 64] with tanh, diagonal Gaussian with state-independent
log_std (init 0), orthogonal init (gain sqrt(2) hidden, 0.01 policy head, 1 value head);
actions are clipped to the Box [-1, 1] before the env step, as SB3 does.
Timeouts are bootstrapped like SB3 1.6 ``collect_rollouts``:
reward += gamma * V(terminal_obs) where TimeLimit truncated the episode.
"""
import math

import torch
from torch import nn


class _LinearFn(torch.autograd.Function):
    """``F.linear`` whose bias gradient is a GEMM with a row of ones instead of a column sum.

    On PyTorch 2.10 / ROCm 7 a hipGraph that runs a GEMM and then a column sum (``sum(0)``) of a
    tensor produced in the same graph returns a wrong sum from its second replay on (the first
    replay and eager runs are right; the round-3 probe (profiles/r03/r03i/probe_graph_reduce.txt): errors of 10^2 on sums of
    ~10^3 at 8 192 and 65 536 rows, the GEMM output itself correct, the same sum as
    ``ones @ g`` correct). A Linear's bias gradient is exactly that column sum of the output
    gradient, so GraphedPPOUpdate's replays trained with wrong hidden-layer bias gradients."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return torch.nn.functional.linear(x, w, b)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1])
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = g @ w
        if ctx.needs_input_grad[1]:
            gw = g2.t() @ x.reshape(-1, x.shape[-1])
        if ctx.needs_input_grad[2]:
            gb = (g2.new_ones(1, g2.shape[0]) @ g2)[0]
        return gx, gw, gb


class _Linear(nn.Linear):
    """nn.Linear (same parameters, initialisation and packing) through _LinearFn."""

    def forward(self, x):
        return _LinearFn.apply(x, self.weight, self.bias)


class MlpActorCritic(nn.Module):
    def __init__(self, obs_dim, act_dim, hidden=(64, 64), log_std_init=0.0):
        super().__init__()
        self.hidden = tuple(hidden)

        def mlp():
            layers, d = [], obs_dim
            for h in hidden:
                layers += [_Linear(d, h), nn.Tanh()]
                d = h
            return nn.Sequential(*layers)

        self.pi_net, self.vf_net = mlp(), mlp()
        self.action_net = _Linear(hidden[-1], act_dim)
        self.value_net = _Linear(hidden[-1], 1)
        self.log_std = nn.Parameter(torch.full((act_dim,), float(log_std_init)))
        for net in (self.pi_net, self.vf_net):
            for m in net:
                if isinstance(m, nn.Linear):
                    nn.init.orthogonal_(m.weight, gain=math.sqrt(2))
                    nn.init.zeros_(m.bias)
        nn.init.orthogonal_(self.action_net.weight, gain=0.01)
        nn.init.zeros_(self.action_net.bias)
        nn.init.orthogonal_(self.value_net.weight, gain=1.0)
        nn.init.zeros_(self.value_net.bias)

    def forward(self, obs):
        return self.action_net(self.pi_net(obs)), self.value_net(self.vf_net(obs)).squeeze(-1)

    def value(self, obs):
        return self.value_net(self.vf_net(obs)).squeeze(-1)

    def log_prob(self, mean, actions):
        std = self.log_std.exp()
        return (-((actions - mean) ** 2) / (2 * std * std) - self.log_std - 0.5 * math.log(2 * math.pi)).sum(-1)

    def entropy(self, n):
        return (0.5 + 0.5 * math.log(2 * math.pi) + self.log_std).sum().expand(n)


POLICY_PRECISIONS = {"fp32": 0, "bf16": 1, "fp16x3": 2}  # RR_POLICY_FP32 / RR_POLICY_BF16 / RR_POLICY_FP16X3


# folded fp32 tanh of the rollout pack (rocket_policy.inc kPolFoldTanh): c = 2 log2 e
FOLD_C = 2.88539008177792681


def _rowsum(w):
    """Row sums of a [rows][cols] weight in fp64, column by column (the pack kernel's order)."""
    w = w.double()
    acc = torch.zeros(w.shape[0], dtype=torch.float64, device=w.device)
    for q in range(w.shape[1]):
        acc = acc + w[:, q]
    return acc


class PolicyPack:
    """Packs an ``MlpActorCritic``'s weights into the fragment-ordered buffer of the fused
    HIP policy kernel (layout: rl_rocket_amd/csrc/rocket_policy.inc, offsets from
    ``rr_policy_layout``). ``pack()`` is pure device tensor work on the live parameters,
    so it can sit inside a captured graph and always reflects the current weights.
    ``precision`` "fp32" (default, SB3-exact to fp32 rounding), "bf16" (tower weights
    as bf16 MFMA fragments, opt-in) or "fp16x3" (tower weights 2^8 W split into fp16
    hi / lo planes, biases 2^16 b: the split-fp16 MFMA path, fp32-level accuracy)."""

    def __init__(self, policy, obs_dim, act_dim, device, precision="fp32"):
        import ctypes

        from . import _lib

        if precision not in POLICY_PRECISIONS:
            raise ValueError("precision must be one of %s" % sorted(POLICY_PRECISIONS))
        self.precision, self.prec = precision, POLICY_PRECISIONS[precision]
        lib = _lib.load()
        off = (ctypes.c_int64 * 12)()
        size = _lib.check(lib.rr_policy_layout(obs_dim, act_dim, self.prec, off), "rr_policy_layout")
        self.off = dict(zip(("L1A", "B1", "L2A", "B2", "TOWER", "PI", "VF", "HA", "HV", "HB", "VB", "LS"), list(off)))
        self.size, self.obs_dim, self.act_dim, self.policy = size, obs_dim, act_dim, policy
        self.buf = torch.zeros(size + 4, dtype=torch.float32, device=device)  # +4: 16-B alignment slack
        if self.buf.data_ptr() % 16:
            raise RuntimeError("packed policy buffer not 16-B aligned")
        dev = device
        lane = torch.arange(64, device=dev)
        r, hh = lane & 31, lane >> 5
        reg = torch.arange(16, device=dev)

        def row(rg, h):  # D-layout row of register rg in lane half h
            return (rg & 3) + 8 * (rg >> 2) + 4 * h

        half = torch.arange(2, device=dev)
        m = torch.arange(2, device=dev)
        # B[m][half][reg] = b[32m + row(reg, half)]
        self.b_i = (32 * m[:, None, None] + row(reg[None, None, :], half[None, :, None])).reshape(-1)
        if self.prec:
            # bf16: L1A[m][s][lane][j] = W1[32m + r][16s + 8hh + j];
            # L2A[m][t][s][lane][j] = W2[32m + r][32t + 16s + 8(j>>2) + 4hh + (j&3)]
            kp1 = (obs_dim + 15) // 16
            s_ = torch.arange(kp1, device=dev)
            j = torch.arange(8, device=dev)
            shp1 = (2, kp1, 64, 8)
            self.l1_i = (32 * m.view(2, 1, 1, 1) + r.view(1, 1, 64, 1)).expand(shp1).reshape(-1)
            self.l1_k = (16 * s_.view(1, kp1, 1, 1) + 8 * hh.view(1, 1, 64, 1) + j.view(1, 1, 1, 8)).expand(shp1).reshape(-1)
            t = torch.arange(2, device=dev)
            shp2 = (2, 2, 2, 64, 8)
            self.l2_i = (32 * m.view(2, 1, 1, 1, 1) + r.view(1, 1, 1, 64, 1)).expand(shp2).reshape(-1)
            self.l2_k = (32 * t.view(1, 2, 1, 1, 1) + 16 * torch.arange(2, device=dev).view(1, 1, 2, 1, 1)
                         + 8 * (j.view(1, 1, 1, 1, 8) >> 2) + 4 * hh.view(1, 1, 1, 64, 1)
                         + (j.view(1, 1, 1, 1, 8) & 3)).expand(shp2).reshape(-1)
            self.kp1 = kp1
            return
        kp1 = (obs_dim + 1) // 2
        self.kp1 = kp1
        s_ = torch.arange(kp1, device=dev)
        # L1A[m][s][lane] = W1[32m + r][2s + hh]  (k >= obs_dim -> padded column)
        k1 = 2 * s_[None, :, None] + hh[None, None, :]
        self.l1_i = (32 * m[:, None, None] + r[None, None, :]).expand(2, kp1, 64).reshape(-1)
        self.l1_k = k1.expand(2, kp1, 64).reshape(-1)
        # L2A[m][t][g][lane][rr] = W2[32m + r][32t + row(4g + rr, hh)]
        t = torch.arange(2, device=dev)
        g = torch.arange(4, device=dev)
        rr = torch.arange(4, device=dev)
        shp = (2, 2, 4, 64, 4)
        self.l2_i = (32 * m.view(2, 1, 1, 1, 1) + r.view(1, 1, 1, 64, 1)).expand(shp).reshape(-1)
        self.l2_k = (32 * t.view(1, 2, 1, 1, 1) + row(4 * g.view(1, 1, 4, 1, 1) + rr.view(1, 1, 1, 1, 4),
                                                        hh.view(1, 1, 1, 64, 1))).expand(shp).reshape(-1)

    def _tower(self, net, base):
        o = self.off
        w1, b1, w2, b2 = net[0].weight, net[0].bias, net[2].weight, net[2].bias
        kpad = (16 if self.prec else 2) * self.kp1 - self.obs_dim
        w1p = torch.nn.functional.pad(w1, (0, kpad))  # zero columns past obs_dim
        l1, l2 = w1p[self.l1_i, self.l1_k], w2[self.l2_i, self.l2_k]
        bscale = 1.0
        if self.prec == 1:  # RNE to bf16; two bf16 per packed float, element 2q in the low half
            l1 = l1.to(torch.bfloat16).view(torch.float32)
            l2 = l2.to(torch.bfloat16).view(torch.float32)
        elif self.prec == 2:  # [hi, lo] fp16 planes of 2^8 W (RNE); biases at the 2^16 accumulator scale

            def split(w):
                w = w * 256.0
                hi = w.to(torch.float16)
                lo = (w - hi.float()).to(torch.float16)
                return torch.cat([hi.view(torch.float32), lo.view(torch.float32)])

            l1, l2, bscale = split(l1), split(l2), 65536.0
        if self.prec == 0:  # the folded fp32 tanh (rocket_policy.inc kPolFoldTanh), fp64 then one rounding
            c = FOLD_C
            self.buf[base + o["L1A"]: base + o["L1A"] + l1.numel()] = (c * l1.double()).float()
            self.buf[base + o["B1"]: base + o["B1"] + 64] = (c * b1.double()).float()[self.b_i]
            self.buf[base + o["L2A"]: base + o["L2A"] + l2.numel()] = (-2.0 * c * l2.double()).float()
            self.buf[base + o["B2"]: base + o["B2"] + 64] = (c * (b2.double() + _rowsum(w2))).float()[self.b_i]
            return
        self.buf[base + o["L1A"]: base + o["L1A"] + l1.numel()] = l1
        self.buf[base + o["B1"]: base + o["B1"] + 64] = b1[self.b_i] * bscale
        self.buf[base + o["L2A"]: base + o["L2A"] + l2.numel()] = l2
        self.buf[base + o["B2"]: base + o["B2"] + 64] = b2[self.b_i] * bscale

    def _sources(self):
        p = self.policy
        ts = [p.pi_net[0].weight, p.pi_net[0].bias, p.pi_net[2].weight, p.pi_net[2].bias,
              p.vf_net[0].weight, p.vf_net[0].bias, p.vf_net[2].weight, p.vf_net[2].bias,
              p.action_net.weight, p.action_net.bias, p.value_net.weight, p.value_net.bias, p.log_std]
        for t in ts:
            if t.dtype != torch.float32 or not t.is_contiguous() or t.device != self.buf.device:
                raise ValueError("rr_policy_pack needs contiguous fp32 parameters on the rollout device")
        return ts

    @torch.no_grad()
    def pack(self):
        """One HIP launch (rr_policy_pack) from the live parameter tensors."""
        import ctypes

        from . import _lib

        ts = self._sources()
        src = (ctypes.c_void_p * 13)(*[t.data_ptr() for t in ts])
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.buf.device).cuda_stream)
        _lib.check(_lib.load().rr_policy_pack(self.obs_dim, self.act_dim, self.prec, src,
                                              ctypes.c_void_p(self.buf.data_ptr()), stream), "rr_policy_pack")
        return self.buf

    @torch.no_grad()
    def pack_reference(self):
        """The same layout with PyTorch index ops (test reference for rr_policy_pack)."""
        p, o, na = self.policy, self.off, self.act_dim
        self._tower(p.pi_net, o["PI"])
        self._tower(p.vf_net, o["VF"])
        wa, wv = p.action_net.weight, p.value_net.weight
        if self.prec == 0:  # folded: the heads read r2 with tanh = 1 - 2 r2
            self.buf[o["HA"]: o["HA"] + 64 * na] = (-2.0 * wa[:, self.b_i]).reshape(-1)
            self.buf[o["HV"]: o["HV"] + 64] = -2.0 * wv[0, self.b_i]
            self.buf[o["HB"]: o["HB"] + na] = (p.action_net.bias.double() + _rowsum(wa)).float()
            self.buf[o["VB"]: o["VB"] + 1] = (p.value_net.bias.double() + _rowsum(wv)).float()
        else:
            self.buf[o["HA"]: o["HA"] + 64 * na] = wa[:, self.b_i].reshape(-1)
            self.buf[o["HV"]: o["HV"] + 64] = wv[0, self.b_i]
            self.buf[o["HB"]: o["HB"] + na] = p.action_net.bias
            self.buf[o["VB"]: o["VB"] + 1] = p.value_net.bias
        self.buf[o["LS"]: o["LS"] + na] = p.log_std
        return self.buf


class DeviceRollout:
    """Collects ``n_steps`` transitions from a ``RocketBatch`` (auto-reset, TimeLimit)
    into device tensors [n_steps, N, ...] and computes GAE on device.

    ``fused=True`` (default for an ``MlpActorCritic`` with 64x64 towers): per step one
    fp32-MFMA HIP launch for policy forward + sampling + buffer writes (``rr_policy_act``),
    the fused env step, one launch for the timeout bootstrap (``rr_policy_bootstrap``);
    GAE in one launch (``rr_gae``). ``fused=False``: the same algorithm in PyTorch ops.
    ``one_launch=True`` (default where possible: fused, RK4 / Euler env) collapses the whole
    ``collect`` to ONE launch (``rr_rollout_collect``: every env runs policy, sample, env step,
    bootstrap and buffer writes for all ``n_steps`` with its state in registers, then V(last
    obs) and its GAE scan); ``per_step=True`` keeps one launch per step (``rr_rollout_step``)
    + bootstrap + GAE launches. All three paths produce bitwise the same rollout.
    ``policy_dtype="fp16x3"`` (fused only) runs the towers on fp16 MFMA with every operand
    split into fp16 hi + lo halves and three MFMAs per k step: fp32-level results (values
    within ~3e-6 of the PyTorch fp32 policy, as the fp32 path) at 1.44x the collection rate.
    ``policy_dtype="bf16"`` (fused only, opt-in) runs the towers on bf16 MFMA with fp32
    accumulation: actions / values / log-probs then differ from the fp32 policy by the bf16
    rounding of obs, weights and the first hidden layer (the stored log-probs are those of
    the bf16 mean; PPO's first-epoch ratio starts within ~1e-3 of 1 instead of at 1)."""

    def __init__(self, batch, policy, n_steps=16, gamma=0.99, gae_lambda=0.95, generator=None, fused=None,
                 seed=0, policy_dtype="fp32", one_launch=None, per_step=False):
        self.env, self.policy = batch, policy
        self.n_steps, self.gamma, self.lam = n_steps, gamma, gae_lambda
        n, ns, na = batch.num_envs, batch.state_dim, batch.action_dim
        dev = batch.device
        f = dict(device=dev, dtype=torch.float32)
        self.obs = torch.zeros((n_steps, n, ns), **f)
        self.actions = torch.zeros((n_steps, n, na), **f)
        self.rewards = torch.zeros((n_steps, n), **f)
        self.starts = torch.zeros((n_steps, n), **f)   # SB3 episode_starts
        self.values = torch.zeros((n_steps, n), **f)
        self.log_probs = torch.zeros((n_steps, n), **f)
        self.advantages = torch.zeros((n_steps, n), **f)
        self.returns = torch.zeros((n_steps, n), **f)
        self.last_obs = batch.reset().clone()
        self.last_start = torch.ones((n,), **f)
        self.last_value = torch.zeros((n,), **f)
        self.last_done = torch.zeros((n,), **f)
        self.gen = generator
        self._clipped = torch.zeros((n, na), **f)
        self._tobs = torch.zeros((n, ns), **f)
        self._r = torch.zeros((n,), **f)
        if fused is None:
            fused = isinstance(policy, MlpActorCritic) and policy.hidden == (64, 64) and (ns, na) in ((14, 3), (7, 2))
        self.fused = bool(fused)
        if policy_dtype not in POLICY_PRECISIONS:
            raise ValueError("policy_dtype must be one of %s" % sorted(POLICY_PRECISIONS))
        if policy_dtype != "fp32" and not self.fused:
            raise ValueError("policy_dtype=%r needs the fused HIP policy path" % policy_dtype)
        self.policy_dtype = policy_dtype
        dopri = self.fused and int(batch.params.integrator) == 2  # RR_INT_DOPRI5: two-launch path
        if one_launch is None:
            one_launch = self.fused and not dopri
        if one_launch and (not self.fused or dopri):
            raise ValueError("one_launch needs the fused policy and an RK4 / Euler env")
        self.one_launch = bool(one_launch)
        self.per_step = bool(per_step) or not self.one_launch  # one_launch + not per_step: rr_rollout_collect
        if self.fused:
            from . import _lib

            self._lib = _lib.load()
            self._pack = PolicyPack(policy, ns, na, dev, precision=policy_dtype)
            self.iter = torch.zeros((1,), dtype=torch.int64, device=dev)  # advanced by every collect (graph-safe)
            self.seed = int(seed) & (2 ** 64 - 1)
            self._ones = torch.ones((n,), dtype=torch.uint8, device=dev)
            self._zeros = torch.zeros((n,), **f)
            import ctypes

            from .batch import _ptr

            self._c, self._p = ctypes, _ptr
            bufs = _lib.RrBuffers()
            _lib.check(self._lib.rr_get_buffers(batch._h, ctypes.byref(bufs)), "rr_get_buffers")
            self._term_obs = ctypes.c_void_p(bufs.terminal_obs)
            batch.done.fill_(1)  # SB3: _last_episode_starts = ones before the first rollout

    @torch.no_grad()
    def collect(self):
        if self.fused:
            return self._collect_fused()
        env, pol = self.env, self.policy
        for t in range(self.n_steps):
            obs = self.last_obs
            mean, value = pol(obs)
            noise = torch.randn(mean.shape, device=mean.device, generator=self.gen)
            act = mean + pol.log_std.exp() * noise
            self.obs[t].copy_(obs)
            self.actions[t].copy_(act)
            self.values[t].copy_(value)
            self.log_probs[t].copy_(pol.log_prob(mean, act))
            self.starts[t].copy_(self.last_start)
            torch.clamp(act, -1.0, 1.0, out=self._clipped)
            nobs, rew, done, trunc = env.step(self._clipped)
            # SB3 1.6: bootstrap timeouts with the value of the terminal observation
            env.copy_terminal(out=(self._tobs, None, None))
            # a select, as the fused kernels: terminal rows of envs that are not done are stale
            # (possibly non-finite), and NaN * 0 would leak into the reward
            torch.where(trunc.bool(), torch.addcmul(rew, pol.value(self._tobs), trunc.float(), value=self.gamma),
                        rew, out=self._r)
            self.rewards[t].copy_(self._r)
            self.last_obs.copy_(nobs)
            self.last_start.copy_(done.float())
        self.last_value.copy_(pol.value(self.last_obs))
        self.last_done.copy_(self.last_start)
        self._gae()

    def _collect_fused(self):
        """one_launch: the whole rollout + GAE in one rr_rollout_collect launch, or (per_step)
        one rr_rollout_step per step (the env's obs buffer is written on the last step only),
        then V(last obs). Otherwise two launches per step: rr_policy_act
        (forward + sample of step t, bootstrap of step t-1, episode-start flags) and the
        fused env step; obs are read in place from the env's output buffer."""
        env, lib, c, p = self.env, self._lib, self._c, self._p
        from . import _lib

        n, ns, na = env.num_envs, env.state_dim, env.action_dim
        params = p(self._pack.pack())
        stream = c.c_void_p(torch.cuda.current_stream(env.device).cuda_stream)
        it, obs, done = p(self.iter), p(env.obs), p(env.done)
        prec = self._pack.prec
        if self.one_launch and not self.per_step:
            _lib.check(lib.rr_rollout_collect(env._h, params, prec, self.seed, it, self.n_steps, self.gamma, self.lam,
                                              p(self.obs), p(self.actions), p(self.values), p(self.log_probs),
                                              p(self.starts), p(self.rewards), p(self.advantages), p(self.returns),
                                              p(self.last_value), p(self.last_done), p(self.last_start), obs,
                                              p(env.reward), done, p(env.truncated), p(env.terms), stream),
                       "rr_rollout_collect")
            self.iter.add_(1)
            return
        if self.one_launch:
            T = self.n_steps
            for t in range(T):
                _lib.check(lib.rr_rollout_step(env._h, params, prec, self.seed, it, t, self.gamma, p(self.obs[t]),
                                               p(self.actions[t]), p(self.values[t]), p(self.log_probs[t]),
                                               p(self.starts[t]), p(self.rewards[t]), obs if t == T - 1 else None,
                                               p(env.reward), done, p(env.truncated), p(env.terms), stream),
                           "rr_rollout_step")
            _lib.check(lib.rr_policy_bootstrap(params, ns, na, prec, n, None, None, None, self.gamma, None, obs,
                                               p(self.last_value), stream), "rr_policy_bootstrap")
            self._finish(stream)
            return
        for t in range(self.n_steps):
            prev = t > 0
            _lib.check(lib.rr_policy_act(params, ns, na, prec, n, env.env_id_offset, obs, self.seed, it, t, p(self._clipped),
                                         p(self.actions[t]), p(self.values[t]), p(self.log_probs[t]), p(self.obs[t]),
                                         self._term_obs if prev else None, p(env.truncated) if prev else None,
                                         p(env.reward) if prev else None, self.gamma,
                                         p(self.rewards[t - 1]) if prev else None, done, p(self.starts[t]), stream),
                       "rr_policy_act")
            env.step(self._clipped)
        _lib.check(lib.rr_policy_bootstrap(params, ns, na, prec, n, self._term_obs, p(env.truncated), p(env.reward),
                                           self.gamma, p(self.rewards[self.n_steps - 1]), obs, p(self.last_value),
                                           stream), "rr_policy_bootstrap")
        self._finish(stream)

    def _finish(self, stream):
        """last_done / last_start from the env's done flags, GAE (rr_gae), advance the
        noise counter."""
        from . import _lib

        env, lib, p = self.env, self._lib, self._p
        n = env.num_envs
        self.last_done.copy_(env.done)
        self.last_start.copy_(env.done)
        _lib.check(lib.rr_gae(self.n_steps, n, p(self.rewards), p(self.values), p(self.starts), p(self.last_value),
                              p(self.last_done), self.gamma, self.lam, p(self.advantages), p(self.returns), stream),
                   "rr_gae")
        self.iter.add_(1)

    def _gae(self):
        """SB3 RolloutBuffer.compute_returns_and_advantage, on device."""
        last_gae = torch.zeros_like(self.last_value)
        for t in reversed(range(self.n_steps)):
            if t == self.n_steps - 1:
                nonterminal = 1.0 - self.last_done
                next_values = self.last_value
            else:
                nonterminal = 1.0 - self.starts[t + 1]
                next_values = self.values[t + 1]
            delta = self.rewards[t] + self.gamma * next_values * nonterminal - self.values[t]
            last_gae = delta + self.gamma * self.lam * nonterminal * last_gae
            self.advantages[t].copy_(last_gae)
        torch.add(self.advantages, self.values, out=self.returns)


def _allreduce_grads(params, group):
    """Average the gradients of `params` over the ranks of `group` with ONE all_reduce of a
    flat buffer (the 64x64 MlpPolicy is ~10.6 k parameters: a single 42 KB message per
    minibatch, RCCL over xGMI with the "nccl" backend)."""
    import torch.distributed as dist

    grads = [p.grad for p in params if p.grad is not None]
    flat = torch.cat([g.reshape(-1) for g in grads])
    if flat.is_cuda and dist.get_backend(group) == "gloo":  # CPU rehearsal of the N > 1 path
        host = flat.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        flat.copy_(host)
    else:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    flat /= dist.get_world_size(group)
    k = 0
    for g in grads:
        g.copy_(flat[k:k + g.numel()].view_as(g))
        k += g.numel()


def _policy_tensors(policy):
    """The 13 parameter tensors in rr_policy_pack / rr_ppo_grad order."""
    p = policy
    return [p.pi_net[0].weight, p.pi_net[0].bias, p.pi_net[2].weight, p.pi_net[2].bias,
            p.vf_net[0].weight, p.vf_net[0].bias, p.vf_net[2].weight, p.vf_net[2].bias,
            p.action_net.weight, p.action_net.bias, p.value_net.weight, p.value_net.bias, p.log_std]


def fused_grad_supported(policy, obs_dim, act_dim):
    return (isinstance(policy, MlpActorCritic) and policy.hidden == (64, 64)
            and (obs_dim, act_dim) in ((14, 3), (7, 2)))


class PPOGrad:
    """The PPO minibatch loss + backward as ONE HIP pipeline (``rr_ppo_grad``: fp32 MFMA forward
    and backward of both towers over the gathered minibatch, fixed-order workgroup sums).

    ``__call__(idx)`` WRITES ``p.grad`` of the policy's 13 parameters (allocated here once and
    kept: the library holds their addresses, so do not set them to None — use
    ``zero_grad(set_to_none=False)`` or none at all, the call overwrites) for the minibatch
    ``idx`` (int64 device tensor of 2 .. ``batch_size`` rows of the flattened rollout) and fills
    ``stats`` = [policy_loss, value_loss, entropy, clip_fraction, approx_kl]. Same loss as
    ``ppo_update`` (SB3 1.6 PPO.train); gradients equal autograd's to fp32 rounding
    (``tests/test_gpu_ppo.py``). Stream-ordered on the current stream; graph-capturable."""

    def __init__(self, policy, ro, batch_size, clip_range=0.2, ent_coef=0.01, vf_coef=0.5):
        import ctypes

        from . import _lib

        n = ro.n_steps * ro.env.num_envs
        ns, na = ro.env.state_dim, ro.env.action_dim
        if not fused_grad_supported(policy, ns, na):
            raise ValueError("PPOGrad needs an MlpActorCritic with 64x64 towers and (obs, act) in ((14, 3), (7, 2))")
        if not 2 <= batch_size <= n:
            raise ValueError("batch_size must be in [2, n_steps * num_envs]")
        self._lib, self._c = _lib.load(), ctypes
        self.ns, self.na, self.bs = ns, na, int(batch_size)
        self.coef = (float(clip_range), float(ent_coef), float(vf_coef))
        dev = ro.obs.device
        self.data = [ro.obs.reshape(n, ns), ro.actions.reshape(n, na), ro.log_probs.reshape(n),
                     ro.advantages.reshape(n), ro.returns.reshape(n)]
        for t in self.data:
            if not t.is_contiguous() or t.dtype != torch.float32:
                raise ValueError("rollout tensors must be contiguous fp32")
        self.params = _policy_tensors(policy)
        for p in self.params:
            if p.dtype != torch.float32 or not p.is_contiguous() or p.device != dev:
                raise ValueError("rr_ppo_grad needs contiguous fp32 parameters on the rollout device")
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        nbytes = ctypes.c_int64()
        _lib.check(self._lib.rr_ppo_workspace_size(ns, na, self.bs, ctypes.byref(nbytes)), "rr_ppo_workspace_size")
        self.ws = torch.empty((nbytes.value + 15) // 16 * 4, dtype=torch.float32, device=dev)
        self.stats = torch.zeros(5, dtype=torch.float32, device=dev)
        self._src = (ctypes.c_void_p * 13)(*[p.data_ptr() for p in self.params])
        self._grads = [p.grad for p in self.params]
        self._dst = (ctypes.c_void_p * 13)(*[g.data_ptr() for g in self._grads])
        self._nbytes = nbytes.value

    def __call__(self, idx):
        from . import _lib

        c = self._c
        if (idx.dtype != torch.int64 or not 2 <= idx.numel() <= self.bs or not idx.is_contiguous()
                or idx.device != self.ws.device):
            raise ValueError("idx must be a contiguous int64 device tensor of 2 .. batch_size rows")
        for p, g in zip(self.params, self._grads):
            if p.grad is not g:
                raise RuntimeError("a parameter's .grad was replaced; PPOGrad writes into the tensors it allocated")
        clip, ent, vf = self.coef
        o, a, lp, adv, ret = self.data
        stream = c.c_void_p(torch.cuda.current_stream(self.ws.device).cuda_stream)
        _lib.check(self._lib.rr_ppo_grad(self.ns, self.na, self._src, self._dst, o.data_ptr(), a.data_ptr(),
                                         lp.data_ptr(), adv.data_ptr(), ret.data_ptr(), idx.data_ptr(), idx.numel(),
                                         clip, ent, vf, self.stats.data_ptr(), self.ws.data_ptr(), self._nbytes,
                                         stream), "rr_ppo_grad")
        return self.stats


def clip_adam_supported(optimizer, params):
    if type(optimizer) is not torch.optim.Adam or len(optimizer.param_groups) != 1:
        return False
    g = optimizer.param_groups[0]
    if {id(p) for p in g["params"]} != {id(p) for p in params} or len(params) > 16:
        return False
    return (g.get("capturable", False) and not g.get("amsgrad", False) and not g.get("maximize", False)
            and g.get("weight_decay", 0) == 0 and not torch.is_tensor(g["betas"][0])
            and all(p.dtype == torch.float32 and p.is_contiguous() and p.is_cuda for p in params))


class ClipAdam:
    """``clip_grad_norm_(params, max_grad_norm)`` + ``optimizer.step()`` for a
    ``torch.optim.Adam(capturable=True)`` in two launches (``rr_clip_adam``), on the optimizer's own
    state tensors (created here, as Adam's first step would, if absent), so the optimizer object
    stays the source of truth (state_dict, later eager steps). The learning rate is read from a
    device scalar that ``__call__`` refreshes from ``param_groups[0]["lr"]`` when called eagerly;
    inside a captured graph call ``sync_lr()`` before replays (GraphedPPOUpdate.update does)."""

    def __init__(self, optimizer, params, max_grad_norm):
        import ctypes

        from . import _lib

        if not clip_adam_supported(optimizer, params):
            raise ValueError("ClipAdam needs a capturable torch.optim.Adam over exactly these fp32 CUDA parameters "
                             "(one group, no weight decay / amsgrad / maximize, <= 16 tensors)")
        self.opt, self.params = optimizer, list(params)
        self.max_norm = float(max_grad_norm) if max_grad_norm is not None else 0.0
        dev = self.params[0].device
        for p in self.params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            st = optimizer.state[p]
            if not st:
                st["step"] = torch.zeros((), dtype=torch.float32, device=dev)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            if not st["step"].is_cuda or st["step"].dtype != torch.float32:
                raise ValueError("ClipAdam needs the capturable Adam's device float32 step tensors")
        self.lr = torch.zeros(1, dtype=torch.float32, device=dev)
        self.sync_lr()
        n = len(self.params)
        P = ctypes.c_void_p * n
        self._tensors = [(p, p.grad, optimizer.state[p]["exp_avg"], optimizer.state[p]["exp_avg_sq"],
                          optimizer.state[p]["step"]) for p in self.params]
        self._ptrs = [P(*[t[k].data_ptr() for t in self._tensors]) for k in range(5)]
        self._numel = (ctypes.c_int64 * n)(*[p.numel() for p in self.params])
        self._lib, self._c = _lib.load(), ctypes
        nbytes = ctypes.c_int64()
        _lib.check(self._lib.rr_clip_adam_workspace_size(sum(p.numel() for p in self.params), ctypes.byref(nbytes)),
                   "rr_clip_adam_workspace_size")
        self._ws = torch.empty((nbytes.value + 3) // 4, dtype=torch.float32, device=dev)
        self._nbytes = nbytes.value

    def sync_lr(self):
        self.lr.fill_(float(self.opt.param_groups[0]["lr"]))

    def __call__(self):
        from . import _lib

        for p, g, m, v, s in self._tensors:
            st = self.opt.state[p]
            if p.grad is not g or st["exp_avg"] is not m or st["exp_avg_sq"] is not v or st["step"] is not s:
                raise RuntimeError("a gradient or Adam state tensor was replaced; ClipAdam holds their addresses")
        if not torch.cuda.is_current_stream_capturing():
            self.sync_lr()
        grp = self.opt.param_groups[0]
        b1, b2 = grp["betas"]
        _lib.check(self._lib.rr_clip_adam(len(self.params), *self._ptrs, self._numel, self.max_norm,
                                          self.lr.data_ptr(), float(b1), float(b2), float(grp["eps"]),
                                          self._ws.data_ptr(), self._nbytes,
                                          self._c.c_void_p(torch.cuda.current_stream(self.lr.device).cuda_stream)),
                   "rr_clip_adam")


class PPOUpdate(PPOGrad):
    """A whole PPO minibatch step — ``PPOGrad`` then ``ClipAdam``'s clip + Adam step on the same 13
    tensors — as ONE library call (``rr_ppo_update``). Without a gradient all_reduce between the
    two halves, the clip's norm is summed by the gradient finish. The optimizer launch also repacks
    the towers for the next call and sums the next minibatch's advantage statistics. A chain of
    minibatches therefore takes three launches each instead of five; the first takes four.

    ``__call__(idx, next_idx=None, chained=False)``:
      * ``chained=True`` says that the previous call on this object was given ``next_idx=idx`` and
        that nothing else has written the parameters since.
      * The optimizer is the source of truth, as with ``ClipAdam``: its exp_avg / exp_avg_sq /
        step tensors are updated in place.
      * ``lr`` is read from a device scalar. ``sync_lr()`` refreshes it, and eager calls do so
        themselves."""

    def __init__(self, policy, optimizer, ro, batch_size, clip_range=0.2, ent_coef=0.01, vf_coef=0.5,
                 max_grad_norm=0.5):
        import ctypes

        from . import _lib

        super().__init__(policy, ro, batch_size, clip_range, ent_coef, vf_coef)
        if not clip_adam_supported(optimizer, list(policy.parameters())):
            raise ValueError("PPOUpdate needs a capturable torch.optim.Adam over the policy's parameters "
                             "(one group, no weight decay / amsgrad / maximize)")
        self.opt, self.max_norm = optimizer, float(max_grad_norm) if max_grad_norm is not None else 0.0
        dev = self.ws.device
        for p in self.params:
            st = optimizer.state[p]
            if not st:
                st["step"] = torch.zeros((), dtype=torch.float32, device=dev)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            if not st["step"].is_cuda or st["step"].dtype != torch.float32:
                raise ValueError("PPOUpdate needs the capturable Adam's device float32 step tensors")
        self._state = [(optimizer.state[p]["exp_avg"], optimizer.state[p]["exp_avg_sq"], optimizer.state[p]["step"])
                       for p in self.params]
        P = ctypes.c_void_p * 13
        self._params_w = P(*[p.data_ptr() for p in self.params])
        self._m, self._v, self._s = (P(*[st[k].data_ptr() for st in self._state]) for k in range(3))
        self.lr = torch.zeros(1, dtype=torch.float32, device=dev)
        self.sync_lr()
        nbytes = ctypes.c_int64()
        _lib.check(self._lib.rr_ppo_update_workspace_size(self.ns, self.na, self.bs, ctypes.byref(nbytes)),
                   "rr_ppo_update_workspace_size")
        self.ws = torch.empty((nbytes.value + 15) // 16 * 4, dtype=torch.float32, device=dev)
        self._nbytes = nbytes.value
        self._next = None  # (address, rows) of the last call's next_idx: what chained=True may follow

    def sync_lr(self):
        self.lr.fill_(float(self.opt.param_groups[0]["lr"]))

    def __call__(self, idx, next_idx=None, chained=False):
        from . import _lib

        c = self._c
        for t in (idx,) if next_idx is None else (idx, next_idx):
            if (t.dtype != torch.int64 or not 2 <= t.numel() <= self.bs or not t.is_contiguous()
                    or t.device != self.ws.device):
                raise ValueError("idx / next_idx must be contiguous int64 device tensors of 2 .. batch_size rows")
        if next_idx is not None and next_idx.numel() > idx.numel():
            raise ValueError("next_idx may not be longer than idx")
        if chained and self._next != (idx.data_ptr(), idx.numel()):
            raise ValueError("chained=True needs the previous call on this PPOUpdate to have had next_idx=idx")
        for p, g, (m, v, s) in zip(self.params, self._grads, self._state):
            st = self.opt.state[p]
            if p.grad is not g or st["exp_avg"] is not m or st["exp_avg_sq"] is not v or st["step"] is not s:
                raise RuntimeError("a gradient or Adam state tensor was replaced; PPOUpdate holds their addresses")
        if not torch.cuda.is_current_stream_capturing():
            self.sync_lr()
        grp = self.opt.param_groups[0]
        b1, b2 = grp["betas"]
        clip, ent, vf = self.coef
        o, a, lp, adv, ret = self.data
        nxt = None if next_idx is None else next_idx.data_ptr()
        _lib.check(self._lib.rr_ppo_update(
            self.ns, self.na, self._params_w, self._dst, self._m, self._v, self._s, o.data_ptr(), a.data_ptr(),
            lp.data_ptr(), adv.data_ptr(), ret.data_ptr(), idx.data_ptr(), idx.numel(), nxt,
            0 if next_idx is None else next_idx.numel(), clip, ent, vf, self.max_norm, self.lr.data_ptr(), float(b1),
            float(b2), float(grp["eps"]), self.stats.data_ptr(), 1 if chained else 0, self.ws.data_ptr(),
            self._nbytes, c.c_void_p(torch.cuda.current_stream(self.ws.device).cuda_stream)), "rr_ppo_update")
        self._next = None if next_idx is None else (next_idx.data_ptr(), next_idx.numel())
        return self.stats


def _epoch_perms(n, n_epochs, dev, generator=None):
    """The epochs' permutations for the fused updates, each later one drawn on a side stream
    while the caller runs the previous epoch on the current stream (torch's randperm at 1 M rows
    is a ~0.25 ms chain of small sort launches). Same draws, same order, same generator as a
    sequential loop of torch.randperm calls; each yielded tensor is ready on the current stream."""
    if n_epochs <= 0:
        return
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    nxt = torch.randperm(n, device=dev, generator=generator)
    for e in range(n_epochs):
        perm, ready = nxt, None
        if e + 1 < n_epochs:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                nxt = torch.randperm(n, device=dev, generator=generator)
                ready = side.record_event()
        yield perm
        if ready is not None:
            main.wait_event(ready)
            nxt.record_stream(main)  # drawn on the side stream, read on this one


def ppo_update(policy, optimizer, ro, n_epochs=10, batch_size=65536, clip_range=0.2, ent_coef=0.01,
               vf_coef=0.5, max_grad_norm=0.5, generator=None, group=None, fused=False):
    """SB3 1.6 PPO.train on the device-resident rollout (advantage normalisation per
    minibatch, clipped surrogate, unclipped value loss, entropy bonus, grad-norm clip).
    ent_coef 0.01 as main_6DOF.py:68.

    Multi-GPU (one policy replica per GPU): with a torch.distributed `group`
    every rank collects from its own env shard and updates on its own rollout; the
    minibatch gradients are averaged over the ranks (one all_reduce) before the grad-norm
    clip and the optimizer step, so replicas that start equal stay equal. Ranks must run
    the same number of minibatches (equal shard sizes); advantages are normalised per
    rank's minibatch.

    ``fused=True``: the loss + backward of every minibatch is ``PPOGrad`` (one HIP pipeline)
    instead of PyTorch autograd, and for a capturable Adam the clip + optimizer step is
    ``ClipAdam`` (one launch) on the optimizer's own state; the all_reduce is unchanged."""
    n = ro.n_steps * ro.env.num_envs
    if fused:
        perms = _epoch_perms(n, n_epochs, ro.obs.device, generator)
        if n % min(batch_size, n) == 1:
            # checked before the first minibatch: a 1-row remainder cannot be normalised (PPOGrad
            # refuses it) and failing there would leave the epoch's earlier Adam steps applied
            raise ValueError("n_steps * num_envs = %d leaves a 1-row last minibatch at batch_size %d (rr_ppo_grad "
                             "needs >= 2 rows); choose another batch_size" % (n, batch_size))
        params = list(policy.parameters())
        stats = None
        if group is None and clip_adam_supported(optimizer, params):
            # the whole minibatch step in one call, chained: each call sums the next one's statistics
            step = PPOUpdate(policy, optimizer, ro, min(batch_size, n), clip_range, ent_coef, vf_coef, max_grad_norm)
            for perm in perms:
                for s in range(0, n, step.bs):
                    nxt = perm[s + step.bs:s + 2 * step.bs] if s + step.bs < n else None
                    stats = step(perm[s:s + step.bs], nxt, chained=s > 0)
            return {} if stats is None else dict(zip(("policy_loss", "value_loss", "entropy"), stats[:3].tolist()))
        grad = PPOGrad(policy, ro, min(batch_size, n), clip_range, ent_coef, vf_coef)
        adam = ClipAdam(optimizer, params, max_grad_norm) if clip_adam_supported(optimizer, params) else None
        for perm in perms:
            for s in range(0, n, grad.bs):
                stats = grad(perm[s:s + grad.bs])
                if group is not None:
                    _allreduce_grads(params, group)
                if adam is not None:
                    adam()
                else:
                    torch.nn.utils.clip_grad_norm_(params, max_grad_norm)
                    optimizer.step()
        return {} if stats is None else dict(zip(("policy_loss", "value_loss", "entropy"), stats[:3].tolist()))
    obs = ro.obs.reshape(n, -1)
    act = ro.actions.reshape(n, -1)
    old_lp = ro.log_probs.reshape(n)
    adv_all = ro.advantages.reshape(n)
    ret = ro.returns.reshape(n)
    stats = {}
    for _ in range(n_epochs):
        perm = torch.randperm(n, device=obs.device, generator=generator)
        for s in range(0, n, batch_size):
            idx = perm[s:s + batch_size]
            mean, value = policy(obs[idx])
            lp = policy.log_prob(mean, act[idx])
            adv = adv_all[idx]
            adv = (adv - adv.mean()) / (adv.std() + 1e-8)
            ratio = torch.exp(lp - old_lp[idx])
            pg = -torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - clip_range, 1 + clip_range)).mean()
            vf = torch.nn.functional.mse_loss(ret[idx], value)
            ent = -policy.entropy(len(idx)).mean()
            loss = pg + ent_coef * ent + vf_coef * vf
            optimizer.zero_grad(set_to_none=True)
            loss.backward()
            if group is not None:
                _allreduce_grads(list(policy.parameters()), group)
            torch.nn.utils.clip_grad_norm_(policy.parameters(), max_grad_norm)
            optimizer.step()
            stats = {"policy_loss": pg.detach(), "value_loss": vf.detach(), "entropy": -ent.detach()}
    return {k: float(v) for k, v in stats.items()}


class GraphedPPOUpdate:
    """``ppo_update``'s minibatch step — gather, forward, clipped-surrogate / value / entropy
    loss, backward, (multi-GPU gradient all_reduce), grad-norm clip, Adam step — captured ONCE
    into a hipGraph — one graph per EPOCH: the minibatch steps of one pass over the rollout,
    each reading its rows from a static permutation buffer that ``update`` refills with
    ``torch.randperm`` before every replay (no per-minibatch index copy or graph launch).

    ``fused`` (default: wherever ``PPOGrad`` supports the policy) takes the loss + backward from
    ``PPOGrad`` (rr_ppo_grad: one fp32-MFMA HIP pipeline) instead of PyTorch autograd, whose
    tall-skinny GEMMs over the 65 536-row minibatch run far below the GPU's rate (the weight
    gradient dW = g^T x alone ~190 us per layer: profiles/r03/r03i); the gradients then
    match the eager update's to fp32 rounding instead of bitwise. ``fused=False`` captures the
    PyTorch ops themselves (bitwise the eager ``ppo_update``).

    Needs an optimizer created with ``capturable=True`` (``torch.optim.Adam(..., capturable=True)``:
    its step count lives on the device) and ``n_steps * num_envs`` divisible by ``batch_size``.
    The warm-up steps the capture requires run on the real parameters and are undone (parameters
    and optimizer state restored in place), so the first ``update`` starts from the same state
    as the eager ``ppo_update`` would, and computes the same minibatch steps (``fused=False``: same
    kernels, same order; ``tests/test_gpu_rollout.py``). Multi-GPU: ``group`` must be an RCCL ("nccl") group —
    the all_reduce is captured with the rest."""

    def __init__(self, policy, optimizer, ro, batch_size=65536, clip_range=0.2, ent_coef=0.01, vf_coef=0.5,
                 max_grad_norm=0.5, group=None, fused=None):
        if not all(g.get("capturable", False) for g in optimizer.param_groups):
            raise ValueError("GraphedPPOUpdate needs an optimizer with capturable=True")
        n = ro.n_steps * ro.env.num_envs
        if n % batch_size:
            raise ValueError("n_steps * num_envs (%d) must be a multiple of batch_size (%d)" % (n, batch_size))
        if group is not None:
            import torch.distributed as dist
            if dist.get_backend(group) != "nccl":
                raise ValueError("a captured gradient all_reduce needs the nccl (RCCL) backend")
        self.policy, self.optimizer, self.ro, self.group = policy, optimizer, ro, group
        self.n, self.bs = n, batch_size
        dev = ro.obs.device
        self.obs = ro.obs.reshape(n, -1)
        self.act = ro.actions.reshape(n, -1)
        self.old_lp = ro.log_probs.reshape(n)
        self.adv_all = ro.advantages.reshape(n)
        self.ret = ro.returns.reshape(n)
        self.coef = (clip_range, ent_coef, vf_coef, max_grad_norm)
        self.perm = torch.arange(n, device=dev)  # refilled per epoch; minibatch k = perm[k bs : (k + 1) bs]
        self._perm_bufs = self._perm_stream = None  # update(): the next epoch's permutation, drawn aside
        self._first = None  # prepare(): the event of the next update's first draw
        self.n_mb = n // batch_size
        params = list(policy.parameters())
        # state to restore after the warm-up steps (in place: the graph keeps these tensors)
        saved_p = [p.detach().clone() for p in params]
        saved_s = {id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in optimizer.state[p].items()}
                   for p in params if p in optimizer.state}
        # static gradient buffers (allocated outside the graph): the captured step copies
        # torch.autograd.grad's results into them, so no accumulation into .grad is captured. The
        # policy's Linear layers must take their bias gradient as a GEMM (_LinearFn): a column sum
        # after a GEMM in the same graph is wrong from the second replay on (profiles/r03/r03i/probe_graph_reduce.txt)
        self.params = params
        for p in params:
            p.grad = torch.zeros_like(p)
        if fused is None:
            fused = fused_grad_supported(policy, ro.env.state_dim, ro.env.action_dim)
        self.fused = bool(fused)
        # fused, one replica, capturable Adam: the chained whole-minibatch call (rr_ppo_update)
        self._update = (PPOUpdate(policy, optimizer, ro, batch_size, clip_range, ent_coef, vf_coef, max_grad_norm)
                        if self.fused and group is None and clip_adam_supported(optimizer, params) else None)
        self._grad = (PPOGrad(policy, ro, batch_size, clip_range, ent_coef, vf_coef)
                      if self.fused and self._update is None else None)
        self._adam = (ClipAdam(optimizer, params, max_grad_norm)
                      if self._grad is not None and clip_adam_supported(optimizer, params) else None)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for k in range(3):
                self._step(self._mb(k % self.n_mb), k % self.n_mb)
        torch.cuda.current_stream(dev).wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            for k in range(self.n_mb):
                self.stats = self._step(self._mb(k), k)
        with torch.no_grad():
            for p, v in zip(params, saved_p):
                p.copy_(v)
            for p in params:
                st = optimizer.state.get(p)
                if not st:
                    continue
                old = saved_s.get(id(p))
                for k, v in st.items():
                    if torch.is_tensor(v):
                        if old is not None and k in old:
                            v.copy_(old[k])
                        else:
                            v.zero_()  # state the warm-up created: back to a fresh optimizer's
        torch.cuda.synchronize(dev)

    def _mb(self, k):
        return self.perm[k * self.bs:(k + 1) * self.bs]

    def _step(self, i, k=0):
        clip_range, ent_coef, vf_coef, max_grad_norm = self.coef
        pol = self.policy
        if self._update is not None:
            st = self._update(i, self._mb(k + 1) if k + 1 < self.n_mb else None, chained=k > 0)
            return {"policy_loss": st[0], "value_loss": st[1], "entropy": st[2]}
        if self.fused:
            st = self._grad(i)
            if self.group is not None:
                _allreduce_grads(self.params, self.group)
            if self._adam is not None:
                self._adam()
            else:
                torch.nn.utils.clip_grad_norm_(self.params, max_grad_norm)
                self.optimizer.step()
            return {"policy_loss": st[0], "value_loss": st[1], "entropy": st[2]}
        mean, value = pol(self.obs[i])
        lp = pol.log_prob(mean, self.act[i])
        adv = self.adv_all[i]
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
        ratio = torch.exp(lp - self.old_lp[i])
        pg = -torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - clip_range, 1 + clip_range)).mean()
        vf = torch.nn.functional.mse_loss(self.ret[i], value)
        ent = -pol.entropy(self.bs).mean()
        loss = pg + ent_coef * ent + vf_coef * vf
        for p, g in zip(self.params, torch.autograd.grad(loss, self.params)):
            p.grad.copy_(g)
        if self.group is not None:
            _allreduce_grads(self.params, self.group)
        torch.nn.utils.clip_grad_norm_(pol.parameters(), max_grad_norm)
        self.optimizer.step()
        return {"policy_loss": pg.detach(), "value_loss": vf.detach(), "entropy": -ent.detach()}

    def _perm_streams(self):
        dev = self.obs.device
        if self._perm_bufs is None:
            self._perm_bufs = (torch.empty_like(self.perm), torch.empty_like(self.perm))
            self._perm_stream = torch.cuda.Stream(dev)
        return torch.cuda.current_stream(dev), self._perm_bufs, self._perm_stream

    def prepare(self, generator=None):
        """Draw the next ``update``'s first-epoch permutation now, on the side stream: called
        before the rollout collect, the draw runs beside it instead of ahead of the first
        epoch. It is the draw ``update`` would make first; pass ``update`` the same generator
        and draw nothing else from it in between."""
        main, bufs, side = self._perm_streams()
        side.wait_stream(main)  # the previous update's readers of bufs[0] are done
        with torch.cuda.stream(side):
            torch.randperm(self.n, out=bufs[0], generator=generator)
            self._first = side.record_event()

    def update(self, n_epochs=10, generator=None):
        """n_epochs passes over the rollout in shuffled minibatches (ppo_update's order:
        one torch.randperm per epoch).

        Each later epoch's permutation is drawn on a side stream while the previous epoch's graph
        replays: torch's randperm is a ~0.25 ms chain of small sort launches at 1 M rows, and the
        learner's kernels leave most of each SIMD's wave slots free. The draws are issued in the
        same order from the same generator, so the permutations are the sequential loop's. After
        ``prepare`` the first epoch uses the permutation drawn there."""
        for o in (self._adam, self._update):
            if o is not None:
                o.sync_lr()  # the graph reads lr from the device: follow param_groups[0]["lr"]
        main, bufs, side = self._perm_streams()
        ready, self._first = self._first, None
        if ready is None:  # no prepare(): the first epoch's draw in line
            torch.randperm(self.n, out=bufs[0], generator=generator)
        for e in range(n_epochs):
            cur = bufs[e % 2]
            if ready is not None:
                main.wait_event(ready)
            self.perm.copy_(cur)
            if e + 1 < n_epochs:
                side.wait_stream(main)  # the other buffer's last reader (the previous copy) is done
                with torch.cuda.stream(side):
                    torch.randperm(self.n, out=bufs[(e + 1) % 2], generator=generator)
                    ready = side.record_event()
            self.graph.replay()
        return {k: float(v) for k, v in self.stats.items()}
