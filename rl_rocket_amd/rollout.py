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


class MlpActorCritic(nn.Module):
    def __init__(self, obs_dim, act_dim, hidden=(64, 64), log_std_init=0.0):
        super().__init__()

        def mlp():
            layers, d = [], obs_dim
            for h in hidden:
                layers += [nn.Linear(d, h), nn.Tanh()]
                d = h
            return nn.Sequential(*layers)

        self.pi_net, self.vf_net = mlp(), mlp()
        self.action_net = nn.Linear(hidden[-1], act_dim)
        self.value_net = nn.Linear(hidden[-1], 1)
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


class DeviceRollout:
    """Collects ``n_steps`` transitions from a ``RocketBatch`` (auto-reset, TimeLimit)
    into device tensors [n_steps, N, ...] and computes GAE on device."""

    def __init__(self, batch, policy, n_steps=16, gamma=0.99, gae_lambda=0.95, generator=None):
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

    @torch.no_grad()
    def collect(self):
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
            torch.addcmul(rew, pol.value(self._tobs), trunc.float(), value=self.gamma, out=self._r)
            self.rewards[t].copy_(self._r)
            self.last_obs.copy_(nobs)
            self.last_start.copy_(done.float())
        self.last_value.copy_(pol.value(self.last_obs))
        self.last_done.copy_(self.last_start)
        self._gae()

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


def ppo_update(policy, optimizer, ro, n_epochs=10, batch_size=65536, clip_range=0.2, ent_coef=0.01,
               vf_coef=0.5, max_grad_norm=0.5, generator=None):
    """SB3 1.6 PPO.train on the device-resident rollout (advantage normalisation per
    minibatch, clipped surrogate, unclipped value loss, entropy bonus, grad-norm clip).
    ent_coef 0.01 as main_6DOF.py:114."""
    n = ro.n_steps * ro.env.num_envs
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
            torch.nn.utils.clip_grad_norm_(policy.parameters(), max_grad_norm)
            optimizer.step()
            stats = {"policy_loss": pg.detach(), "value_loss": vf.detach(), "entropy": -ent.detach()}
    return {k: float(v) for k, v in stats.items()}
