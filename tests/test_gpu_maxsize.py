"""The largest batch one env handle takes (rr_create: n * (state_dim + 3) * 4 bytes must fit the
kernels' 32-bit buffer offsets, so 63 161 283 6DOF / 107 374 182 3DOF envs): one step at that N,
fast (RK4) and exact (DOPRI5), with ground-event rows at the head and the tail of the batch. Every
sampled row (head, tail, spread) is bitwise the same row stepped in a small batch, the done list
names exactly the done envs (indices past 2^26), and the sampled rows agree with the CPU oracle at
the mode's tolerance (fast: the north star's 1e-5; exact: 1e-8, as test_gpu_exact.py)."""
import numpy as np
import pytest

from gpu_util import TOL_STATE, floored_rel

pytestmark = pytest.mark.gpu


def _max_n(ns):
    return 0xFFFFFFFF // ((ns + 3) * 4)


@pytest.mark.parametrize("model,integrator", [(6, "rk4"), (6, "dopri5"), (3, "rk4"), (3, "dopri5")])
def test_maximum_batch_step(model, integrator, oracle_mod):
    import torch

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF

    ns, na = (14, 3) if model == 6 else (7, 2)
    n = _max_n(ns)
    kw = dict(model=model, device="cuda:0", max_episode_steps=0, auto_reset=False, compute_terms=True,
              integrator=integrator, **(ENV_CONFIG_6DOF if model == 6 else {}))
    exact = integrator == "dopri5"
    rng = np.random.default_rng(model)
    sel = np.unique(np.concatenate([np.arange(256), rng.integers(0, n, 1024), np.arange(n - 2048, n)]))
    ev = np.concatenate([np.arange(0, 32), np.arange(n - 2000, n, 40)])  # ground-event rows, all in sel
    alt, vel = (0, 3) if model == 6 else (1, 4)

    b = RocketBatch(n, **kw)
    b.reset()
    st, v0, _ = b.get_state64() if exact else b.get_state()
    evd = torch.from_numpy(ev).to("cuda:0")
    st[alt, evd] = 0.5
    st[vel, evd] = -20.0
    (b.set_state64 if exact else b.set_state)(st, v0=v0)
    gen = torch.Generator(device="cuda:0").manual_seed(3)
    a = torch.rand((n, na), device="cuda:0", generator=gen) * 2 - 1
    obs, rew, done, _ = b.step(a)
    idx, _, _, _ = b.fetch_done()
    seld = torch.from_numpy(sel).to("cuda:0")
    big = dict(obs=obs[seld].cpu(), rew=rew[seld].cpu(), done=done[seld].cpu(), terms=b.terms[:, seld].cpu(),
               st=(b.get_state64() if exact else b.get_state())[0][:, seld].cpu())
    d_all = done.cpu().numpy().astype(bool)
    st_in, v0_in, a_in = st[:, seld].cpu(), v0[seld].cpu(), a[seld].cpu()
    del st, v0, a, obs, rew, done, seld, evd
    b.close()
    torch.cuda.empty_cache()

    assert np.array_equal(np.sort(idx), np.flatnonzero(d_all))
    assert d_all[ev].all() and idx.max() > n - 100

    m = len(sel)
    s = RocketBatch(m, **kw)
    (s.set_state64 if exact else s.set_state)(st_in, v0=v0_in)
    o2, r2, d2, _ = s.step(a_in.to("cuda:0"))
    small = dict(obs=o2.cpu(), rew=r2.cpu(), done=d2.cpu(), terms=s.terms.cpu(),
                 st=(s.get_state64() if exact else s.get_state())[0].cpu())
    s.close()
    for k in small:
        assert torch.equal(big[k], small[k]), k

    # the sampled rows against the CPU oracle; ic rows carry v0 as their first velocity component
    # (sqrt(v0 * v0) == v0 in IEEE fp32)
    ic = np.zeros((m, ns), np.float32)
    ic[:, 3] = v0_in.numpy()
    cfg = oracle_mod.make_cfg(model, **(oracle_mod.ENV_CONFIG_6DOF if model == 6 else oracle_mod.DEFAULTS_3DOF))
    s_in = st_in.numpy().T.astype(np.float64)
    ref = oracle_mod.step(cfg, ic, 0.0, s_in, a_in.numpy(), nthreads=8)
    e = floored_rel(small["st"].numpy().T, ref["state_out"], np.array(cfg.normalizer[:ns])).max()
    print("N = %d %s: %d sampled rows, %d done (%d listed), oracle state err %.3g"
          % (n, integrator, m, d_all.sum(), len(idx), e))
    assert e < (1e-8 if exact else TOL_STATE)
    assert np.array_equal(small["done"].numpy().astype(bool), ref["done"].astype(bool))


def test_maximum_batch_rollout_collect():
    """configs[4]'s on-device collect at the largest 6DOF batch, n_steps 2 and TimeLimit 1 (every
    env truncates and auto-resets inside the rollout, so the timeout bootstrap's value tower runs in
    every wave): the one-launch collect (rr_rollout_collect) is bitwise the per-step kernels
    (rr_rollout_step) on every buffer and on the env state, and the values of sampled rows, head and
    tail, match the fp32 PyTorch policy on their stored obs (the rollout tests' tolerance)."""
    import torch

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF
    from rl_rocket_amd.rollout import DeviceRollout
    from test_gpu_rollout import TOL, _policy

    n, T = _max_n(14), 2
    pol = _policy(14, 3, seed=5)
    ros = []
    for per_step in (False, True):
        env = RocketBatch(n, model=6, device="cuda:0", max_episode_steps=1, **ENV_CONFIG_6DOF)
        ros.append(DeviceRollout(env, pol, n_steps=T, policy_dtype="fp32", one_launch=True, per_step=per_step,
                                 seed=23))
    for ro in ros:
        ro.collect()
    torch.cuda.synchronize()
    a, b = ros
    for name in ("obs", "actions", "values", "log_probs", "starts", "rewards", "advantages", "returns",
                 "last_value", "last_done"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    for x, y in zip(a.env.get_state(), b.env.get_state()):
        assert torch.equal(x, y)
    assert bool(a.starts[1].all())  # TimeLimit 1: every env restarted at step 1
    sel = torch.cat([torch.arange(4096), torch.arange(n - 4096, n)]).to("cuda:0")
    with torch.no_grad():
        _, value = pol(a.obs[:, sel].reshape(-1, 14))
    assert (a.values[:, sel].reshape(-1) - value).abs().max().item() < TOL
    assert torch.isfinite(a.advantages).all()
    for ro in ros:
        ro.env.close()
