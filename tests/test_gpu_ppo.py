"""rr_ppo_grad (rl_rocket_amd/csrc/rocket_ppo.inc, PPOGrad): the PPO minibatch loss + backward of
the MlpPolicy on fp32 MFMA, against PyTorch autograd of the same loss (rollout.ppo_update's,
SB3 1.6 PPO.train) evaluated in float64 on the same parameters and minibatch.

Tolerance: per gradient tensor, max |fused - fp64| <= 1e-4 * max |fp64| + 1e-7 (fp32 sums over
up to 65 536 samples in another order, tanh via exp2 / rcp: the PyTorch fp32 autograd of the same
loss lands at the same level, printed beside it). Stats (policy_loss, value_loss, entropy,
clip_fraction, approx_kl) within 1e-5 relative + 1e-6 (clip_fraction: within 2 samples)."""
import copy
import types

import pytest

pytestmark = pytest.mark.gpu


def _setup(ns, na, n, seed=0):
    import torch
    from rl_rocket_amd.rollout import MlpActorCritic

    g = torch.Generator("cuda:0").manual_seed(seed)
    torch.manual_seed(seed)
    pol = MlpActorCritic(ns, na).cuda()
    with torch.no_grad():  # off SB3's small-gain init so every weight and bias matters
        for p in pol.parameters():
            p.add_(0.2 * torch.randn(p.shape, device="cuda:0", generator=g))
    f = dict(device="cuda:0", dtype=torch.float32)
    obs = 0.7 * torch.randn((n, ns), generator=g, **f)
    act = torch.randn((n, na), generator=g, **f)
    with torch.no_grad():
        mean, _ = pol(obs)
        old_lp = pol.log_prob(mean, act) + 0.25 * torch.randn((n,), generator=g, **f)  # ratios on both sides of the clip
    adv = 2.0 * torch.randn((n,), generator=g, **f) + 0.3
    ret = 5.0 * torch.randn((n,), generator=g, **f)
    ro = types.SimpleNamespace(n_steps=1, env=types.SimpleNamespace(num_envs=n, state_dim=ns, action_dim=na),
                               obs=obs.view(1, n, ns), actions=act.view(1, n, na), log_probs=old_lp.view(1, n),
                               advantages=adv.view(1, n), returns=ret.view(1, n))
    return pol, ro, g


def _reference(pol, ro, idx, dtype, clip=0.2, ent_coef=0.01, vf_coef=0.5):
    """ppo_update's loss for one minibatch (autograd) in `dtype`."""
    import torch
    from rl_rocket_amd.rollout import _policy_tensors

    p = copy.deepcopy(pol).to(dtype)
    n = ro.env.num_envs
    obs = ro.obs.reshape(n, -1)[idx].to(dtype)
    act = ro.actions.reshape(n, -1)[idx].to(dtype)
    old = ro.log_probs.reshape(n)[idx].to(dtype)
    adv = ro.advantages.reshape(n)[idx].to(dtype)
    ret = ro.returns.reshape(n)[idx].to(dtype)
    mean, value = p(obs)
    lp = p.log_prob(mean, act)
    adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    ratio = torch.exp(lp - old)
    pg = -torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
    vf = torch.nn.functional.mse_loss(ret, value)
    ent = -p.entropy(len(idx)).mean()
    (pg + ent_coef * ent + vf_coef * vf).backward()
    with torch.no_grad():
        lr = lp - old
        stats = [pg.item(), vf.item(), -ent.item(), ((ratio - 1).abs() > clip).double().mean().item(),
                 ((torch.exp(lr) - 1) - lr).mean().item()]
    return [t.grad.double() for t in _policy_tensors(p)], stats


NAMES = ["pi.W1", "pi.b1", "pi.W2", "pi.b2", "vf.W1", "vf.b1", "vf.W2", "vf.b2", "W_action", "b_action",
         "W_value", "b_value", "log_std"]


@pytest.mark.parametrize("ns,na", [(14, 3), (7, 2)])
@pytest.mark.parametrize("bs", [65536, 1000, 2])
def test_ppo_grad_matches_autograd(ns, na, bs):
    import torch
    from rl_rocket_amd.rollout import PPOGrad, _policy_tensors

    n = 70000
    pol, ro, g = _setup(ns, na, n, seed=ns + bs)
    idx = torch.randperm(n, device="cuda:0", generator=g)[:bs].contiguous()
    grad = PPOGrad(pol, ro, bs)
    stats = grad(idx).tolist()
    torch.cuda.synchronize()
    fused = [t.grad.double() for t in _policy_tensors(pol)]
    ref64, st64 = _reference(pol, ro, idx, torch.float64)
    ref32, _ = _reference(pol, ro, idx, torch.float32)
    for name, a, r, t in zip(NAMES, fused, ref64, ref32):
        scale = r.abs().max().item()
        err, err32 = (a - r).abs().max().item(), (t - r).abs().max().item()
        print("%-9s max|ref| %.3e  fused err %.2e  torch-fp32 err %.2e" % (name, scale, err, err32))
        assert err <= 1e-4 * scale + 1e-7, (name, err, scale, err32)
    for k, (a, r) in enumerate(zip(stats, st64)):
        tol = 2.0 / bs if k == 3 else 1e-5 * abs(r) + 1e-6
        assert abs(a - r) <= tol, (k, a, r)


def test_ppo_grad_overwrites_and_is_deterministic():
    """Two calls on the same minibatch give bitwise the same gradients (fixed-order sums), written
    over whatever the .grad tensors held."""
    import torch
    from rl_rocket_amd.rollout import PPOGrad, _policy_tensors

    n = 20000
    pol, ro, g = _setup(14, 3, n, seed=3)
    idx = torch.randperm(n, device="cuda:0", generator=g)[:8192].contiguous()
    grad = PPOGrad(pol, ro, 8192)
    grad(idx)
    first = [t.grad.clone() for t in _policy_tensors(pol)]
    for t in _policy_tensors(pol):
        t.grad.fill_(123.0)
    grad(idx)
    for a, t in zip(first, _policy_tensors(pol)):
        assert torch.equal(a, t.grad)


def test_epoch_perms_are_the_sequential_draws():
    """ppo_update(fused=True)'s permutations, each later epoch's drawn on a side stream: the same
    tensors as a sequential loop of torch.randperm on the same generator, each one ready on the
    caller's stream when it is yielded (a slow consumer in between changes nothing)."""
    import torch
    from rl_rocket_amd.rollout import _epoch_perms

    n = 1 << 17
    seen = []
    x = torch.randn(4096, 4096, device="cuda:0")
    for p in _epoch_perms(n, 4, torch.device("cuda:0"), torch.Generator("cuda:0").manual_seed(21)):
        x = x @ x.T * 1e-3  # keep the current stream busy while the next draw runs aside
        seen.append(p.clone())
    gen = torch.Generator("cuda:0").manual_seed(21)
    want = [torch.randperm(n, device="cuda:0", generator=gen) for _ in range(4)]
    torch.cuda.synchronize()
    assert len(seen) == 4
    for e, (a, b) in enumerate(zip(seen, want)):
        assert torch.equal(a, b), e
    assert list(_epoch_perms(n, 0, torch.device("cuda:0"))) == []


@pytest.mark.parametrize("prepared", [False, True])
def test_graphed_update_draws_the_sequential_permutations(prepared):
    """GraphedPPOUpdate.update draws each later epoch's permutation on a side stream while the
    previous epoch replays (and, after prepare(), the first one before the update): every epoch
    still sees exactly the permutation a sequential loop of torch.randperm calls on the same
    generator gives (n = 65 536: torch's on-device sort path)."""
    import torch
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF
    from rl_rocket_amd.rollout import DeviceRollout, GraphedPPOUpdate, MlpActorCritic

    n, T, bs = 8192, 8, 16384
    env = RocketBatch(n, model=6, device="cuda:0", max_episode_steps=30, **ENV_CONFIG_6DOF)
    torch.manual_seed(12)
    pol = MlpActorCritic(14, 3).cuda()
    ro = DeviceRollout(env, pol, n_steps=T, seed=4)
    ro.collect()
    opt = torch.optim.Adam(pol.parameters(), lr=1e-3, capturable=True)
    g = GraphedPPOUpdate(pol, opt, ro, batch_size=bs, fused=True)
    seen = []

    class _Record:  # stands in for the epoch's graph: what the replay would read
        def replay(self):
            seen.append(g.perm.clone())

    g.graph = _Record()
    gen0 = torch.Generator("cuda:0").manual_seed(13)
    if prepared:
        g.prepare(gen0)
        ro.collect()  # what prepare() is for: the draw runs beside the collect
    g.update(n_epochs=5, generator=gen0)
    gen = torch.Generator("cuda:0").manual_seed(13)
    want = [torch.randperm(n * T, device="cuda:0", generator=gen) for _ in range(5)]
    torch.cuda.synchronize()
    assert len(seen) == 5
    for e, (a, b) in enumerate(zip(seen, want)):
        assert torch.equal(a, b), e
    assert len({tuple(a[:8].tolist()) for a in seen}) == 5  # five different draws
    env.close()


def test_fused_update_graphed_equals_eager_and_tracks_autograd():
    """ppo_update(fused=True) and GraphedPPOUpdate(fused=True) from the same state and shuffling:
    bitwise equal (same launches in the same order); and against the PyTorch-autograd ppo_update,
    with Adam(eps=1.0) so that parameter steps are proportional to the gradients (not their
    signs): within 1e-6 after two epochs."""
    import torch
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF
    from rl_rocket_amd.rollout import DeviceRollout, GraphedPPOUpdate, MlpActorCritic, ppo_update

    n, T, bs = 8192, 8, 16384
    env = RocketBatch(n, model=6, device="cuda:0", max_episode_steps=30, **ENV_CONFIG_6DOF)
    torch.manual_seed(11)
    pol = MlpActorCritic(14, 3).cuda()
    ro = DeviceRollout(env, pol, n_steps=T, seed=4)
    ro.collect()
    torch.cuda.synchronize()
    pols = [copy.deepcopy(pol) for _ in range(3)]
    opts = [torch.optim.Adam(p.parameters(), lr=1e-3, eps=1.0, capturable=True) for p in pols]
    g = GraphedPPOUpdate(pols[2], opts[2], ro, batch_size=bs, fused=True)
    assert g.fused
    gen = lambda: torch.Generator("cuda:0").manual_seed(9)  # noqa: E731
    sa = ppo_update(pols[0], opts[0], ro, n_epochs=2, batch_size=bs, generator=gen())
    sb = ppo_update(pols[1], opts[1], ro, n_epochs=2, batch_size=bs, generator=gen(), fused=True)
    sc = g.update(n_epochs=2, generator=gen())
    torch.cuda.synchronize()
    for x, y in zip(pols[1].parameters(), pols[2].parameters()):
        assert torch.equal(x, y)
    moved = max((x - y).abs().max().item() for x, y in zip(pol.parameters(), pols[1].parameters()))
    worst = max((x - y).abs().max().item() for x, y in zip(pols[0].parameters(), pols[1].parameters()))
    print("moved %.3e, fused vs autograd %.3e" % (moved, worst))
    assert moved > 1e-5
    assert worst <= 1e-6, worst
    for k in sa:
        assert abs(sa[k] - sb[k]) <= 1e-4 * max(1.0, abs(sa[k])), (k, sa[k], sb[k])
        assert abs(sb[k] - sc[k]) <= 1e-6 * max(1.0, abs(sb[k])), (k, sb[k], sc[k])
    env.close()


def test_ppo_grad_rejects_bad_arguments():
    import torch
    from rl_rocket_amd.rollout import PPOGrad

    pol, ro, g = _setup(14, 3, 1000, seed=1)
    grad = PPOGrad(pol, ro, 512)
    with pytest.raises(ValueError):
        grad(torch.arange(513, device="cuda:0"))  # more rows than the workspace was sized for
    with pytest.raises(ValueError):
        grad(torch.arange(1, device="cuda:0"))  # a 1-sample minibatch has no std
    with pytest.raises(ValueError):
        grad(torch.arange(512, device="cuda:0", dtype=torch.int32))
    pol.pi_net[0].bias.grad = None
    with pytest.raises(RuntimeError):
        grad(torch.arange(512, device="cuda:0"))
    with pytest.raises(ValueError):
        PPOGrad(pol, ro, 1)


def test_clip_adam_matches_torch():
    """rr_clip_adam (ClipAdam) against clip_grad_norm_ + torch.optim.Adam(capturable=True) on the
    same gradients for 6 steps (clip active on the first 3, a learning-rate change after 3):
    parameters, clipped gradients and the optimizer's exp_avg / exp_avg_sq / step within fp32
    rounding."""
    import torch
    from rl_rocket_amd.rollout import ClipAdam, MlpActorCritic

    torch.manual_seed(5)
    pa = MlpActorCritic(14, 3).cuda()
    pb = copy.deepcopy(pa)
    oa = torch.optim.Adam(pa.parameters(), lr=3e-4, eps=1e-5, capturable=True)
    ob = torch.optim.Adam(pb.parameters(), lr=3e-4, eps=1e-5, capturable=True)
    adam = ClipAdam(ob, list(pb.parameters()), 0.5)
    g = torch.Generator("cuda:0").manual_seed(2)
    for step in range(6):
        if step == 3:
            for o in (oa, ob):
                o.param_groups[0]["lr"] = 1e-4
        scale = 1.0 if step < 3 else 1e-3
        for x, y in zip(pa.parameters(), pb.parameters()):
            gr = scale * torch.randn(x.shape, device="cuda:0", generator=g)
            x.grad = gr.clone()
            y.grad.copy_(gr)
        torch.nn.utils.clip_grad_norm_(list(pa.parameters()), 0.5)
        oa.step()
        adam()
        torch.cuda.synchronize()
        for x, y in zip(pa.parameters(), pb.parameters()):
            sa, sb = oa.state[x], ob.state[y]
            assert float(sa["step"]) == float(sb["step"]) == step + 1
            assert (x - y).abs().max().item() <= 1e-6 * max(1.0, x.abs().max().item())
            assert torch.allclose(x.grad, y.grad, rtol=1e-5, atol=1e-9)
            assert torch.allclose(sa["exp_avg"], sb["exp_avg"], rtol=1e-5, atol=1e-9)
            assert torch.allclose(sa["exp_avg_sq"], sb["exp_avg_sq"], rtol=1e-5, atol=1e-12)


def _rollout_for_update(n=8192, T=8, seed=4, model=6):
    import torch
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF
    from rl_rocket_amd.rollout import DeviceRollout, MlpActorCritic

    env = RocketBatch(n, model=model, device="cuda:0", max_episode_steps=30, **(ENV_CONFIG_6DOF if model == 6 else {}))
    torch.manual_seed(11)
    pol = MlpActorCritic(env.state_dim, env.action_dim).cuda()
    ro = DeviceRollout(env, pol, n_steps=T, seed=seed)
    ro.collect()
    torch.cuda.synchronize()
    return env, pol, ro


def test_fused_update_with_the_shipped_adam_tracks_autograd():
    """The shipped optimizer setting (Adam lr 3e-4, eps 1e-5: bench.py, SB3's defaults) over 3
    epochs x 4 minibatches, fused (rr_ppo_grad + rr_clip_adam, graphed) against the PyTorch-autograd
    ppo_update from the same state and shuffling. With eps = 1e-5 an Adam step is ~lr * sign(g)
    while |g| >> eps, so a gradient element near 0 whose fp32 rounding differs between the two
    paths can step the other way: the bar is on the whole update, not bitwise. Parameters within
    5 % of how far the update moved them, the policy's means / values on the rollout's obs within
    2e-3 (absolute; they are O(0.1-10)), the last minibatch's loss statistics within 2 %."""
    import torch
    from rl_rocket_amd.rollout import GraphedPPOUpdate, ppo_update

    env, pol, ro = _rollout_for_update()
    bs = 16384
    pols = [copy.deepcopy(pol) for _ in range(2)]
    opts = [torch.optim.Adam(p.parameters(), lr=3e-4, eps=1e-5, capturable=True) for p in pols]
    gen = lambda: torch.Generator("cuda:0").manual_seed(21)  # noqa: E731
    sa = ppo_update(pols[0], opts[0], ro, n_epochs=3, batch_size=bs, generator=gen())
    g = GraphedPPOUpdate(pols[1], opts[1], ro, batch_size=bs, fused=True)
    sb = g.update(n_epochs=3, generator=gen())
    torch.cuda.synchronize()
    moved = max((x - y).abs().max().item() for x, y in zip(pol.parameters(), pols[0].parameters()))
    drift = max((x - y).abs().max().item() for x, y in zip(pols[0].parameters(), pols[1].parameters()))
    obs = ro.obs.reshape(-1, 14)[:20000]
    with torch.no_grad():
        (ma, va), (mb, vb) = pols[0](obs), pols[1](obs)
    out = max((ma - mb).abs().max().item(), (va - vb).abs().max().item())
    print("moved %.3e, parameter drift %.3e, output drift %.3e" % (moved, drift, out), sa, sb)
    assert moved > 1e-3
    assert drift <= 0.05 * moved, (drift, moved)
    assert out <= 2e-3, out
    for k in sa:
        assert abs(sa[k] - sb[k]) <= 0.02 * max(1.0, abs(sa[k])), (k, sa[k], sb[k])
    env.close()


def test_fused_update_refuses_a_one_row_remainder_before_stepping():
    """ppo_update(fused=True) with n_steps * num_envs % batch_size == 1 raises before the first
    minibatch (the policy and optimizer are untouched); a remainder of >= 2 rows is a valid last
    minibatch."""
    import torch
    from rl_rocket_amd.rollout import ppo_update

    env, pol, ro = _rollout_for_update(n=1000, T=8)  # 8000 rows
    opt = torch.optim.Adam(pol.parameters(), lr=3e-4, eps=1e-5, capturable=True)
    before = [p.detach().clone() for p in pol.parameters()]
    with pytest.raises(ValueError):
        ppo_update(pol, opt, ro, n_epochs=1, batch_size=7999, fused=True)
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(before, pol.parameters()))
    assert not opt.state  # no Adam step ran
    stats = ppo_update(pol, opt, ro, n_epochs=1, batch_size=3999, fused=True)  # 2-row remainder
    torch.cuda.synchronize()
    assert all(abs(v) < 1e9 for v in stats.values())
    assert any(not torch.equal(a, b) for a, b in zip(before, pol.parameters()))
    env.close()


def test_rollout_and_learner_forwards_agree():
    """The fp32 rollout runs the tanh FOLDED into its packed weights (rocket_policy.inc kPolFoldTanh,
    include/rocket_hip.h RR_POLICY_FP32); the learner (rr_ppo_grad) packs and runs the unfolded
    tanh. On the same parameters and the rollout's own samples the two forwards agree to rounding,
    not bit for bit: with old_log_prob = the rollout's log_prob and returns = the rollout's values,
    rr_ppo_grad's approx_kl (mean (r - 1) - log r) is ~0, no ratio is clipped, and its value loss
    (the mean squared gap between the two value forwards) is ~0. Bars: approx_kl <= 1e-9 (a log-prob
    gap of ~4e-5), rms value gap <= 1e-5 x (1 + rms value)."""
    import torch
    from rl_rocket_amd.rollout import PPOGrad

    env, pol, ro = _rollout_for_update(n=8192, T=8, seed=9)
    n = ro.n_steps * env.num_envs
    ro_cmp = types.SimpleNamespace(n_steps=ro.n_steps, env=ro.env, obs=ro.obs, actions=ro.actions,
                                   log_probs=ro.log_probs, advantages=ro.advantages, returns=ro.values.clone())
    grad = PPOGrad(pol, ro_cmp, n)
    idx = torch.arange(n, device="cuda:0", dtype=torch.int64)
    pl, vl, ent, clip_frac, approx_kl = grad(idx).tolist()
    torch.cuda.synchronize()
    rms_v = ro.values.double().pow(2).mean().sqrt().item()
    print("approx_kl %.3e clip_fraction %.3g rms value gap %.3e (rms value %.3f)" % (approx_kl, clip_frac, vl ** 0.5,
                                                                                 rms_v))
    assert clip_frac == 0.0
    assert abs(approx_kl) <= 1e-9
    assert vl ** 0.5 <= 1e-5 * (1.0 + rms_v)
    env.close()


@pytest.mark.parametrize("model", [6, 3])
def test_ppo_update_chain_carries_what_a_fresh_prep_computes(model):
    """rr_ppo_update chained (each call's optimizer launch repacks the towers from the updated
    parameters — the inverse of the pack — and sums the next minibatch's advantage statistics)
    against the same calls each packing and summing for itself: after 2 epochs x 4 minibatches
    (the last one 2 rows short, a shorter next_batch) every parameter, gradient and Adam state
    tensor is bitwise equal. Both paths also stay within fp32 rounding of PPOGrad + ClipAdam (the
    clip's norm is summed in another order)."""
    import torch
    from rl_rocket_amd.rollout import ClipAdam, PPOGrad, PPOUpdate

    env, pol, ro = _rollout_for_update(model=model)
    n = ro.n_steps * ro.env.num_envs
    bs = 16384
    pols = [copy.deepcopy(pol) for _ in range(3)]
    opts = [torch.optim.Adam(p.parameters(), lr=1e-3, eps=1.0, capturable=True) for p in pols]
    upd = [PPOUpdate(pols[k], opts[k], ro, bs) for k in range(2)]
    grad, adam = PPOGrad(pols[2], ro, bs), ClipAdam(opts[2], list(pols[2].parameters()), 0.5)
    g = torch.Generator("cuda:0").manual_seed(5)
    for _ in range(2):
        perm = torch.randperm(n, device="cuda:0", generator=g)[:4 * bs - 2]
        mbs = [perm[s:s + bs] for s in range(0, len(perm), bs)]
        for k, idx in enumerate(mbs):
            nxt = mbs[k + 1] if k + 1 < len(mbs) else None
            upd[0](idx, nxt, chained=k > 0)
            upd[1](idx)
            grad(idx)
            adam()
    torch.cuda.synchronize()
    for x, y, z in zip(*[list(p.parameters()) for p in pols]):
        assert torch.equal(x, y)
        assert torch.equal(x.grad, y.grad)
        assert torch.equal(opts[0].state[x]["exp_avg"], opts[1].state[y]["exp_avg"])
        assert torch.equal(opts[0].state[x]["exp_avg_sq"], opts[1].state[y]["exp_avg_sq"])
        assert float(opts[0].state[x]["step"]) == float(opts[2].state[z]["step"]) == 8
        assert (x - z).abs().max().item() <= 1e-6 * max(1.0, z.abs().max().item())
    with pytest.raises(ValueError):
        upd[0](mbs[0][:bs - 2], mbs[1])  # next_idx longer than idx
    with pytest.raises(ValueError):
        upd[0](mbs[1], chained=True)  # the last call handed over no next minibatch
    env.close()
