"""The fused on-device rollout kernels (rl_rocket_amd/csrc/rocket_policy.inc) against the
PyTorch restatement of SB3's MlpPolicy / collect_rollouts / GAE (rl_rocket_amd/rollout.py),
fp32. Tolerances: 2e-5 absolute on policy outputs of O(1) (MFMA fp32 fma chains in another
order, tanh via exp2/rcp), 1e-5 on GAE.

The opt-in bf16 policy (RR_POLICY_BF16) is checked against a PyTorch emulation of the same
roundings (obs, tower weights and the first hidden layer RNE to bf16, fp32 elsewhere): 99 %
of envs within 1e-4 and all within 1e-2 (an fp32-level difference can move one hidden unit
across a bf16 rounding boundary: one bf16 ulp, <= 4e-3 relative, times an O(1) weight)."""
import ctypes
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 2e-5
PREC = {"fp32": 0, "bf16": 1, "fp16x3": 2}
EXACTISH = ("fp32", "fp16x3")  # checked against the fp32 PyTorch policy itself


def _bf(t):
    import torch

    return t.to(torch.bfloat16).float()


def _emulated_bf16(pol, obs):
    """(mean, value) of the policy with the bf16 kernel's roundings."""
    import torch

    def tower(net):
        h1 = torch.tanh(_bf(obs) @ _bf(net[0].weight).T + net[0].bias)
        return torch.tanh(_bf(h1) @ _bf(net[2].weight).T + net[2].bias)

    with torch.no_grad():
        return pol.action_net(tower(pol.pi_net)), pol.value_net(tower(pol.vf_net)).squeeze(-1)


def _check_close(got, ref, tag):
    err = (got - ref).abs().flatten()
    q99 = err.quantile(0.99).item() if err.numel() <= 2 ** 24 else err.max().item()
    print(tag, "max err", err.max().item(), "q99", q99)
    assert err.max().item() < 1e-2 and q99 < 1e-4


def _policy(ns, na, seed=0):
    import torch
    from rl_rocket_amd.rollout import MlpActorCritic

    torch.manual_seed(seed)
    pol = MlpActorCritic(ns, na).cuda()
    with torch.no_grad():  # move off SB3's small-gain init so every weight matters
        for prm in pol.parameters():
            prm.add_(0.3 * torch.randn_like(prm))
    return pol


@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16x3"])
@pytest.mark.parametrize("ns,na", [(14, 3), (7, 2)])
def test_policy_act_matches_torch(ns, na, prec):
    import torch
    from rl_rocket_amd import _lib
    from rl_rocket_amd.batch import _ptr
    from rl_rocket_amd.rollout import PolicyPack

    lib = _lib.load()
    n = 4096 + 37  # ragged last wave
    pol = _policy(ns, na)
    params = PolicyPack(pol, ns, na, torch.device("cuda:0"), precision=prec).pack()
    pc = PREC[prec]
    obs = torch.randn((n, ns), device="cuda:0") * 2
    it = torch.tensor([5], dtype=torch.int64, device="cuda:0")
    act_env, act = torch.empty((n, na), device="cuda:0"), torch.empty((n, na), device="cuda:0")
    val, lp, ocopy = (torch.empty((n,), device="cuda:0"), torch.empty((n,), device="cuda:0"),
                      torch.empty((n, ns), device="cuda:0"))
    _lib.check(lib.rr_policy_act(_ptr(params), ns, na, pc, n, 0, _ptr(obs), 123, _ptr(it), 3, _ptr(act_env), _ptr(act),
                                 _ptr(val), _ptr(lp), _ptr(ocopy), None, None, None, 0.0, None, None, None, None),
               "rr_policy_act")
    torch.cuda.synchronize()
    with torch.no_grad():
        mean, v = pol(obs)
        std = pol.log_std.exp()
    if prec in EXACTISH:
        print(prec, "value err", (val - v).abs().max().item())
        assert (val - v).abs().max().item() < TOL
    else:
        print("bf16 vs fp32 policy: value", (val - v).abs().max().item())
        mean, v = _emulated_bf16(pol, obs)
        _check_close(val, v, "bf16 value")
    assert torch.equal(ocopy, obs)
    assert torch.equal(act_env, act.clamp(-1, 1))
    eps = (act - mean) / std
    ref_lp = (-0.5 * eps ** 2 - pol.log_std - 0.5 * math.log(2 * math.pi)).sum(-1)
    lp_err = (lp - ref_lp).abs()
    # bf16: eps is recovered through the emulated mean, so a mean difference d shows as eps * d / std
    assert lp_err.max().item() < (1e-4 if prec in EXACTISH else 5e-2)
    if prec == "bf16":
        assert lp_err.quantile(0.99).item() < 1e-3
    e = eps.cpu().numpy()
    assert abs(e.mean()) < 0.05 and abs(e.std() - 1) < 0.05  # N(0, 1) draws
    # determinism and fresh noise per (iter, t)
    act2 = torch.empty_like(act)
    _lib.check(lib.rr_policy_act(_ptr(params), ns, na, pc, n, 0, _ptr(obs), 123, _ptr(it), 3, _ptr(act_env), _ptr(act2),
                                 _ptr(val), _ptr(lp), None, None, None, None, 0.0, None, None, None, None),
               "rr_policy_act")
    it.add_(1)
    act3 = torch.empty_like(act)
    _lib.check(lib.rr_policy_act(_ptr(params), ns, na, pc, n, 0, _ptr(obs), 123, _ptr(it), 3, _ptr(act_env), _ptr(act3),
                                 _ptr(val), _ptr(lp), None, None, None, None, 0.0, None, None, None, None),
               "rr_policy_act")
    torch.cuda.synchronize()
    assert torch.equal(act, act2)
    assert not torch.equal(act, act3)
    # the action mean itself: with log_std = -30 the sample is the mean to fp32 rounding
    with torch.no_grad():
        pol.log_std.fill_(-30.0)
    params = PolicyPack(pol, ns, na, torch.device("cuda:0"), precision=prec).pack()
    _lib.check(lib.rr_policy_act(_ptr(params), ns, na, pc, n, 0, _ptr(obs), 123, _ptr(it), 3, _ptr(act_env), _ptr(act),
                                 _ptr(val), _ptr(lp), None, None, None, None, 0.0, None, None, None, None),
               "rr_policy_act")
    torch.cuda.synchronize()
    if prec in EXACTISH:
        with torch.no_grad():
            assert (act - pol(obs)[0]).abs().max().item() < TOL
    else:
        _check_close(act, _emulated_bf16(pol, obs)[0], "bf16 mean")


@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16x3"])
@pytest.mark.parametrize("ns,na", [(14, 3), (7, 2)])
def test_policy_pack_kernel_matches_reference(ns, na, prec):
    import torch
    from rl_rocket_amd.rollout import PolicyPack

    pk = PolicyPack(_policy(ns, na, seed=4), ns, na, torch.device("cuda:0"), precision=prec)
    ref = pk.pack_reference().clone()
    pk.buf.fill_(float("nan"))
    out = pk.pack()
    torch.cuda.synchronize()
    assert torch.equal(out[:pk.size].view(torch.int32), ref[:pk.size].view(torch.int32))  # bitwise (bf16 RNE)


@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16x3"])
def test_policy_bootstrap_and_gae(prec):
    import torch
    from rl_rocket_amd import _lib
    from rl_rocket_amd.batch import _ptr
    from rl_rocket_amd.rollout import PolicyPack

    lib = _lib.load()
    n, ns, na = 8192, 14, 3
    pol = _policy(ns, na, seed=1)
    params = PolicyPack(pol, ns, na, torch.device("cuda:0"), precision=prec).pack()
    pc = PREC[prec]
    tobs = torch.randn((n, ns), device="cuda:0")
    trunc = (torch.rand((n,), device="cuda:0") < 0.01).to(torch.uint8)
    trunc[:300] = 0  # whole workgroups without a truncation take the copy-only path
    rew = torch.randn((n,), device="cuda:0")
    out = torch.empty_like(rew)
    obs = torch.randn((n, ns), device="cuda:0")
    vout = torch.empty_like(rew)
    _lib.check(lib.rr_policy_bootstrap(_ptr(params), ns, na, pc, n, _ptr(tobs), _ptr(trunc), _ptr(rew), 0.99, _ptr(out),
                                       _ptr(obs), _ptr(vout), None), "rr_policy_bootstrap")
    torch.cuda.synchronize()
    with torch.no_grad():
        if prec in EXACTISH:
            ref = rew + 0.99 * pol.value(tobs) * trunc.float()
            vref = pol.value(obs)
        else:
            ref = rew + 0.99 * _emulated_bf16(pol, tobs)[1] * trunc.float()
            vref = _emulated_bf16(pol, obs)[1]
    close = (lambda a, b, tag: _check_close(a, b, tag)) if prec == "bf16" else \
        (lambda a, b, tag: (a - b).abs().max().item() < TOL or pytest.fail(tag))
    close(out, ref, "bootstrap")
    close(vout, vref, "last value")
    # the same bootstrap fused into rr_policy_act (step t's launch does step t-1's)
    act_env, act = torch.empty((n, na), device="cuda:0"), torch.empty((n, na), device="cuda:0")
    val, lp, out2, st = (torch.empty((n,), device="cuda:0") for _ in range(4))
    done = (torch.rand((n,), device="cuda:0") < 0.1).to(torch.uint8)
    it = torch.zeros((1,), dtype=torch.int64, device="cuda:0")
    _lib.check(lib.rr_policy_act(_ptr(params), ns, na, pc, n, 0, _ptr(obs), 1, _ptr(it), 0, _ptr(act_env), _ptr(act),
                                 _ptr(val), _ptr(lp), None, _ptr(tobs), _ptr(trunc), _ptr(rew), 0.99, _ptr(out2),
                                 _ptr(done), _ptr(st), None), "rr_policy_act")
    torch.cuda.synchronize()
    close(out2, ref, "fused bootstrap")
    assert torch.equal(st, done.float())
    close(val, vref, "value")
    # GAE kernel vs the PyTorch scan (T = 37: the device scan runs in 16-step chunks, 16 + 16 + 5)
    for T in (16, 37):
        r, v, s = torch.randn((T, n), device="cuda:0"), torch.randn((T, n), device="cuda:0"), \
            (torch.rand((T, n), device="cuda:0") < 0.05).float()
        lv, ld = torch.randn((n,), device="cuda:0"), (torch.rand((n,), device="cuda:0") < 0.05).float()
        adv, ret = torch.empty_like(r), torch.empty_like(r)
        _lib.check(lib.rr_gae(T, n, _ptr(r), _ptr(v), _ptr(s), _ptr(lv), _ptr(ld), 0.99, 0.95, _ptr(adv), _ptr(ret),
                              None), "rr_gae")
        torch.cuda.synchronize()
        last, ref_adv = torch.zeros(n, device="cuda:0"), torch.empty_like(r)
        for t in reversed(range(T)):
            nt = 1.0 - (ld if t == T - 1 else s[t + 1])
            nv = lv if t == T - 1 else v[t + 1]
            last = r[t] + 0.99 * nv * nt - v[t] + 0.99 * 0.95 * nt * last
            ref_adv[t] = last
        assert (adv - ref_adv).abs().max().item() < 1e-5, T
        assert (ret - (ref_adv + v)).abs().max().item() < 1e-5, T


@pytest.mark.parametrize("fused,prec", [(True, "fp32"), (False, "fp32"), (True, "bf16"), (True, "fp16x3")])
def test_fused_collect_matches_semantics(fused, prec):
    """A fused and an unfused rollout of the same policy share every deterministic output
    (value of each visited obs, buffer layout) and both are graph-capturable."""
    import torch
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF
    from rl_rocket_amd.rollout import DeviceRollout

    n, T = 4096, 8
    env = RocketBatch(n, model=6, device="cuda:0", max_episode_steps=6, **ENV_CONFIG_6DOF)
    pol = _policy(14, 3, seed=2)
    ro = DeviceRollout(env, pol, n_steps=T, fused=fused, policy_dtype=prec)
    assert ro.fused == fused
    ro.collect()
    if prec in EXACTISH:
        with torch.no_grad():
            v = pol.value(ro.obs.reshape(-1, 14)).reshape(T, n)
        assert (ro.values - v).abs().max().item() < TOL
    else:
        _check_close(ro.values.reshape(-1), _emulated_bf16(pol, ro.obs.reshape(-1, 14))[1], "rollout values")
    for tns in (ro.obs, ro.actions, ro.rewards, ro.values, ro.log_probs, ro.advantages, ro.returns):
        assert torch.isfinite(tns).all()
    assert ro.starts[1:].sum() > 0  # TimeLimit 6 < T: episodes restart inside the rollout
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            ro.collect()
    torch.cuda.current_stream().wait_stream(st)
    a0 = ro.actions.clone()
    g.replay()
    torch.cuda.synchronize()
    assert torch.isfinite(ro.rewards).all() and not torch.equal(a0, ro.actions)
    env.close()


@pytest.mark.parametrize("prec,T", [("fp32", 8), ("bf16", 8), ("fp16x3", 8), ("fp32", 37)])
@pytest.mark.parametrize("model", [6, 3])
def test_one_launch_rollout_bitwise_equals_two_launch(model, prec, T):
    """rr_rollout_collect (the whole rollout + GAE in one kernel) and rr_rollout_step (policy +
    env step in one kernel per step) against rr_policy_act + rr_step: every rollout buffer,
    the env outputs (incl. reward terms), the terminal rows and the env state bitwise equal
    over two collects (TimeLimit 6 < n_steps: truncation bootstraps and auto-resets inside the
    rollout; ragged N: idle waves in the last workgroup; n_steps 37: the collect kernel's GAE
    scan runs in 16-step chunks, 16 + 16 + 5)."""
    import torch
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF
    from rl_rocket_amd.rollout import DeviceRollout

    n = 4096 + 37
    ns, na = (14, 3) if model == 6 else (7, 2)
    kw = ENV_CONFIG_6DOF if model == 6 else {}
    pol = _policy(ns, na, seed=3)
    ros = []
    for one, per_step in ((False, True), (True, True), (True, False)):
        env = RocketBatch(n, model=model, device="cuda:0", max_episode_steps=6, compute_terms=True, **kw)
        ro = DeviceRollout(env, pol, n_steps=T, policy_dtype=prec, one_launch=one, per_step=per_step, seed=11)
        assert ro.one_launch == one and ro.per_step == per_step
        ros.append(ro)
    for _ in range(2):
        for ro in ros:
            ro.collect()
        torch.cuda.synchronize()
        a = ros[0]
        for b in ros[1:]:
            for name in ("obs", "actions", "values", "log_probs", "starts", "rewards", "advantages", "returns",
                         "last_value", "last_done", "last_start"):
                x, y = getattr(a, name), getattr(b, name)
                assert torch.equal(x, y), (name, b.per_step, (x - y).abs().max().item())
            for name in ("obs", "reward", "done", "truncated", "terms"):
                assert torch.equal(getattr(a.env, name), getattr(b.env, name)), (name, b.per_step)
            for x, y in zip(a.env.get_state(), b.env.get_state()):
                assert torch.equal(x, y), b.per_step
            ta, tb = a.env.copy_terminal(), b.env.copy_terminal()
            for x, y in zip(ta, tb):
                assert torch.equal(x, y), b.per_step
            assert torch.equal(a.iter, b.iter)
    assert a.starts[1:].sum() > 0 and (a.rewards != 0).any()
    for ro in ros:
        ro.env.close()


def test_rollout_collect_full_size_configs4():
    """BASELINE configs[4] at its size: N = 65536 6DOF envs, TimeLimit 800, n_steps 16 (the
    bench's collect), fp32 policy. The one-launch collect (rr_rollout_collect) is bitwise the
    per-step path (rr_rollout_step launches, main_6DOF.py:62-69 scale-up); its values and
    action means match the fp32 PyTorch MlpPolicy on the collected obs, and its log-probs are
    the PyTorch log-density of the stored actions under that policy."""
    import torch
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF
    from rl_rocket_amd.rollout import DeviceRollout

    n, T = 65536, 16
    pol = _policy(14, 3, seed=4)
    ros = []
    for per_step in (False, True):
        env = RocketBatch(n, model=6, device="cuda:0", max_episode_steps=800, **ENV_CONFIG_6DOF)
        ros.append(DeviceRollout(env, pol, n_steps=T, policy_dtype="fp32", one_launch=True, per_step=per_step,
                                 seed=21))
    for _ in range(4):  # 64 steps: random-policy episodes end after 44-105 steps, so resets occur
        for ro in ros:
            ro.collect()
    torch.cuda.synchronize()
    a, b = ros
    for name in ("obs", "actions", "values", "log_probs", "starts", "rewards", "advantages", "returns",
                 "last_value", "last_done"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    for x, y in zip(a.env.get_state(), b.env.get_state()):
        assert torch.equal(x, y)
    with torch.no_grad():
        mean, value = pol(a.obs.reshape(-1, 14))
        lp = pol.log_prob(mean, a.actions.reshape(-1, 3))
    assert (a.values.reshape(-1) - value).abs().max().item() < TOL
    assert (a.log_probs.reshape(-1) - lp).abs().max().item() < 5e-4
    # the stored actions are mean + std * N(0, 1) noise around the PyTorch means
    z = ((a.actions.reshape(-1, 3) - mean) / pol.log_std.exp()).double()
    assert abs(z.mean().item()) < 0.01 and abs(z.std().item() - 1.0) < 0.01
    assert a.starts.sum() > 0 and torch.isfinite(a.advantages).all()
    for ro in ros:
        ro.env.close()


def test_unfused_bootstrap_ignores_stale_terminal_rows():
    """the PyTorch rollout path selects r + gamma V(terminal obs) only where an env
    was truncated, so a NaN left in the terminal buffer of a running env cannot reach its reward."""
    import torch
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF
    from rl_rocket_amd.rollout import DeviceRollout

    n = 2048
    env = RocketBatch(n, model=6, device="cuda:0", max_episode_steps=5, **ENV_CONFIG_6DOF)
    ro = DeviceRollout(env, _policy(14, 3, seed=6), n_steps=8, fused=False)
    env.copy_terminal()  # warm
    orig = env.copy_terminal

    def poisoned(out=None):  # every terminal row NaN except where the last step truncated
        res = orig(out)
        res[0][env.truncated == 0] = float("nan")
        return res

    env.copy_terminal = poisoned
    ro.collect()
    assert torch.isfinite(ro.rewards).all() and torch.isfinite(ro.advantages).all()
    env.close()


def test_graphed_ppo_update_equals_eager():
    """GraphedPPOUpdate (the minibatch update captured once in a hipGraph, replayed per
    minibatch) against the eager ppo_update from the same parameters, optimizer state, rollout
    and shuffling: the same parameters after two epochs (same kernels in the same order), and the
    capture's warm-up steps leave no trace."""
    import copy

    import torch
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF
    from rl_rocket_amd.rollout import DeviceRollout, GraphedPPOUpdate, ppo_update

    n, T, bs = 8192, 8, 8192
    env = RocketBatch(n, model=6, device="cuda:0", max_episode_steps=30, **ENV_CONFIG_6DOF)
    pol = _policy(14, 3, seed=7)
    ro = DeviceRollout(env, pol, n_steps=T, seed=3)
    ro.collect()
    torch.cuda.synchronize()
    pa, pb = copy.deepcopy(pol), copy.deepcopy(pol)
    oa = torch.optim.Adam(pa.parameters(), lr=3e-4, eps=1e-5, capturable=True)
    ob = torch.optim.Adam(pb.parameters(), lr=3e-4, eps=1e-5, capturable=True)
    g = GraphedPPOUpdate(pb, ob, ro, batch_size=bs, fused=False)
    for x, y in zip(pa.parameters(), pb.parameters()):  # warm-up undone
        assert torch.equal(x, y)
    sa = ppo_update(pa, oa, ro, n_epochs=2, batch_size=bs, generator=torch.Generator("cuda:0").manual_seed(5))
    sb = g.update(n_epochs=2, generator=torch.Generator("cuda:0").manual_seed(5))
    torch.cuda.synchronize()
    worst = max((x - y).abs().max().item() for x, y in zip(pa.parameters(), pb.parameters()))
    moved = max((x - y).abs().max().item() for x, y in zip(pol.parameters(), pb.parameters()))
    assert moved > 0  # the update did something
    assert worst <= 1e-6, worst
    for k in sa:
        assert abs(sa[k] - sb[k]) <= 1e-5 * max(1.0, abs(sa[k])), (k, sa[k], sb[k])
    env.close()
