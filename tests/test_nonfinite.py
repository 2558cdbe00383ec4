"""Non-finite states and actions.

The reference's step on a non-finite state or action never returns: scipy's RK45 gets a NaN
step size, its `h_abs < min_step` test is False for ever and `_step_impl` loops
(simulator.py:236-241). Had it failed it would return status -1 and the env would be done
(`done = bool(status)`, rocket_env.py:702 / :158). The defined behaviour here is that failure:
  * oracle and exact mode (DOPRI5): the solver stops with TOO_SMALL_STEP, status -1, the state
    is the last accepted one (the input state: no step was accepted), done;
  * fast mode (RK4): a post-step state with a NaN / inf component is done, status -1 in the
    terms plane (unless the ground event fired), the next obs is the auto-reset one;
  * every other env of the batch is bitwise unaffected.
"""
import numpy as np
import pytest

NAN, INF = float("nan"), float("inf")


def _bad_rows(model):
    """(row, kind, column, value): state components and action components set non-finite."""
    if model == 6:
        st = [(3, "s", 0, NAN), (5, "s", 4, INF), (8, "s", 7, NAN), (11, "s", 11, -INF), (13, "s", 13, NAN),
              (17, "s", 6, INF)]
        ac = [(20, "a", 0, NAN), (22, "a", 1, INF), (25, "a", 2, NAN), (27, "a", 2, INF), (29, "a", 2, -INF)]
    else:
        st = [(3, "s", 0, NAN), (5, "s", 1, INF), (8, "s", 2, INF), (11, "s", 3, NAN), (13, "s", 5, -INF),
              (17, "s", 6, NAN)]
        ac = [(20, "a", 0, NAN), (22, "a", 1, INF), (25, "a", 1, -INF)]
    return st + ac


def _kw(model):
    from oracle import oracle as O
    return O.ENV_CONFIG_6DOF if model == 6 else O.DEFAULTS_3DOF


def _clean(model, n, seed=0):
    rng = np.random.default_rng(seed)
    kw = _kw(model)
    ns, na = (14, 3) if model == 6 else (7, 2)
    lo = np.float32(kw["IC"]) - np.float32(kw["ICRange"]) / 2
    hi = np.float32(kw["IC"]) + np.float32(kw["ICRange"]) / 2
    s = rng.uniform(lo, hi, (n, ns)).astype(np.float32)
    if model == 6:
        s[:, 6:10] /= np.linalg.norm(s[:, 6:10], axis=1, keepdims=True)
    a = rng.uniform(-1, 1, (n, na)).astype(np.float32)
    return s, a


def _inject(model, s, a):
    s, a = s.copy(), a.copy()
    rows = []
    for r, kind, c, v in _bad_rows(model):
        (s if kind == "s" else a)[r, c] = v
        rows.append(r)
    return s, a, np.array(rows)


@pytest.mark.parametrize("model", [6, 3])
def test_oracle_stops_with_status_minus_one(model, oracle_mod):
    """The oracle (CPU restatement of scipy RK45) returns on non-finite rows: status -1, done,
    the input state (no step accepted); finite rows unchanged by the guard."""
    n = 32
    s, a = _clean(model, n)
    sb, ab, bad = _inject(model, s, a)
    cfg = oracle_mod.make_cfg(model, **_kw(model))
    ref = oracle_mod.step(cfg, s, 0.0, s.astype(np.float64), a)
    out = oracle_mod.step(cfg, s, 0.0, sb.astype(np.float64), ab)
    good = np.setdiff1d(np.arange(n), bad)
    assert out["done"][bad].all()
    # status -1 except where the solver never sees the non-finite value: the 3DOF altitude z enters
    # no derivative (simulator.py:88-130), so z = inf integrates "fine" (status 0) and the bounds
    # check ends the episode
    fine = (out["status"][bad] == 0)
    assert (out["status"][bad][~fine] == -1).all()
    assert fine.sum() == (1 if model == 3 else 0) and out["bounds_violation"][bad][fine].all()
    for k in ("state_out", "obs", "reward", "status", "done"):
        np.testing.assert_array_equal(out[k][good], ref[k][good])
    act_rows = np.array([r for r, kind, _, _ in _bad_rows(model) if kind == "a"])
    st_in = sb[act_rows].astype(np.float64)
    if model == 6:  # the input state, after _normalize_quaternion
        st_in[:, 6:10] /= np.linalg.norm(st_in[:, 6:10], axis=1, keepdims=True)
    else:
        st_in[:, 2] = np.fmod(np.fmod(st_in[:, 2], 2 * np.pi) + 2 * np.pi, 2 * np.pi)
    np.testing.assert_allclose(out["state_out"][act_rows], st_in, rtol=1e-15, atol=0)


def _gpu_step(model, s, a, integrator="rk4", auto_reset=True, n_steps=1):
    import torch
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF

    n = len(s)
    kw = ENV_CONFIG_6DOF if model == 6 else {}
    b = RocketBatch(n, model=model, device="cuda:0", max_episode_steps=800, auto_reset=auto_reset,
                    episode_stats=True, compute_terms=True, integrator=integrator, **kw)
    b.reset()
    ic = s.astype(np.float32)
    v0 = np.sqrt((np.nan_to_num(ic[:, 3:6 if model == 6 else 5], posinf=0.0, neginf=0.0) ** 2).sum(1)).astype(np.float32)
    if integrator == "dopri5":
        b.set_state64(torch.from_numpy(np.ascontiguousarray(s.astype(np.float64).T)), v0=torch.from_numpy(v0))
    else:
        b.set_state(torch.from_numpy(np.ascontiguousarray(s.T)), v0=torch.from_numpy(v0))
    act = torch.from_numpy(a).cuda()
    outs = []
    for _ in range(n_steps):
        obs, rew, done, trunc = b.step(act)
        o = dict(obs=obs.cpu().numpy(), reward=rew.cpu().numpy(), done=done.cpu().numpy().astype(bool),
                 terms=b.terms.cpu().numpy().T.copy(), state=b.get_state()[0].cpu().numpy().T.copy())
        o["tidx"], o["tobs"], _, _ = b.fetch_done()
        outs.append(o)
    b.close()
    return outs


@pytest.mark.gpu
@pytest.mark.parametrize("model", [6, 3])
@pytest.mark.parametrize("help_max", [None, "0"])
def test_fast_kernel_ends_non_finite_episodes(model, help_max, monkeypatch):
    """Both step kernels: the helper-wave kernel (N <= RR_HELP_MAX_N, default) and the plain one
    (RR_HELP_MAX_N=0, what every N > 131 072 runs)."""
    if help_max is not None:
        monkeypatch.setenv("RR_HELP_MAX_N", help_max)
    n = 300  # ragged: 4.7 waves
    s, a = _clean(model, n, seed=model)
    sb, ab, bad = _inject(model, s, a)
    good = np.setdiff1d(np.arange(n), bad)
    ref = _gpu_step(model, s, a, n_steps=3)
    out = _gpu_step(model, sb, ab, n_steps=3)
    o0 = out[0]
    assert o0["done"][bad].all(), np.nonzero(~o0["done"][bad])
    status = o0["terms"][:, -1]
    assert (status[bad] == -1.0).all(), status[bad]
    assert set(np.unique(status[good])) <= {0.0, 1.0}
    # the bad rows' terminal obs carry the non-finite state; they restart from finite ICs
    tpos = np.searchsorted(o0["tidx"], bad)
    assert np.array_equal(o0["tidx"][tpos], bad)
    assert not np.isfinite(o0["tobs"][tpos]).all(1).any()
    for o in out:
        assert np.isfinite(o["obs"][bad]).all() and np.isfinite(o["state"][bad]).all()
    # every other env: bitwise what it does in a batch without the bad rows (the second and
    # third steps keep stepping the bad rows with their non-finite actions: done every step)
    for o, r in zip(out, ref):
        for k in ("obs", "reward", "done", "terms", "state"):
            assert np.array_equal(o[k][good], r[k][good]), k
    act_bad = np.array([r for r, kind, _, _ in _bad_rows(model) if kind == "a"])
    for o in out[1:]:
        assert o["done"][act_bad].all()


@pytest.mark.gpu
@pytest.mark.parametrize("model", [6, 3])
def test_fast_kernel_without_auto_reset_keeps_reporting_done(model):
    n = 64
    s, a = _clean(model, n, seed=7)
    sb, ab, bad = _inject(model, s, a)
    out = _gpu_step(model, sb, ab, auto_reset=False, n_steps=2)
    for o in out:
        assert o["done"][bad].all()
        assert not np.isfinite(o["state"][bad]).all(1).any()


@pytest.mark.gpu
@pytest.mark.parametrize("model,lean", [(6, False), (3, False), (6, True)])
def test_exact_mode_stops_like_the_oracle(model, lean, oracle_mod, monkeypatch):
    """DOPRI5 exact mode terminates on non-finite rows (status -1, done) with the oracle's
    state; the other rows bitwise as in a clean batch. lean: the 6DOF lean two-waves-per-SIMD
    kernel (RR_EXACT_LEAN_MIN_N=0; what N above CUs x 256 runs; 3DOF has no lean kernel)."""
    if lean:
        monkeypatch.setenv("RR_EXACT_LEAN_MIN_N", "0")
    n = 128
    s, a = _clean(model, n, seed=11)
    sb, ab, bad = _inject(model, s, a)
    good = np.setdiff1d(np.arange(n), bad)
    ref = _gpu_step(model, s, a, integrator="dopri5", auto_reset=False)[0]
    out = _gpu_step(model, sb, ab, integrator="dopri5", auto_reset=False)[0]
    assert out["done"][bad].all()
    for k in ("obs", "reward", "done", "terms", "state"):
        assert np.array_equal(out[k][good], ref[k][good]), k
    cfg = oracle_mod.make_cfg(model, **_kw(model))
    orc = oracle_mod.step(cfg, sb, 0.0, sb.astype(np.float64), ab)
    np.testing.assert_array_equal(out["terms"][bad, -1], orc["status"][bad].astype(np.float32))
    fin = np.isfinite(orc["state_out"][bad]).all(1)
    assert fin.sum() >= 3  # the non-finite-action rows keep their (finite) input state
    np.testing.assert_allclose(out["state"][bad][fin], orc["state_out"][bad][fin].astype(np.float32), rtol=1e-6,
                               atol=1e-6)


def _nan_equal(x, y):
    import torch

    return bool(((x == y) | (torch.isnan(x) & torch.isnan(y))).all())


@pytest.mark.gpu
@pytest.mark.parametrize("model", [6, 3])
@pytest.mark.parametrize("per_step", [False, True])
def test_rollout_kernels_end_non_finite_episodes(model, per_step):
    """the on-device rollout (rr_rollout_collect, one launch, in its own translation
    unit; per_step: rr_rollout_step) ends an episode whose state turns non-finite, as rr_step
    does: rows with a NaN / inf state component step to status -1 (terms plane), done, and
    restart from finite initial conditions (the next collect's obs are finite); every other env's
    rollout buffers, outputs and state are bitwise those of a twin batch without the bad rows
    (a NaN in one env's MFMA column reaches no other env)."""
    import torch
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF
    from rl_rocket_amd.rollout import DeviceRollout, MlpActorCritic

    n = 4096 + 37
    ns, na = (14, 3) if model == 6 else (7, 2)
    kw = ENV_CONFIG_6DOF if model == 6 else {}
    torch.manual_seed(5)
    pol = MlpActorCritic(ns, na).cuda()
    bad = np.array([3, 64, 65, 700, 4100])
    cols = np.array([0, 4, ns - 1, 6 if model == 6 else 2, 3])
    vals = [float("nan"), float("inf"), float("nan"), -float("inf"), float("nan")]
    ros = []
    for poison in (False, True):
        env = RocketBatch(n, model=model, device="cuda:0", max_episode_steps=800, compute_terms=True, **kw)
        ro = DeviceRollout(env, pol, n_steps=1, one_launch=True, per_step=per_step, seed=3)
        st, v0, _ = env.get_state()
        if poison:
            for r, c, v in zip(bad, cols, vals):
                st[c, r] = v
        env.set_state(st, v0=v0)
        ros.append(ro)
    good = torch.ones(n, dtype=torch.bool, device="cuda:0")
    good[torch.as_tensor(bad, device="cuda:0")] = False
    for k in range(2):
        for ro in ros:
            ro.collect()
        torch.cuda.synchronize()
        clean, dirty = ros
        status = dirty.env.terms[-1]
        if k == 0:
            assert (status[~good] == -1.0).all() and (dirty.env.done[~good] == 1).all(), status[~good]
        assert torch.isfinite(dirty.env.obs[~good]).all()  # auto-reset to finite initial conditions
        for name in ("obs", "actions", "values", "log_probs", "starts", "rewards", "advantages", "returns",
                     "last_value", "last_done"):
            x, y = getattr(clean, name), getattr(dirty, name)
            assert _nan_equal(x[..., good] if x.dim() == 1 else x[:, good], y[..., good] if y.dim() == 1 else
                              y[:, good]), (name, k)
        for name in ("obs", "reward", "done", "truncated"):
            assert torch.equal(getattr(clean.env, name)[good], getattr(dirty.env, name)[good]), name
        assert torch.equal(clean.env.terms[:, good], dirty.env.terms[:, good])
        assert torch.equal(clean.env.get_state()[0][:, good], dirty.env.get_state()[0][:, good])
    for ro in ros:
        ro.env.close()
