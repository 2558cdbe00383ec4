"""GPU: counter words, checkpoints, sharded stepping and the packed-row / all-gather path
(the multi-GPU design of SURVEY.md §8e exercised on one GPU)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _env6():
    from rl_rocket_amd.params import ENV_CONFIG_6DOF
    return ENV_CONFIG_6DOF


def _actions(n, na, steps, seed):
    import torch

    g = torch.Generator(device="cuda:0")
    g.manual_seed(seed)
    return [torch.rand((n, na), device="cuda:0", generator=g) * 2 - 1 for _ in range(steps)]


@pytest.mark.parametrize("model", [6, 3])
def test_step_rows_is_bitwise_step(model):
    """rr_step_rows writes (obs, reward, done) rows bitwise equal to rr_step's three outputs,
    with the same state, truncation flags and reward terms, over steps with resets."""
    import torch
    from rl_rocket_amd.batch import RocketBatch

    n = 4096 + 77
    kw = _env6() if model == 6 else {}
    a = RocketBatch(n, model=model, device="cuda:0", max_episode_steps=30, compute_terms=True, **kw)
    b = RocketBatch(n, model=model, device="cuda:0", max_episode_steps=30, compute_terms=True, **kw)
    a.reset()
    b.reset()
    rows = torch.empty((n, a.state_dim + 2), device="cuda:0")
    ns = a.state_dim
    for act in _actions(n, a.action_dim, 45, 3):
        obs, rew, done, trunc = a.step(act)
        b.step_rows(act, rows)
        assert torch.equal(rows[:, :ns], obs)
        assert torch.equal(rows[:, ns], rew)
        assert torch.equal(rows[:, ns + 1], done.float())
        assert torch.equal(b.truncated, trunc)
        assert torch.equal(b.terms, a.terms)
    for x, y in zip(a.get_state(), b.get_state()):
        assert torch.equal(x, y)


@pytest.mark.parametrize("model", [6, 3])
def test_sharded_stepping_is_bitwise_one_batch(model):
    """envs are independent and the reset stream is keyed on global ids, so three
    uneven shards (rl_rocket_amd.dist.shard, env_id_offset = shard offset) step bitwise like one
    batch of all envs: obs, rewards, done / truncated, terminal rows and state, over 60 steps
    with TimeLimit 25 (every env resets at least twice)."""
    import torch
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.dist import shard

    n, world = 20000 + 3, 3
    kw = _env6() if model == 6 else {}
    whole = RocketBatch(n, model=model, device="cuda:0", max_episode_steps=25, **kw)
    parts = []
    for r in range(world):
        m, off = shard(n, world, r)
        parts.append((off, m, RocketBatch(m, model=model, device="cuda:0", max_episode_steps=25, env_id_offset=off,
                                          **kw)))
    o_all = whole.reset()
    for off, m, p in parts:
        assert torch.equal(p.reset(), o_all[off:off + m])
    resets = 0
    for act in _actions(n, whole.action_dim, 60, 11):
        obs, rew, done, trunc = whole.step(act)
        idx, tobs, ret, ln = whole.fetch_done()
        resets += len(idx)
        for off, m, p in parts:
            o2, r2, d2, t2 = p.step(act[off:off + m])
            assert torch.equal(o2, obs[off:off + m])
            assert torch.equal(r2, rew[off:off + m])
            assert torch.equal(d2, done[off:off + m])
            assert torch.equal(t2, trunc[off:off + m])
            i2, to2, ret2, ln2 = p.fetch_done()
            sel = (idx >= off) & (idx < off + m)
            np.testing.assert_array_equal(i2 + off, idx[sel])
            np.testing.assert_array_equal(to2, tobs[sel])
            np.testing.assert_array_equal(ret2, ret[sel])
            np.testing.assert_array_equal(ln2, ln[sel])
    assert resets >= 2 * n
    st = whole.get_state()
    for off, m, p in parts:
        st2 = p.get_state()
        assert torch.equal(st2[0], st[0][:, off:off + m])
        assert torch.equal(st2[1], st[1][off:off + m])
        assert torch.equal(st2[2], st[2][off:off + m])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_graph_captured_step_and_allgather_rccl():
    """The multi-GPU hot path on one GPU: rr_step_rows into ShardGather's send rows + ONE
    RCCL all_gather_into_tensor ("nccl" backend, world 1), captured in a hipGraph. Replays give
    bitwise the outputs of the same steps run eagerly through rr_step."""
    import torch
    import torch.distributed as dist
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.dist import ShardGather

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        n = 65536
        a = RocketBatch(n, model=6, device=dev, max_episode_steps=30, **_env6())
        b = RocketBatch(n, model=6, device=dev, max_episode_steps=30, **_env6())
        a.reset()
        b.reset()
        g = ShardGather(n, 14, dev)
        acts = _actions(n, 3, 8, 5)
        g.step(b, acts[0])  # eager warm-up (communicator set up outside the capture)
        a.step(acts[0])
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(graph, stream=s):
                for k in range(1, 4):
                    g.step(b, acts[k])
        torch.cuda.current_stream().wait_stream(s)
        for rep in range(2):  # two replays = steps 1..3, 4..6 of the eager twin
            graph.replay()
            for k in range(1, 4):
                obs, rew, done, _ = a.step(acts[k])
            torch.cuda.synchronize()
            assert torch.equal(g.obs, obs)
            assert torch.equal(g.reward, rew)
            assert torch.equal(g.done, done.float())
        assert torch.equal(a.get_state()[0], b.get_state()[0])
    finally:
        dist.destroy_process_group()


def test_counter_layout_and_reset_keys_beyond_65536_episodes():
    """The counter word holds the TimeLimit steps in E = bits(max_episode_steps) bits (10 for
    the reference's TimeLimit 800) and the episode number above them (22 bits), so one env's
    reset keys do not repeat after 65 536 episodes: episodes e and e + 65536 (and e + 2^21)
    ending at the same step draw different initial conditions (with the round-1 16 / 16 layout
    they were the same key)."""
    import torch
    from rl_rocket_amd.batch import RocketBatch

    n = 64
    b = RocketBatch(n, model=6, device="cuda:0", max_episode_steps=800, **_env6())
    assert b.counter_bits == 10
    assert RocketBatch(8, model=6, device="cuda:0", max_episode_steps=0, **_env6()).counter_bits == 16
    assert RocketBatch(8, model=6, device="cuda:0", max_episode_steps=1, **_env6()).counter_bits == 1
    b.reset()
    ck = b.checkpoint()
    act = torch.zeros((n, 3), device="cuda:0")
    ics = []
    for ep in (5, 5 + 65536, 5 + (1 << 21)):
        ck["counter"] = torch.as_tensor(b.make_counter(799, ep), device="cuda:0").expand(n).contiguous()
        b.restore(ck)
        obs, rew, done, trunc = b.step(act)  # step 800: TimeLimit -> reset keyed on (gid, counter word)
        assert bool(trunc.all())
        ics.append(obs.clone())
        el, epn = b.split_counter(b.checkpoint()["counter"])
        assert bool((el == 0).all()) and bool((epn == ep + 1).all())
    for i in range(3):
        for j in range(i + 1, 3):
            assert not torch.equal(ics[i], ics[j])
            assert bool((ics[i] != ics[j]).any(dim=1).all())  # every env's IC differs


def test_checkpoint_restore_is_bitwise():
    """checkpoint() / restore() round-trips state, v0, counter words (reset-stream keys) and
    the Monitor running return: the steps after a restore are bitwise the steps after the
    checkpoint, incl. the episode returns of finished episodes (set_state alone
    dropped the running return and the episode field)."""
    import torch
    from rl_rocket_amd.batch import RocketBatch

    n = 5000
    b = RocketBatch(n, model=6, device="cuda:0", max_episode_steps=40, **_env6())
    b.reset()
    acts = _actions(n, 3, 70, 9)
    for act in acts[:30]:
        b.step(act)
    ck = {k: v.clone() for k, v in b.checkpoint().items()}

    def run():
        out = []
        for act in acts[30:]:
            obs, rew, done, trunc = b.step(act)
            idx, tobs, ret, ln = b.fetch_done()
            out.append((obs.clone(), rew.clone(), done.clone(), idx.copy(), ret.copy(), ln.copy()))
        return out

    first = run()
    b.restore(ck)
    second = run()
    for x, y in zip(first, second):
        for u, v in zip(x[:3], y[:3]):
            assert torch.equal(u, v)
        for u, v in zip(x[3:], y[3:]):
            np.testing.assert_array_equal(u, v)
    assert any(len(x[3]) for x in first)
    # set_state without counter words keeps the episode field and clears the steps
    cw = torch.as_tensor(b.make_counter(17, 123), device="cuda:0").expand(n).contiguous()
    b.restore(dict(ck, counter=cw))
    b.set_state(ck["state"], v0=ck["v0"])
    el, ep = b.split_counter(b.checkpoint()["counter"])
    assert bool((el == 0).all()) and bool((ep == 123).all())


@pytest.mark.parametrize("model,n,soa", [(6, 4096 + 77, False), (6, 20003, False), (6, 131072 + 5, True), (6, 65536, False),
                                         (3, 20003, True), (3, 4096 + 77, False)])
def test_step_repeat_direct_launch_is_bitwise_step(model, n, soa):
    """bench.py's event-timed direct-launch region (tools/libbench_timed.so: K rr_step calls
    queued behind the host-released gate kernel, two timing events around them) and
    rr_step_repeat under stream capture: bitwise the same outputs, terminal rows, Monitor
    returns, counter words and state as one rr_step per step, across a re-seed."""
    import torch
    from bench import TimedLoop
    from rl_rocket_amd.batch import RocketBatch

    kw = _env6() if model == 6 else {}
    mk = lambda: RocketBatch(n, model=model, device="cuda:0", max_episode_steps=30, compute_terms=True,  # noqa: E731
                             action_soa=soa, **kw)
    a, b = mk(), mk()
    a.reset()
    b.reset()
    loop = TimedLoop(b)
    pool = torch.rand((3, n, a.action_dim), device="cuda:0", generator=torch.Generator("cuda:0").manual_seed(5)) * 2 - 1
    if soa:
        pool = pool.transpose(1, 2).contiguous()
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    for e in ev:
        e.record()
    resets = 0
    for chunk, seed in ((7, None), (25, 99), (1, None), (40, None)):
        if seed is not None:
            a.seed(seed)
            b.seed(seed)
        for t in range(chunk):
            a.step(pool[t % 3])
            resets += int(a.done.sum())
        fn, fargs = loop.call(pool, chunk, ev)
        assert fn(*fargs) == 0
        torch.cuda.synchronize()
        assert ev[0].elapsed_time(ev[1]) > 0.0
        for x, y in ((a.obs, b.obs), (a.reward, b.reward), (a.done, b.done), (a.truncated, b.truncated),
                     (a.terms, b.terms)):
            assert torch.equal(x, y)
        for x, y in zip(a.get_state(), b.get_state()):
            assert torch.equal(x, y)
        ca, cb = a.checkpoint(), b.checkpoint()
        for k in ca:
            assert torch.equal(ca[k], cb[k]), k
    assert resets > n // 2
    # captured: the graph records the by-value kernel; replays match eager steps
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            b.step_repeat(pool, 3)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(2):
        for t in range(3):
            a.step(pool[t])
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(a.obs, b.obs) and torch.equal(a.reward, b.reward)
    for x, y in zip(a.get_state(), b.get_state()):
        assert torch.equal(x, y)


@pytest.mark.parametrize("model,n,help_max", [(6, 4096 + 77, None), (6, 20003, None), (6, 20003, 0), (3, 4096 + 77, 0)])
def test_reseed_applies_to_graphs_captured_before(model, n, help_max, monkeypatch):
    """every kernel reads the reset-stream key from the device copy of the parameters,
    so a hipGraph captured BEFORE rr_seed resets with the NEW key when replayed after it — with
    helper waves (N <= RR_HELP_MAX_N: one main wave per workgroup at 4 173 envs, four at 20 003)
    and without them (RR_HELP_MAX_N=0: the main waves draw the candidates). Replays are bitwise an
    eager twin seeded the same way, and differ from a twin that kept the old seed."""
    import torch
    from rl_rocket_amd.batch import RocketBatch

    if help_max is not None:
        monkeypatch.setenv("RR_HELP_MAX_N", str(help_max))
    kw = _env6() if model == 6 else {}
    mk = lambda: RocketBatch(n, model=model, device="cuda:0", max_episode_steps=3, **kw)  # noqa: E731
    a, b, c = mk(), mk(), mk()
    for e in (a, b, c):
        e.reset()
    acts = _actions(n, a.action_dim, 6, 21)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for act in acts:
                b.step(act)
    torch.cuda.current_stream().wait_stream(s)
    a.seed(777)
    b.seed(777)
    g.replay()
    for act in acts:
        a.step(act)
        c.step(act)
    torch.cuda.synchronize()
    assert torch.equal(a.obs, b.obs) and torch.equal(a.reward, b.reward) and torch.equal(a.done, b.done)
    for x, y in zip(a.get_state(), b.get_state()):
        assert torch.equal(x, y)
    assert not torch.equal(a.get_state()[0], c.get_state()[0])  # the key changed the resets


def test_seed_between_replays_on_another_stream():
    """a graph captured on stream S and replayed on stream R is not a launch of the handle,
    so rr_seed does not track it (include/rocket_hip.h); the documented protocol — order the replay
    before the seed (here: synchronise R) — gives the first replay the old key and the second the new
    one, bitwise an eager twin that seeds between the same steps."""
    import torch
    from rl_rocket_amd.batch import RocketBatch

    n = 20003
    mk = lambda: RocketBatch(n, model=6, device="cuda:0", max_episode_steps=2, **_env6())  # noqa: E731
    a, b = mk(), mk()
    for e in (a, b):
        e.reset()
    acts = _actions(n, 3, 4, 33)
    cap, rep = torch.cuda.Stream(), torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(cap):
        with torch.cuda.graph(g, stream=cap):
            for act in acts:
                b.step(act)
    torch.cuda.synchronize()
    rep.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(rep):
        g.replay()
    rep.synchronize()  # the caller orders the replay before the seed
    b.seed(4242)
    with torch.cuda.stream(rep):
        g.replay()
    for act in acts:
        a.step(act)
    a.seed(4242)
    for act in acts:
        a.step(act)
    torch.cuda.synchronize()
    assert torch.equal(a.obs, b.obs) and torch.equal(a.reward, b.reward)
    for x, y in zip(a.get_state(), b.get_state()):
        assert torch.equal(x, y)


def test_elapsed_saturates_past_the_time_limit():
    """without auto-reset a finished env keeps stepping; its elapsed field saturates
    at 2^E - 1 (E = 3 bits for TimeLimit 5) instead of wrapping into the episode field, so
    TimeLimit keeps reporting done (and truncated where the physics did not end the episode),
    as gym's TimeLimit does for every step past the limit."""
    import torch
    from rl_rocket_amd.batch import RocketBatch

    n = 256
    b = RocketBatch(n, model=6, device="cuda:0", max_episode_steps=5, auto_reset=False, episode_stats=True,
                    compute_terms=True, **_env6())
    assert b.counter_bits == 3
    b.reset()
    act = torch.zeros((n, 3), device="cuda:0")
    for t in range(1, 21):
        obs, rew, done, trunc = b.step(act)
        phys = (b.terms[-2] > 0.5) | (b.terms[-1] > 0.5)
        el, ep = b.split_counter(b.checkpoint()["counter"])
        assert bool((el == min(t, 7)).all()) and bool((ep == 1).all()), t
        if t >= 5:
            assert bool(done.bool().all()), t
            assert torch.equal(trunc.bool(), ~phys), t
        else:
            assert torch.equal(done.bool(), phys), t


def test_make_counter_rejects_spilling_values():
    from rl_rocket_amd.batch import RocketBatch

    b = RocketBatch(8, model=6, device="cuda:0", max_episode_steps=800, **_env6())
    assert b.make_counter(1023, 5).view(np.uint32)[()] == (5 << 10) | 1023
    with pytest.raises(ValueError):
        b.make_counter(1024)
    with pytest.raises(ValueError):
        b.make_counter(3, 1 << 22)


def test_copy_terminal_writes_only_the_done_rows():
    """rr_copy_terminal copies the terminal rows of the envs done at the last step (from its
    done masks) and leaves every other destination row untouched: the rows equal the host done
    list of rr_fetch_done."""
    import torch
    from rl_rocket_amd.batch import RocketBatch

    n = 4096 + 77
    b = RocketBatch(n, model=6, device="cuda:0", max_episode_steps=30, **_env6())
    b.reset()
    ck = b.checkpoint()
    ck["counter"] = torch.as_tensor(b.make_counter(np.arange(n) % 30), device="cuda:0")
    b.restore(ck)
    tobs = torch.full((n, 14), float("nan"), device="cuda:0")
    ret = torch.full((n,), -7.0, device="cuda:0")
    ln = torch.full((n,), -1, dtype=torch.int32, device="cuda:0")
    b.step(_actions(n, 3, 1, 2)[0])
    b.copy_terminal(out=(tobs, ret, ln))
    idx, to, r, l = b.fetch_done()
    assert 0 < len(idx) < n
    np.testing.assert_array_equal(tobs.cpu().numpy()[idx], to)
    np.testing.assert_array_equal(ret.cpu().numpy()[idx], r)
    np.testing.assert_array_equal(ln.cpu().numpy()[idx], l)
    rest = np.setdiff1d(np.arange(n), idx)
    assert np.isnan(tobs.cpu().numpy()[rest]).all()
    assert (ret.cpu().numpy()[rest] == -7.0).all() and (ln.cpu().numpy()[rest] == -1).all()


def test_seed_is_stream_ordered_and_refused_inside_a_capture():
    """rr_seed writes the key in the order of the env's stream (launches queued before
    it on that stream read the old key; it synchronises that stream only) and refuses a stream that
    is being captured (RR_EINVAL) instead of synchronising the device inside a capture; the
    capture itself stays valid and replays bitwise like the eager twin."""
    import torch
    from rl_rocket_amd import _lib
    from rl_rocket_amd.batch import RocketBatch

    n = 4096 + 77
    mk = lambda: RocketBatch(n, model=6, device="cuda:0", max_episode_steps=3, **_env6())  # noqa: E731
    a, b = mk(), mk()
    for e in (a, b):
        e.reset()
    acts = _actions(n, a.action_dim, 4, 5)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for k, act in enumerate(acts):
                b.step(act)
                if k == 1:
                    with pytest.raises(_lib.RocketHipError, match="captured"):
                        b.seed(99)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    for act in acts:
        a.step(act)
    torch.cuda.synchronize()
    assert torch.equal(a.obs, b.obs) and torch.equal(a.get_state()[0], b.get_state()[0])
    # stream order: steps queued on the stream before the re-seed keep the old key, after it the new
    c, d = mk(), mk()
    for e in (c, d):
        e.reset()
    for act in acts[:2]:
        c.step(act)
        d.step(act)
    c.seed(1234)  # right behind the queued steps, no synchronise of ours in between
    torch.cuda.synchronize()
    d.seed(1234)
    for act in acts[2:]:
        c.step(act)
        d.step(act)
    torch.cuda.synchronize()
    assert torch.equal(c.obs, d.obs) and torch.equal(c.get_state()[0], d.get_state()[0])


@pytest.mark.parametrize("model,n,forced", [(6, 20003, True), (3, 20003, True), (6, (1 << 20) + 5, False)])
def test_whole_line_done_path_is_bitwise_the_partial_line_path(model, n, forced, monkeypatch):
    """above RR_WHOLE_LINE_MIN_N (default 1 << 20 envs) the plain step kernel stores the
    terminal return / length and the reset v0 from EVERY lane of a wave that has a done lane, as
    whole lines. That path (forced at 20 003 envs with RR_WHOLE_LINE_MIN_N=0, and at its default
    threshold just past 1 M envs) against the partial-line path (threshold above N), both on the
    plain kernel (RR_HELP_MAX_N=0), with auto-reset, Monitor returns and TimeLimit 7: obs, reward,
    done / truncated, terms, state, v0, counter words, running returns and the done lists
    (indices, terminal rows, returns, lengths) are bitwise equal at every step."""
    import torch
    from rl_rocket_amd.batch import RocketBatch

    monkeypatch.setenv("RR_HELP_MAX_N", "0")
    kw = _env6() if model == 6 else {}
    mk = lambda: RocketBatch(n, model=model, device="cuda:0", max_episode_steps=7, episode_stats=True,  # noqa: E731
                             compute_terms=True, **kw)
    if forced:
        monkeypatch.setenv("RR_WHOLE_LINE_MIN_N", "0")
    else:
        monkeypatch.delenv("RR_WHOLE_LINE_MIN_N", raising=False)
    a = mk()
    monkeypatch.setenv("RR_WHOLE_LINE_MIN_N", str(1 << 40))
    b = mk()
    a.reset()
    b.reset()
    ends = 0
    for t, act in enumerate(_actions(n, a.action_dim, 18, 13)):
        oa = [x.clone() for x in a.step(act)]
        ob = b.step(act)
        for x, y in zip(oa, ob):
            assert torch.equal(x, y), t
        assert torch.equal(a.terms, b.terms), t
        ia, toa, ra, la = a.fetch_done()
        ib, tob, rb, lb = b.fetch_done()
        np.testing.assert_array_equal(ia, ib)
        np.testing.assert_array_equal(toa, tob)
        np.testing.assert_array_equal(ra, rb)
        np.testing.assert_array_equal(la, lb)
        ends += len(ia)
    assert ends >= 2 * n  # every env ended at least twice (TimeLimit 7 over 18 steps)
    ca, cb = a.checkpoint(), b.checkpoint()
    for k in ca:
        assert torch.equal(ca[k], cb[k]), k


def test_seed_on_another_stream_waits_for_the_handles_launches():
    """steps of a handle queued on stream A, then rr_seed on stream B without any
    synchronise of the caller: the seed waits for the device (the handle's last launch went to
    another stream), so the queued steps read the OLD key — bitwise a twin that synchronised
    before seeding — and every later step the new one."""
    import torch
    from rl_rocket_amd.batch import RocketBatch

    n = 65536
    mk = lambda: RocketBatch(n, model=6, device="cuda:0", max_episode_steps=2, **_env6())  # noqa: E731
    a, b = mk(), mk()
    for e in (a, b):
        e.reset()
    acts = _actions(n, 3, 12, 8)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    sa.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(sa):
        for act in acts[:8]:  # TimeLimit 2: every env resets on every second step, keyed on the seed
            a.step(act)
    with torch.cuda.stream(sb):
        a.seed(4321)
    for act in acts[:8]:
        b.step(act)
    torch.cuda.synchronize()
    b.seed(4321)
    torch.cuda.current_stream().wait_stream(sa)
    for act in acts[8:]:
        a.step(act)
        b.step(act)
    torch.cuda.synchronize()
    assert torch.equal(a.obs, b.obs)
    for x, y in zip(a.get_state(), b.get_state()):
        assert torch.equal(x, y)


def test_seed_orders_after_every_stream_the_handle_used():
    """steps queued on stream A, then on stream B, then rr_seed on a third stream C with
    no synchronise by the caller: the key copy waits for the work of BOTH earlier streams (the
    per-handle event recorded on each), so every queued step reads the old key — bitwise a twin
    that synchronised before seeding — and every later step the new one."""
    import torch
    from rl_rocket_amd.batch import RocketBatch

    n = 65536
    mk = lambda: RocketBatch(n, model=6, device="cuda:0", max_episode_steps=2, **_env6())  # noqa: E731
    a, b = mk(), mk()
    for e in (a, b):
        e.reset()
    acts = _actions(n, 3, 16, 9)
    sa, sb, sc = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    sa.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(sa):
        for act in acts[:6]:
            a.step(act)
    sb.wait_stream(sa)
    with torch.cuda.stream(sb):
        for act in acts[6:12]:
            a.step(act)
    with torch.cuda.stream(sc):
        a.seed(987)
    for act in acts[:12]:
        b.step(act)
    torch.cuda.synchronize()
    b.seed(987)
    torch.cuda.current_stream().wait_stream(sb)
    for act in acts[12:]:
        a.step(act)
        b.step(act)
    torch.cuda.synchronize()
    assert torch.equal(a.obs, b.obs)
    for x, y in zip(a.get_state(), b.get_state()):
        assert torch.equal(x, y)


@pytest.mark.parametrize("integrator", ["rk4", "dopri5"])
@pytest.mark.parametrize("model", [6, 3])
def test_unaligned_obs_output_is_bitwise_the_aligned_one(model, integrator):
    """The obs rows go out through each wave's LDS tile as 16-B stores when the obs pointer is
    16-B aligned, else dword by dword (store_obs_tile; since round 5 also in the exact kernel).
    A twin env writing its obs 4 bytes off alignment, with a ragged last wave, must produce the
    same obs / reward / done bitwise at every step (auto-reset within the 40 steps)."""
    import torch

    from rl_rocket_amd.batch import RocketBatch

    n = 4096 + 37
    kw = _env6() if model == 6 else {}
    mk = lambda: RocketBatch(n, model=model, device="cuda:0", max_episode_steps=15, integrator=integrator,  # noqa: E731
                             **kw)
    a, b = mk(), mk()
    a.reset()
    b.reset()
    ns = a.state_dim
    raw = torch.empty((n * ns + 1,), dtype=torch.float32, device="cuda:0")
    obs_u = raw[1:].view(n, ns)
    assert obs_u.data_ptr() % 16 != 0
    out = (obs_u, torch.empty_like(b.reward), torch.empty_like(b.done), torch.empty_like(b.truncated))
    for act in _actions(n, a.action_dim, 40, 7):
        oa, ra, da, _ = a.step(act)
        ob, rb, db, _ = b.step(act, out=out)
        torch.cuda.synchronize()
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db)
    a.close()
    b.close()
