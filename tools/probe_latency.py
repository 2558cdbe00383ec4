"""Host-side latency of the short paths (diagnostic, not part of the product):

A. the driver's headline protocol (N = 65 536, K = 20 direct launches): where the wall clock's
   fixed cost beyond K x the per-launch device time goes — the benchmark gate (tools/
   libbench_timed.so), the first submission, the closing synchronize — against K direct launches
   from one C call with no gate (rr_step_repeat) and a Python loop of rr_step;
B. the single-env gym shim (N = 1): its step as it stands, against leaner forms (pinned zero-copy
   action / outputs, one copy of the state, one synchronize) and the bare launch + synchronize.

Prints one JSON line. Run it under different host-wait settings in separate processes (the HIP
runtime reads them at start-up)."""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from rl_rocket_amd.batch import RocketBatch  # noqa: E402
from rl_rocket_amd.envs import Rocket6DOF  # noqa: E402
from rl_rocket_amd.params import ENV_CONFIG_6DOF, MAX_EPISODE_STEPS  # noqa: E402


def med(xs):
    return round(statistics.median(xs), 2)


def part_a(dev, reps=30, K=20):
    n = 65536
    env = RocketBatch(n, model="6DOF", device=dev, max_episode_steps=MAX_EPISODE_STEPS, auto_reset=True,
                      episode_stats=False, **ENV_CONFIG_6DOF)
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    pool = torch.rand((8, n, 3), device=dev, generator=g) * 2 - 1
    loop = bench.TimedLoop(env)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    ev1.record()
    fn, fargs = loop.call(pool, 5, (ev0, ev1))
    fn(*fargs)
    torch.cuda.synchronize()
    out = {}
    for name in ("gate", "repeat", "pyloop", "gate", "repeat", "pyloop"):
        rows = []
        for _ in range(reps):
            torch.cuda.synchronize()
            if name == "gate":
                fn, fargs = loop.call(pool, K, (ev0, ev1))
                t0 = time.perf_counter()
                fn(*fargs)
            elif name == "repeat":
                t0 = time.perf_counter()
                ev0.record()
                env.step_repeat(pool, K)
                ev1.record()
            else:
                t0 = time.perf_counter()
                ev0.record()
                for k in range(K):
                    env.step(pool[k % 8])
                ev1.record()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            rows.append(((t2 - t0) * 1e6, (t1 - t0) * 1e6, ev0.elapsed_time(ev1) * 1e3))
        out[name] = {"wall_us": med([r[0] for r in rows]), "wall_min_us": round(min(r[0] for r in rows), 2),
                     "submit_us": med([r[1] for r in rows]), "events_us": med([r[2] for r in rows]),
                     "wall_minus_events_us": med([r[0] - r[2] for r in rows]),
                     "per_step_wall_us": round(med([r[0] for r in rows]) / K, 3),
                     "per_step_events_us": round(med([r[2] for r in rows]) / K, 3)}
    # host time of ONE rr_step call on an idle queue (ctypes call + launch), and of 20 back to back
    P = __import__("ctypes").c_void_p
    lib, h, sp = env.lib, env._h, P(torch.cuda.current_stream(dev).cuda_stream)
    args = [P(pool[0].data_ptr()), P(env.obs.data_ptr()), P(env.reward.data_ptr()), P(env.done.data_ptr()),
            P(env.truncated.data_ptr()), None, sp]
    one = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lib.rr_step(h, *args)
        one.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize()
    out["rr_step_call_idle_queue_us"] = med(one)
    env.close()
    return out


def part_b(dev, steps=2000):
    rng = np.random.default_rng(0)
    acts = rng.uniform(-1, 1, (256, 3)).astype(np.float32)
    res = {}

    # 1. the shim as it stands
    env = Rocket6DOF(device=dev, **ENV_CONFIG_6DOF)
    env.reset()
    for k in range(50):
        if env.step(acts[k % 256])[2]:
            env.reset()
    t0 = time.perf_counter()
    for k in range(steps):
        if env.step(acts[k % 256])[2]:
            env.reset()
    res["shim_us"] = round((time.perf_counter() - t0) / steps * 1e6, 2)
    env.close()
    from rl_rocket_amd.envs import Rocket

    env = Rocket(device=dev)
    env.reset()
    t0 = time.perf_counter()
    for k in range(steps):
        if env.step(acts[k % 256][:2])[2]:
            env.reset()
    res["shim3_us"] = round((time.perf_counter() - t0) / steps * 1e6, 2)
    env.close()

    b = RocketBatch(1, model="6DOF", device=dev, max_episode_steps=0, auto_reset=False, episode_stats=False,
                    compute_terms=True, **ENV_CONFIG_6DOF)
    b.reset()
    pin = dict(pin_memory=True)
    a_h = torch.empty((1, 3), dtype=torch.float32, **pin)
    obs_h = torch.empty((1, 14), dtype=torch.float32, **pin)
    rew_h = torch.empty((1,), dtype=torch.float32, **pin)
    done_h = torch.empty((1,), dtype=torch.uint8, **pin)
    tr_h = torch.empty((1,), dtype=torch.uint8, **pin)
    terms_h = torch.empty((b.n_terms + 2, 1), dtype=torch.float32, **pin)
    st_d = torch.empty((14, 1), dtype=torch.float32, device=dev)
    st_h = torch.empty((14, 1), dtype=torch.float32, **pin)
    import ctypes

    P = ctypes.c_void_p
    lib = b.lib
    s = torch.cuda.current_stream(dev)
    sp = P(s.cuda_stream)

    def step_zero_copy(k, sync):
        np.copyto(a_h.numpy(), acts[k % 256].reshape(1, 3))
        lib.rr_step(b._h, P(a_h.data_ptr()), P(obs_h.data_ptr()), P(rew_h.data_ptr()), P(done_h.data_ptr()),
                    P(tr_h.data_ptr()), P(terms_h.data_ptr()), sp)
        lib.rr_get_state(b._h, P(st_d.data_ptr()), None, None, sp)
        st_h.copy_(st_d, non_blocking=True)
        sync()

    def step_bare(k, sync):
        lib.rr_step(b._h, P(a_h.data_ptr()), P(obs_h.data_ptr()), P(rew_h.data_ptr()), P(done_h.data_ptr()),
                    P(tr_h.data_ptr()), P(terms_h.data_ptr()), sp)
        sync()

    def poll():
        while not s.query():
            pass

    syncs = {"stream_sync": s.synchronize, "device_sync": torch.cuda.synchronize, "poll_query": poll}
    for fname, f in (("zero_copy_state_copy", step_zero_copy), ("bare_launch", step_bare)):
        for sname, sy in syncs.items():
            for k in range(50):
                f(k, sy)
            b.reset()
            t0 = time.perf_counter()
            for k in range(steps):
                f(k, sy)
                if k % 200 == 199:
                    b.reset()
            res["%s__%s_us" % (fname, sname)] = round((time.perf_counter() - t0) / steps * 1e6, 2)
    # an empty device op + sync: the floor of one host round trip
    for sname, sy in syncs.items():
        x = torch.empty(1, device=dev)
        t0 = time.perf_counter()
        for k in range(steps):
            x.fill_(1.0)
            sy()
        res["fill_then_%s_us" % sname] = round((time.perf_counter() - t0) / steps * 1e6, 2)
    b.close()
    return res


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    env_knobs = {k: os.environ.get(k) for k in ("ROC_ACTIVE_WAIT_TIMEOUT", "HSA_ENABLE_INTERRUPT")}
    out = {"knobs": env_knobs, "headline_k20": part_a(dev), "single_env": part_b(dev)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
