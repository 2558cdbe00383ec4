"""RocketVecEnv host path (numpy in / out, Monitor on, N = 65 536): the per-step cost split
(launch / kernel / d2h / infos, RocketVecEnv.timing) in windows of 25 steps over 400 steps, to see
whether the "kernel" share (action H2D + step, device time after the host returns) depends on the
episode phase. Also the H2D of one action batch alone, timed by HIP events."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rl_rocket_amd.params import ENV_CONFIG_6DOF, MAX_EPISODE_STEPS  # noqa: E402
from rl_rocket_amd.vec_env import RocketVecEnv  # noqa: E402


def main():
    n, dev = 65536, "cuda:0"
    rng = np.random.default_rng(0)
    pool = [rng.uniform(-1, 1, (n, 3)).astype(np.float32) for _ in range(8)]
    venv = RocketVecEnv(n, model="6DOF", device=dev, max_episode_steps=MAX_EPISODE_STEPS, monitor=True,
                        **ENV_CONFIG_6DOF)
    venv.reset()
    # per step for the first 120 steps: device time of (action upload + rr_step) by HIP events
    # around batch.step, and the host's synchronize wait after it (the "kernel" split)
    orig = venv.batch.step
    ev = []

    def wrapped(action, out=None):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = orig(action, out=out)
        e1.record()
        ev.append((e0, e1))
        return r

    venv.batch.step = wrapped
    per = []
    for k in range(120):
        venv.timing = {}
        t0 = time.perf_counter()
        _, _, d, _ = venv.step(pool[k % 8])
        wall = time.perf_counter() - t0
        torch.cuda.synchronize()
        e0, e1 = ev[-1]
        per.append((k, round(e0.elapsed_time(e1) * 1e3, 1), round(venv.timing["kernel"] * 1e6, 1),
                    round(wall * 1e6, 1), int(d.sum())))
    venv.batch.step = orig
    print(json.dumps({"step_device_us__sync_wait_us__wall_us__done": per}), flush=True)
    rows = []
    for w in range(16):
        venv.timing = {}
        done = 0
        t0 = time.perf_counter()
        for k in range(25):
            _, _, d, _ = venv.step(pool[k % 8])
            done += int(d.sum())
        dt = time.perf_counter() - t0
        rows.append({"window": w, "us_per_step": dt / 25 * 1e6, "done_per_step": done / 25,
                     **{k: round(v / 25 * 1e6, 1) for k, v in venv.timing.items()}})
        print(json.dumps(rows[-1]), flush=True)
    # the action upload alone (pinned staging + async copy), events on the current stream
    a = torch.empty((n, 3), dtype=torch.float32, device=dev)
    pin = torch.empty((n, 3), dtype=torch.float32, pin_memory=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        a.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(20):
        a.copy_(pin, non_blocking=True)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"h2d_786KB_us": e0.elapsed_time(e1) * 1e3 / 20}))
    venv.close()


if __name__ == "__main__":
    main()
