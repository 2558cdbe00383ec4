"""Host cost and device time of the step's launch paths at the bench workload.

    python tools/launch_cost.py [--n 65536]

For K = 20 and 2000: rr_step_repeat (K launches from one C call) and K RocketBatch.step
calls from Python — host seconds until the call(s) return, and the device time per launch by
HIP events on the launch stream.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    a = ap.parse_args()
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF

    dev = torch.device("cuda", 0)
    env = RocketBatch(a.n, model=6, device=dev, max_episode_steps=800, auto_reset=True, episode_stats=False,
                      **ENV_CONFIG_6DOF)
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    pool = torch.rand((8, a.n, 3), device=dev, generator=g) * 2 - 1
    out = {}
    for K in (20, 2000, 20):
        for how in ("repeat", "python"):
            env.step_repeat(pool, 10)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            t0 = time.perf_counter()
            if how == "repeat":
                env.step_repeat(pool, K)
            else:
                for k in range(K):
                    env.step(pool[k % 8])
            host = time.perf_counter() - t0
            e1.record()
            torch.cuda.synchronize()
            out["%s_k%d" % (how, K)] = {"host_us_per_launch": host * 1e6 / K,
                                       "dev_us_per_launch": e0.elapsed_time(e1) * 1e3 / K}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
