"""Where one headline step launch goes, per wave, from a diagnostic build of the step kernel
(RR_DIAG_STAMPS: s_memtime cycles by phase and the wave's s_memrealtime start / end, written over
the reward of the wave's first 6 envs; rocket_hip.hip step_kernel).

    RR_LIB_PATH=tools/ab/lib_sstamps.so python tools/step_stamps.py [--n 65536] --out F

Phases per main wave: 0 kernel entry -> after the workgroup barrier (helper-wave kernels), 1 ->
the state planes landed, 2 the step's compute (integration, event, reward, obs), 3 the tail (done
compaction, terminal rows / reset, every output store issued). From the 100 MHz real-time clock:
the spread of the waves' start times (dispatch ramp) and of their end times (the launch ends with
the last wave's stores). Fresh phase (steps 6-25 after a reset, the driver's protocol) and steady
state (after 150 steps), each over `--reps` launches.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["entry->barrier", "->state landed", "compute", "tail (outputs issued)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out")
    a = ap.parse_args()
    import numpy as np
    import torch

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF, MAX_EPISODE_STEPS

    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(42)
    pool = torch.rand((8, a.n, 3), device=dev, generator=gen) * 2 - 1
    out = {"n": a.n, "what": __doc__.strip().splitlines()[0], "phases": {}}
    for phase, warm in (("fresh", 5), ("steady", 150)):
        env = RocketBatch(a.n, model=6, device=dev, max_episode_steps=MAX_EPISODE_STEPS, auto_reset=True,
                          episode_stats=False, **ENV_CONFIG_6DOF)
        env.reset()
        for t in range(warm):
            env.step(pool[t % 8])
        cyc, st, en = [], [], []
        for t in range(a.reps):
            _, rew, _, _ = env.step(pool[(warm + t) % 8])
            torch.cuda.synchronize(dev)
            w = a.n // 64
            r = rew.detach().cpu().numpy()[: w * 64].reshape(w, 64)
            cyc.append(r[:, :4].astype(np.float64))
            bits = r[:, 4:6].copy().view(np.uint32).astype(np.int64)
            st.append(bits[:, 0] - bits[:, 0].min())
            en.append(bits[:, 1] - bits[:, 0].min())
        x = np.concatenate(cyc)
        s_, e_ = np.concatenate(st), np.concatenate(en)
        d = {"waves_x_reps": int(x.shape[0]), "cycles": {}}
        for p, name in enumerate(PHASES):
            d["cycles"][name] = {"median": float(np.median(x[:, p])), "p90": float(np.percentile(x[:, p], 90)),
                                 "max": float(x[:, p].max())}
        # 100 MHz ticks -> us, relative to the earliest wave start of the same launch
        d["start_spread_us"] = {"median": float(np.median(s_)) / 100.0, "p90": float(np.percentile(s_, 90)) / 100.0,
                                "max": float(s_.max()) / 100.0}
        d["end_us"] = {"median": float(np.median(e_)) / 100.0, "p90": float(np.percentile(e_, 90)) / 100.0,
                       "max": float(e_.max()) / 100.0}
        out["phases"][phase] = d
        print("[%s]" % phase)
        for name, v in d["cycles"].items():
            print("  %-24s median %7.0f  p90 %7.0f  max %7.0f cycles" % (name, v["median"], v["p90"], v["max"]))
        print("  wave start after the first: median %.2f  p90 %.2f  max %.2f us" % (
            d["start_spread_us"]["median"], d["start_spread_us"]["p90"], d["start_spread_us"]["max"]))
        print("  wave end after the first start: median %.2f  p90 %.2f  max %.2f us" % (
            d["end_us"]["median"], d["end_us"]["p90"], d["end_us"]["max"]))
        env.close()
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
