"""Phase breakdown of one exact-mode step (RR_INT_DOPRI5) from a diagnostic build (RR_DIAG_STAMPS:
per-wave s_memtime cycles, written over the reward of the wave's first 4 envs; rocket_dopri5.inc).

    RR_LIB_PATH=tools/ab/lib_xstamps.so python tools/exact_stamps.py [--n 65536] --out F

Phases: 0 kernel start -> state loaded (and the control denormalised), 1 the adaptive RK45 loop,
2 finish / reward / obs / terminal rows, 3 the output stores issued. Median / p90 over waves of
`--reps` steps after `--warm` steps (episodes under way).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["start->state loaded", "adaptive loop", "finish/reward/obs", "stores issued"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--warm", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out")
    a = ap.parse_args()
    import numpy as np
    import torch

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF, MAX_EPISODE_STEPS

    dev = torch.device("cuda", 0)
    env = RocketBatch(a.n, model=6, device=dev, max_episode_steps=MAX_EPISODE_STEPS, auto_reset=True,
                      episode_stats=False, integrator="dopri5", **ENV_CONFIG_6DOF)
    env.reset()
    gen = torch.Generator(device=dev).manual_seed(42)
    pool = torch.rand((8, a.n, 3), device=dev, generator=gen) * 2 - 1
    for t in range(a.warm):
        env.step(pool[t % 8])
    rows = []
    for t in range(a.reps):
        _, rew, _, _ = env.step(pool[(a.warm + t) % 8])
        torch.cuda.synchronize(dev)
        w = a.n // 64
        rows.append(rew.detach().cpu().numpy()[: w * 64].reshape(w, 64)[:, :4].astype(np.float64))
    x = np.concatenate(rows)
    tot = x.sum(axis=1)
    out = {"n": a.n, "waves_x_reps": int(x.shape[0]), "what": __doc__.strip().splitlines()[0],
           "total_median": float(np.median(tot)), "total_p90": float(np.percentile(tot, 90)), "phases": {}}
    for p, name in enumerate(PHASES):
        out["phases"][name] = {"median": float(np.median(x[:, p])), "p10": float(np.percentile(x[:, p], 10)),
                               "p90": float(np.percentile(x[:, p], 90)), "p99": float(np.percentile(x[:, p], 99)),
                               "max": float(x[:, p].max())}
        print("%-22s median %8.0f  p10 %8.0f  p90 %8.0f  max %8.0f" % (
            name, out["phases"][name]["median"], out["phases"][name]["p10"], out["phases"][name]["p90"],
            out["phases"][name]["max"]))
    # the launch is set by its slowest wave: per step, the slowest wave's total and where it went
    w = a.n // 64
    per_step = x.reshape(a.reps, w, 4)
    slow = per_step.sum(axis=2).argmax(axis=1)
    out["slowest_wave_per_step"] = [[float(v) for v in per_step[r, slow[r]]] for r in range(a.reps)]
    out["cp_max"] = os.environ.get("RR_EXACT_CP_MAX")
    print("slowest wave per step (phases, cycles):", out["slowest_wave_per_step"])
    print("total median %.0f p90 %.0f cycles" % (out["total_median"], out["total_p90"]))
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
