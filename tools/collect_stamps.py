"""Phase breakdown of the one-launch rollout collect from a diagnostic build (RR_DIAG_STAMPS:
per-wave s_memtime cycles of each phase summed over the n_steps of one collect, written over
last_value[wave's first 16 envs]; rocket_rollout.inc).

    RR_LIB_PATH=tools/ab/lib_stamps.so python tools/collect_stamps.py [--n 65536] [--warm 20] --out F

Runs the bench's rollout setup (6DOF, N envs, fp32 towers, n_steps 16), `--warm` collects to
reach steady state (episodes ending), then `--reps` collects, each read back: per phase the
median and p90 over waves of the cycles per step, and the share of the wave's total.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["obs", "vf_l1", "vf_act1", "vf_l2", "vf_act2+head", "pi_l1", "pi_act1", "pi_l2", "pi_act2+heads",
          "sample", "env_step", "bootstrap", "done+reset", "stores", "end(state,V,GAE)", "start(loads,staging)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--warm", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--out")
    a = ap.parse_args()
    import numpy as np
    import torch

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF, MAX_EPISODE_STEPS
    from rl_rocket_amd.rollout import DeviceRollout, MlpActorCritic

    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    env = RocketBatch(a.n, model=6, device=dev, max_episode_steps=MAX_EPISODE_STEPS, auto_reset=True,
                      episode_stats=False, **ENV_CONFIG_6DOF)
    pol = MlpActorCritic(env.state_dim, env.action_dim).to(dev)
    ro = DeviceRollout(env, pol, n_steps=16, fused=True, policy_dtype=a.dtype, one_launch=True)
    for _ in range(a.warm):
        ro.collect()
    torch.cuda.synchronize(dev)
    waves = a.n // 64
    reps = []
    for _ in range(a.reps):
        ro.collect()
        torch.cuda.synchronize(dev)
        lv = ro.last_value.detach().cpu().numpy()[: waves * 64].reshape(waves, 64)[:, :16].astype(np.float64)
        reps.append(lv / 16.0)  # cycles per step
    x = np.concatenate(reps, axis=0)
    tot = x.sum(axis=1)
    out = {"n": a.n, "dtype": a.dtype, "warm_collects": a.warm, "waves_x_reps": int(x.shape[0]),
           "what": "s_memtime cycles per step per wave (phases end/start/total per collect / 16)",
           "total_median": float(np.median(tot)), "total_p90": float(np.percentile(tot, 90)), "phases": {}}
    for p, name in enumerate(PHASES):
        out["phases"][name] = {"median": float(np.median(x[:, p])), "p90": float(np.percentile(x[:, p], 90)),
                               "mean": float(x[:, p].mean()), "share_of_mean_total": float(x[:, p].mean() / tot.mean())}
    for name, d in out["phases"].items():
        print("%-22s median %9.1f  p90 %9.1f  mean %9.1f  %5.1f %%" % (name, d["median"], d["p90"], d["mean"],
                                                                     100 * d["share_of_mean_total"]))
    print("total median %.1f p90 %.1f cycles per step" % (out["total_median"], out["total_p90"]))
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
