"""A/B of the graphed fused PPO update at configs[4] (N = 65 536, n_steps 16, batch_size N: 16
minibatches per epoch): the chained whole-minibatch call (rr_ppo_update, three launches per
minibatch) against rr_ppo_grad + rr_clip_adam (five), same library, interleaved, HIP events.

    python tools/ppo_chain_ab.py [--n 65536] [--reps 3] [--out F]
"""
import argparse
import copy
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import rl_rocket_amd.rollout as R
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF, MAX_EPISODE_STEPS

    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    env = RocketBatch(a.n, model=6, device=dev, max_episode_steps=MAX_EPISODE_STEPS, auto_reset=True,
                      episode_stats=False, **ENV_CONFIG_6DOF)
    pol = R.MlpActorCritic(14, 3).to(dev)
    ro = R.DeviceRollout(env, pol, n_steps=a.steps)
    for _ in range(2):
        ro.collect()
    pols = {k: copy.deepcopy(pol) for k in ("chain", "two_calls")}
    opts = {k: torch.optim.Adam(p.parameters(), lr=3e-4, eps=1e-5, capturable=True) for k, p in pols.items()}
    ups = {"chain": R.GraphedPPOUpdate(pols["chain"], opts["chain"], ro, batch_size=a.n, fused=True)}
    keep = R.PPOUpdate
    R.PPOUpdate = lambda *args, **kw: None  # GraphedPPOUpdate then takes rr_ppo_grad + rr_clip_adam
    try:
        ups["two_calls"] = R.GraphedPPOUpdate(pols["two_calls"], opts["two_calls"], ro, batch_size=a.n, fused=True)
    finally:
        R.PPOUpdate = keep
    assert ups["chain"]._update is not None and ups["two_calls"]._update is None
    res = {k: [] for k in ups}
    for k, u in ups.items():
        u.update(n_epochs=1)
    for _ in range(a.reps):
        for k, u in ups.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            e0.record()
            u.update(n_epochs=10)
            e1.record()
            torch.cuda.synchronize(dev)
            res[k].append(e0.elapsed_time(e1) / 10)
    mb = a.n * a.steps // a.n
    out = {"n": a.n, "minibatches_per_epoch": mb, "epoch_ms": res,
           "us_per_minibatch": {k: [round(v * 1e3 / mb, 2) for v in vs] for k, vs in res.items()}}
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    env.close()


if __name__ == "__main__":
    main()
