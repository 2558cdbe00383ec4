"""Phase breakdown of the PPO gradient kernel (ppo_grad_kernel) from a diagnostic build
(RR_DIAG_STAMPS: per-wave s_memtime cycles of 12 phases, the tile-loop phases summed over the
wave's tiles; rocket_ppo.inc). The kernel writes them past the packed tower images, so this tool
enlarges PPOGrad's workspace by that much.

    RR_LIB_PATH=tools/ab/lib_stamps.so python tools/ppo_stamps.py [--n 65536] --out F
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["start(staging,adv stats)", "gather wait + x^T", "forward towers", "heads + loss derivs",
          "h2/DM -> LDS + dpre2", "head grads", "dpre2/h1 -> LDS", "dh1 MFMAs", "db2 + dW2 MFMAs",
          "dpre1 -> LDS", "dW1 MFMAs", "epilogue(reduce,write)"]
KADVPART, WAVES = 256, 4


def main():
    import numpy as np
    import torch

    from rl_rocket_amd import _lib
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF, MAX_EPISODE_STEPS
    from rl_rocket_amd.rollout import DeviceRollout, MlpActorCritic, PPOGrad

    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--out")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    env = RocketBatch(a.n, model=6, device=dev, max_episode_steps=MAX_EPISODE_STEPS, auto_reset=True,
                      episode_stats=False, **ENV_CONFIG_6DOF)
    pol = MlpActorCritic(14, 3).to(dev)
    ro = DeviceRollout(env, pol, n_steps=a.steps)
    for _ in range(2):
        ro.collect()
    bs = a.n
    g = PPOGrad(pol, ro, bs)
    nwg = min(128, max(1, ((bs + 31) // 32 + WAVES - 1) // WAVES))
    pf = 6412
    pack = (g._nbytes - 2 * KADVPART * 8) // 4 // 2 - nwg * pf
    base = 2 * KADVPART * 2 + 2 * nwg * pf + 2 * pack  # floats: adv partials (doubles) | parts | packs
    extra = 2 * nwg * WAVES * 16
    g.ws = torch.zeros(base + extra + 64, dtype=torch.float32, device=dev)
    g._nbytes = g.ws.numel() * 4
    perm = torch.randperm(a.n * a.steps, device=dev)
    for k in range(4):
        g(perm[k * bs:(k + 1) * bs].contiguous())
    torch.cuda.synchronize()
    st = g.ws[base:base + extra].view(2, nwg, WAVES, 16)[..., :12].cpu().numpy()
    out = {"n": a.n, "batch": bs, "workgroups_per_tower": nwg, "tiles_per_wave": (bs // 32) // (nwg * WAVES),
           "phases": {}}
    for tw, name in ((0, "pi"), (1, "vf")):
        x = st[tw].reshape(-1, 12)
        tot = np.median(x.sum(1))
        out["phases"][name] = {p: {"median": float(np.median(x[:, i])), "p90": float(np.percentile(x[:, i], 90)),
                                   "share": float(np.median(x[:, i]) / tot)} for i, p in enumerate(PHASES)}
        out["phases"][name]["total_median"] = float(tot)
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    env.close()


if __name__ == "__main__":
    main()
