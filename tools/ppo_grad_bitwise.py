"""Bitwise comparison of two builds' PPO learner outputs: rr_ppo_grad gradients and statistics for
a few minibatches of a configs[4]-shaped rollout, each library in its own process (RR_LIB_PATH).

    python tools/ppo_grad_bitwise.py --libs tree,tools/ab/lib_x.so [--n 16384] --out F
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_one(out, n):
    import numpy as np
    import torch

    sys.path.insert(0, ROOT)
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF
    from rl_rocket_amd.rollout import DeviceRollout, MlpActorCritic, PPOGrad

    env = RocketBatch(n, model=6, device="cuda:0", max_episode_steps=30, **ENV_CONFIG_6DOF)
    torch.manual_seed(11)
    pol = MlpActorCritic(14, 3).cuda()
    ro = DeviceRollout(env, pol, n_steps=8, seed=4)
    ro.collect()
    g = PPOGrad(pol, ro, n)
    perm = torch.randperm(n * 8, device="cuda:0", generator=torch.Generator("cuda:0").manual_seed(3))
    res = {}
    for k in range(4):
        st = g(perm[k * n:(k + 1) * n].contiguous())
        torch.cuda.synchronize()
        for i, p in enumerate(g.params):
            res["mb%d_g%d" % (k, i)] = p.grad.cpu().numpy()
        res["mb%d_stats" % k] = st.cpu().numpy()
    np.savez(out, **res)
    env.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs")
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--one")
    ap.add_argument("--out")
    a = ap.parse_args()
    if a.one:
        run_one(a.one, a.n)
        return
    import numpy as np

    files = []
    with tempfile.TemporaryDirectory() as d:
        for k, lib in enumerate(a.libs.split(",")):
            env = dict(os.environ)
            if lib != "tree":
                env["RR_LIB_PATH"] = os.path.abspath(lib)
            f = os.path.join(d, "o%d.npz" % k)
            subprocess.check_call([sys.executable, os.path.abspath(__file__), "--one", f, "--n", str(a.n)], env=env)
            files.append(f)
        x, y = np.load(files[0]), np.load(files[1])
        diff = [k for k in x.files if not np.array_equal(x[k], y[k])]
    out = {"libs": a.libs, "n": a.n, "arrays": len(x.files), "differ": diff, "bitwise": not diff}
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    sys.exit(0 if not diff else 1)


if __name__ == "__main__":
    main()
