"""Bitwise comparison of two builds' exact-mode outputs (RR_INT_DOPRI5): a candidate that only
reorders independent per-component arithmetic must reproduce the shipped kernel's every bit.

    python tools/exact_bitwise_ab.py --libs tree,tools/ab/lib_x.so [--n 65536] [--steps 30] --out F

Each library runs in its own process (RR_LIB_PATH): 6DOF and 3DOF, seeded rows with ground events
(tests/test_gpu_parity.py's generators) stepped once, then `--steps` auto-reset steps of a batch
under TimeLimit 40 from seeded random actions; every output (obs, reward, done, truncated, terms,
fp64 / fp32 state, counters) is saved and compared with numpy.array_equal (NaN == NaN).
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_one(out, n, steps, lean):
    import numpy as np
    import torch

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, ROOT)
    from test_gpu_parity import _random_states3, _random_states6

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF

    if lean:
        os.environ["RR_EXACT_LEAN_MIN_N"] = "0"
    res = {}
    for model in (6, 3):
        kw = ENV_CONFIG_6DOF if model == 6 else {}
        ic, s, a = (_random_states6 if model == 6 else _random_states3)(n, seed=31)
        b = RocketBatch(n, model=model, device="cuda:0", integrator="dopri5", max_episode_steps=0, auto_reset=False,
                        episode_stats=False, compute_terms=True, **kw)
        v0 = np.sqrt((ic[:, 3:6 if model == 6 else 5] ** 2).sum(1, dtype=np.float32)).astype(np.float32)
        b.set_state64(torch.from_numpy(np.ascontiguousarray(s.T)), v0=torch.from_numpy(v0),
                      elapsed=torch.zeros(n, dtype=torch.int32))
        obs, rew, done, _ = b.step(torch.from_numpy(a.astype(np.float32)))
        torch.cuda.synchronize()
        for k, v in (("obs", obs), ("rew", rew), ("done", done), ("terms", b.terms)):
            res["rows%d_%s" % (model, k)] = v.cpu().numpy()
        res["rows%d_state64" % model] = b.get_state64()[0].cpu().numpy()
        b.close()
        b = RocketBatch(20003, model=model, device="cuda:0", integrator="dopri5", max_episode_steps=40,
                        auto_reset=True, compute_terms=True, **kw)
        b.reset()
        g = torch.Generator(device="cuda:0").manual_seed(7)
        for t in range(steps):
            act = torch.rand((20003, b.action_dim), device="cuda:0", generator=g) * 2 - 1
            obs, rew, done, trunc = b.step(act)
            for k, v in (("obs", obs), ("rew", rew), ("done", done), ("trunc", trunc), ("terms", b.terms)):
                res["traj%d_t%d_%s" % (model, t, k)] = v.cpu().numpy()
        st64, v0_, cw = b.get_state64()
        res["traj%d_state64" % model] = st64.cpu().numpy()
        res["traj%d_cw" % model] = cw.cpu().numpy()
        b.close()
    np.savez(out, **res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs")
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--lean", action="store_true")
    ap.add_argument("--one")
    ap.add_argument("--out")
    a = ap.parse_args()
    if a.one:
        run_one(a.one, a.n, a.steps, a.lean)
        return
    import numpy as np

    files = []
    with tempfile.TemporaryDirectory() as d:
        for k, lib in enumerate(a.libs.split(",")):
            env = dict(os.environ)
            if lib != "tree":
                env["RR_LIB_PATH"] = os.path.abspath(lib)
            f = os.path.join(d, "o%d.npz" % k)
            subprocess.check_call([sys.executable, os.path.abspath(__file__), "--one", f, "--n", str(a.n), "--steps",
                                   str(a.steps)] + (["--lean"] if a.lean else []), env=env)
            files.append(f)
        x, y = np.load(files[0]), np.load(files[1])
        diff = [k for k in x.files if not np.array_equal(x[k], y[k], equal_nan=x[k].dtype.kind == "f")]
    out = {"libs": a.libs, "n": a.n, "steps": a.steps, "lean": a.lean, "arrays": len(x.files), "differ": diff,
           "bitwise": not diff}
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    sys.exit(0 if not diff else 1)


if __name__ == "__main__":
    main()
