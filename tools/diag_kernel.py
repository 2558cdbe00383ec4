"""Step-kernel N sweep on the GPU box (and the timing child of tools/ab_kernel.py).

    python tools/diag_kernel.py [--ns 4096,65536,...] [--model 6] [--lib path/to/librocket_hip.so]

Each N runs in its own child process (librocket_hip.so is loaded once per process;
RR_LIB_PATH selects the build). Timing = HIP events around graph replays of 64
back-to-back step launches on the launch stream. Prints one JSON line per run. (The
round-1 ablation builds, RR_DIAG, were removed from the product source in round 2; they
live in the git history, DESIGN.md §3 keeps their numbers.)
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(args):
    import torch

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF

    dev = torch.device("cuda", 0)
    kw = ENV_CONFIG_6DOF if args.model == 6 else {}
    env = RocketBatch(args.n, model=args.model, device=dev, max_episode_steps=800, auto_reset=True,
                      episode_stats=False, integrator=args.integrator, **kw)
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    pool = torch.rand((8, args.n, env.action_dim), device=dev, generator=g) * 2 - 1
    for k in range(30):
        env.step(pool[k % 8])
    torch.cuda.synchronize()
    gs = 64
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            for k in range(gs):
                env.step(pool[k % 8])
    torch.cuda.current_stream().wait_stream(s)
    graph.replay()
    torch.cuda.synchronize()
    reps = max(2, int(args.steps // gs))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(reps):
        graph.replay()
    e1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    us = e0.elapsed_time(e1) * 1e3 / (reps * gs)
    bpe = 189 if args.model == 6 else 101
    print(json.dumps({"variant": args.tag, "model": args.model, "n": args.n, "us_per_step": us,
                      "wall_us_per_step": wall * 1e6 / (reps * gs),
                      "Gsteps_per_s": args.n / us / 1e3, "GBps_alg": args.n * bpe / us / 1e3}), flush=True)
    env.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--tag", default="")
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--ns", default="4096,16384,65536,262144,524288,1048576,4194304")
    ap.add_argument("--lib", default=os.path.join(ROOT, "rl_rocket_amd", "librocket_hip.so"))
    ap.add_argument("--model", type=int, default=6)
    ap.add_argument("--integrator", default="rk4")
    ap.add_argument("--steps", type=int, default=2048)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "diag"))
    args = ap.parse_args()
    if args.child:
        return child(args)
    for n in [int(x) for x in args.ns.split(",")]:
        env = dict(os.environ, RR_LIB_PATH=os.path.abspath(args.lib))
        cmd = [sys.executable, __file__, "--child", "--tag", os.path.basename(args.lib), "--n", str(n), "--model",
               str(args.model), "--integrator", args.integrator, "--steps", str(args.steps)]
        r = subprocess.run(cmd, env=env, timeout=300)
        if r.returncode != 0:
            print(json.dumps({"n": n, "error": r.returncode}), flush=True)
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
