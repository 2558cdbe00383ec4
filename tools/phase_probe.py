"""Step time against episode phase (measurement only): N envs from one reset, stepped back to back
with the bench's seeded action pool; per block of B steps the HIP-event time per step and the
fraction of envs done in the block. Separates the cost of the auto-reset path (done lanes) from
clock changes under sustained load: the same run with auto-reset and TimeLimit off has no done
lanes after the first episode end.

    python tools/phase_probe.py --n 4194304 --steps 400 --block 20 [--no-reset] [--out FILE]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4194304)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--block", type=int, default=20)
    ap.add_argument("--no-reset", action="store_true", help="auto-reset and TimeLimit off")
    ap.add_argument("--out")
    a = ap.parse_args()
    import torch

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF, MAX_EPISODE_STEPS

    dev = torch.device("cuda", 0)
    env = RocketBatch(a.n, model=6, device=dev, max_episode_steps=0 if a.no_reset else MAX_EPISODE_STEPS,
                      auto_reset=not a.no_reset, episode_stats=False, **ENV_CONFIG_6DOF)
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    pool = torch.rand((8, a.n, 3), device=dev, generator=g) * 2 - 1
    # one hipGraph of `block` steps, replayed back to back: no host gaps at any N
    stream = torch.cuda.current_stream(dev)
    out = {}
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(dev)
    s.wait_stream(stream)
    with torch.cuda.stream(s):
        with torch.cuda.graph(gr, stream=s):
            for k in range(a.block):
                out["done"] = env.step(pool[k % 8])[2]
    stream.wait_stream(s)
    torch.cuda.synchronize(dev)
    rows = []
    for b0 in range(0, a.steps, a.block):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        gr.replay()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        rows.append({"step": b0, "us_per_step": e0.elapsed_time(e1) / a.block * 1e3,
                     "done_frac_last_step": float(out["done"].sum().item()) / a.n})
        print(json.dumps(rows[-1]), flush=True)
    env.close()
    res = {"n": a.n, "no_reset": a.no_reset, "block": a.block, "rows": rows}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
