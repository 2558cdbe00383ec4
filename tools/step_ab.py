"""A/B timing of step-kernel builds: the production library against diagnostic and candidate
builds (libraries under tools/ab/, built beforehand in this container with
rl_rocket_amd.build.build_lib(out, defines=[...]) from edited copies of the sources). The round-5
apportionment's RR_DIAG_NO_* / RR_AB_* variants were deleted from csrc/ in round 6 (they live in
git history at 1ad310c); only RR_DIAG_STAMPS (rocket_stamps.h) stays in the source.

    python tools/step_ab.py run --libs base,d_notrans,ab_reward2 [--reps 2] [--n 65536] --out FILE
    python tools/step_ab.py one --lib tools/ab/lib_base.so [--n 65536]      (one library, one process)

`one` measures, in a fresh process that loads the library through RR_LIB_PATH, the headline step
(6DOF RK4, auto-reset, TimeLimit 800, N envs, the bench's 8-batch action pool) as 20-launch
hipGraph replays timed by HIP events, in two phases of an episode:
  * fresh: steps 6-25 after a reset (the driver's bench protocol: warm-up 5, K = 20) — no env ends
    an episode yet, so no lane takes the ground-event or done path;
  * steady: steps 151-170 (~1.5 % of the envs end an episode per step: event and done paths live).
Before every replay the env is restored from a checkpoint taken at the phase start (outside the
timed region), so every replay times the same 20 steps; the per-launch figure is the median over
`--replays` replays (p10 / p90 beside it). `run` calls `one` for every library, interleaved over
`--reps` rounds (ABC ABC) so that clock drift spreads over all of them, and prints one table.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(a):
    import torch

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF, MAX_EPISODE_STEPS

    dev = torch.device("cuda", 0)
    n, K = a.n, 20
    gen = torch.Generator(device=dev).manual_seed(42)
    pool = torch.rand((8, n, 3), device=dev, generator=gen) * 2 - 1
    out = {"lib": os.environ.get("RR_LIB_PATH", "in-tree"), "n": n, "k": K, "replays": a.replays,
           "help_max_n": os.environ.get("RR_HELP_MAX_N")}
    for phase, warm in (("fresh", 5), ("steady", 150)):
        env = RocketBatch(n, model=6, device=dev, max_episode_steps=MAX_EPISODE_STEPS, auto_reset=True,
                          episode_stats=False, **ENV_CONFIG_6DOF)
        env.reset()
        for t in range(warm):
            env.step(pool[t % 8])
        torch.cuda.synchronize(dev)
        ck = {k: v.clone() for k, v in env.checkpoint().items()}
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for t in range(K):
                    env.step(pool[(warm + t) % 8])
        torch.cuda.current_stream(dev).wait_stream(s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        per = []
        for r in range(a.replays + 3):
            env.restore(ck)
            torch.cuda.synchronize(dev)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize(dev)
            if r >= 3:  # the first replays warm the graph
                per.append(e0.elapsed_time(e1) * 1e3 / K)
        done = int(env.done.sum())
        per.sort()
        out[phase] = {"median_us": statistics.median(per), "p10_us": per[len(per) // 10],
                      "p90_us": per[(9 * len(per)) // 10], "done_last_step": done}
        env.close()
    print(json.dumps(out), flush=True)


def run(a):
    libs = [x.strip() for x in a.libs.split(",") if x.strip()]
    rows = {lib: [] for lib in libs}
    for rep in range(a.reps):
        for lib in libs:
            env = dict(os.environ)
            name = lib
            if lib.endswith("@plain"):  # the same library with the plain (no helper waves) kernel
                name = lib[:-len("@plain")]
                env["RR_HELP_MAX_N"] = "0"
            path = name if name.endswith(".so") else os.path.join(ROOT, "tools", "ab", "lib_%s.so" % name)
            if name != "intree":
                env["RR_LIB_PATH"] = path
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "one", "--n", str(a.n), "--replays",
                                str(a.replays)], env=env, capture_output=True, text=True, timeout=240)
            if p.returncode != 0:
                print(p.stderr[-3000:], file=sys.stderr)
                raise SystemExit("step_ab: %s failed (rc %d)" % (lib, p.returncode))
            d = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
            rows[lib].append(d)
            print("rep %d %-16s fresh %.3f us  steady %.3f us" % (rep, lib, d["fresh"]["median_us"],
                                                                 d["steady"]["median_us"]), flush=True)
    base = libs[0]
    summary = {"n": a.n, "reps": a.reps, "replays": a.replays, "what": __doc__.strip().splitlines()[0],
               "libs": {}}
    for lib in libs:
        f = statistics.median([d["fresh"]["median_us"] for d in rows[lib]])
        st = statistics.median([d["steady"]["median_us"] for d in rows[lib]])
        summary["libs"][lib] = {"fresh_us": f, "steady_us": st, "runs": rows[lib]}
    fb = summary["libs"][base]["fresh_us"]
    sb = summary["libs"][base]["steady_us"]
    for lib in libs:
        x = summary["libs"][lib]
        x["fresh_delta_us"] = x["fresh_us"] - fb
        x["steady_delta_us"] = x["steady_us"] - sb
        print("%-16s fresh %.3f (%+.3f)  steady %.3f (%+.3f)" % (lib, x["fresh_us"], x["fresh_delta_us"],
                                                                x["steady_us"], x["steady_delta_us"]), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(summary, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["run", "one"])
    ap.add_argument("--libs", default="base")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--replays", type=int, default=40)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--out")
    a = ap.parse_args()
    (run if a.cmd == "run" else one)(a)


if __name__ == "__main__":
    main()
