"""Interleaved bench.py runs under different HIP runtime environment settings (the variables
must be set before the runtime starts, so every run is its own process).

    python tools/bench_env_ab.py [--rounds 3] [--bench-args "--steps 20 --warmup 5"] "" "HIP_FORCE_DEV_KERNARG=1" ...

Prints per setting the median per-launch device time (roofline.kernel_us) and wall-clock
ms_per_step of the bench line.
"""
import argparse
import json
import os
import shlex
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("settings", nargs="+", help='"" = default, or "VAR=VAL,VAR2=VAL2"')
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--bench-args", default="--steps 20 --warmup 5")
    a = ap.parse_args()
    res = {s: {"kernel_us": [], "wall_us": []} for s in a.settings}
    for _ in range(a.rounds):
        for st in a.settings:
            env = dict(os.environ)
            for kv in [x for x in st.split(",") if x]:
                k, _, v = kv.partition("=")
                env[k] = v
            out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline"]
                                 + shlex.split(a.bench_args), env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:])
                sys.exit(out.returncode)
            line = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
            res[st]["kernel_us"].append(line["roofline"]["kernel_us"])
            res[st]["wall_us"].append(line["ms_per_step"] * 1e3)
    print(json.dumps({"bench_args": a.bench_args, "settings": {
        (s or "default"): {k: {"median": statistics.median(v), "runs": v} for k, v in r.items()}
        for s, r in res.items()}}, indent=1))


if __name__ == "__main__":
    main()
