"""Interleaved timing of the step kernel under different HIP runtime environment settings
(diagnostics): each round runs tools/diag_kernel.py --child once per setting in a fresh
process (the variables must be set before the HIP runtime starts).

    python tools/env_ab.py --lib rl_rocket_amd/librocket_hip.so "" "HIP_FORCE_DEV_KERNARG=1" ...
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("settings", nargs="+", help='"" = default, or "VAR=VAL,VAR2=VAL2"')
    ap.add_argument("--lib", default=os.path.join(ROOT, "rl_rocket_amd", "librocket_hip.so"))
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=2048)
    a = ap.parse_args()
    res = {s: [] for s in a.settings}
    for _ in range(a.rounds):
        for st in a.settings:
            env = dict(os.environ, RR_LIB_PATH=os.path.abspath(a.lib))
            for kv in [x for x in st.split(",") if x]:
                k, _, v = kv.partition("=")
                env[k] = v
            out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "diag_kernel.py"), "--child",
                                  "--n", str(a.n), "--model", "6", "--steps", str(a.steps)], env=env,
                                 capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:])
                sys.exit(out.returncode)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
            res[st].append(json.loads(line)["us_per_step"])
    print(json.dumps({"lib": os.path.relpath(a.lib, ROOT), "n": a.n,
                      "settings": {(s or "default"): {"median_us": statistics.median(v), "runs": v}
                                   for s, v in res.items()}}, indent=1))


if __name__ == "__main__":
    main()
