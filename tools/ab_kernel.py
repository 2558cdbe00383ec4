"""Interleaved A/B timing of kernel source variants on ONE GPU.

    python tools/ab_kernel.py A.hip B.hip [...] [--n 65536] [--rounds 5] [--model 6]
    (a source may carry "@NAME=VAL,+-compiler-flag,..." defines / extra flags)

Each variant is compiled with the product flags (rl_rocket_amd/build.py) into its own
.so; rounds alternate A, B, A, B ... each in a fresh child process (tools/diag_kernel.py
--child: HIP events around hipGraph replays of 64 launches). Reports per-variant median
us/step, so box-to-box and run-to-run drift cancels out of the comparison.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sources", nargs="+")
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--model", type=int, default=6)
    ap.add_argument("--steps", type=int, default=4096)
    ap.add_argument("--integrator", default="rk4")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "ab"))
    a = ap.parse_args()
    from rl_rocket_amd import build as b

    os.makedirs(a.out, exist_ok=True)
    libs = []
    for k, spec in enumerate(a.sources):
        src, _, defs = spec.partition("@")  # "file.hip@NAME=VAL,NAME2=VAL2"
        if src.endswith(".so"):  # prebuilt variant (compiled on the CPU side)
            libs.append(os.path.abspath(src))
            continue
        lib = os.path.join(a.out, "ab_%d.so" % k)
        items = [d for d in defs.split(",") if d]  # "+flag" items are extra compiler flags
        cmd = b.command(out=lib, defines=tuple(d for d in items if not d.startswith("+")),
                        extra=tuple(d[1:] for d in items if d.startswith("+")))
        cmd[-1] = os.path.abspath(src)
        subprocess.check_call(cmd)
        libs.append(lib)
    res = {s: [] for s in a.sources}
    for r in range(a.rounds):
        for src, lib in zip(a.sources, libs):
            env = dict(os.environ, RR_LIB_PATH=lib)
            out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "diag_kernel.py"), "--child",
                                  "--tag", os.path.basename(src), "--n", str(a.n), "--model", str(a.model),
                                  "--steps", str(a.steps), "--integrator", a.integrator], env=env, capture_output=True,
                                 text=True, timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:])
                sys.exit(out.returncode)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
            res[src].append(json.loads(line)["us_per_step"])
    summary = {os.path.relpath(s.partition("@")[0], ROOT) + s.partition("@")[1] + s.partition("@")[2]:
               {"median_us": statistics.median(v), "min_us": min(v), "runs": v} for s, v in res.items()}
    print(json.dumps({"n": a.n, "model": a.model, "variants": summary}, indent=1))


if __name__ == "__main__":
    main()
