"""Interleaved A/B timing of kernel source variants on the rollout leg (bench.py --mode rollout).

    python tools/rollout_ab.py A.hip B.hip@NAME=VAL C.so [...] [--prec fp32,fp16x3] [--rounds 3]

Each variant is compiled with the product flags (rl_rocket_amd/build.py) into its own .so;
rounds alternate the variants, each in a fresh bench.py child (RR_LIB_PATH), and report the
median GPU ms per 16-step collect per precision.
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
    ap.add_argument("--prec", default="fp32,fp16x3,bf16")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--extra", default="", help="extra bench.py arguments")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "ab"))
    a = ap.parse_args()
    from rl_rocket_amd import build as b

    os.makedirs(a.out, exist_ok=True)
    libs = []
    for k, spec in enumerate(a.sources):
        src, _, defs = spec.partition("@")
        if src.endswith(".so"):  # prebuilt variant (compiled on the CPU side)
            libs.append(os.path.abspath(src))
            continue
        lib = os.path.join(a.out, "rab_%d.so" % k)
        items = [d for d in defs.split(",") if d]
        cmd = b.command(out=lib, defines=tuple(d for d in items if not d.startswith("+")),
                        extra=tuple(d[1:] for d in items if d.startswith("+")))
        cmd[-1] = os.path.abspath(src)
        subprocess.check_call(cmd)
        libs.append(lib)
    precs = a.prec.split(",")
    res = {(s, p): [] for s in a.sources for p in precs}
    for r in range(a.rounds):
        for p in precs:
            for src, lib in zip(a.sources, libs):
                env = dict(os.environ, RR_LIB_PATH=lib)
                out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--mode", "rollout",
                                      "--no-cpu-baseline", "--policy-dtype", p] + a.extra.split(),
                                     env=env, capture_output=True, text=True, timeout=300)
                if out.returncode != 0:
                    print(out.stderr[-2000:])
                    sys.exit(out.returncode)
                line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
                res[(src, p)].append(json.loads(line)["gpu_ms_per_collect"])
            print("round", r, p, {s: res[(s, p)][-1] for s in a.sources}, flush=True)
    summary = {"%s [%s]" % (s, p): {"median_ms_per_collect": statistics.median(v), "runs": v}
               for (s, p), v in res.items()}
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
