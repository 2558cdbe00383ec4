"""Roofline fraction of the step kernel from committed rocprofv3 `--stats` summaries, next to
the HIP-event fraction of the bench lines of the same session.

    python tools/rocprof_frac.py profiles/r02/r02x [--out profiles/r02/r02x/rocprof_frac.json]

For every `*_kernel_stats.csv` in the directory: the step kernel's mean duration and the
fraction 189 B x N / mean / 8 TB/s (N and bytes per env-step from the bench lines there).
"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    lines = []
    for path in sorted(glob.glob(os.path.join(a.dir, "bench_k*.json"))):
        with open(path) as f:
            rows = [json.loads(x) for x in f if x.startswith("{")]
        if rows:
            lines.append((os.path.basename(path), rows[-1]))
    if not lines:
        raise SystemExit("no bench_k*.json lines in %s" % a.dir)
    ref = lines[0][1]
    bytes_launch = ref["roofline"]["bytes_per_launch"]
    peak = ref["roofline"]["peak"]
    out = {"bytes_per_launch": bytes_launch, "peak_gbs": peak, "rocprof": {}, "hip_events": {}}
    for name, d in lines:
        out["hip_events"][name] = {"kernel_us": d["roofline"]["kernel_us"], "frac": d["roofline"]["frac"],
                                   "steps": d["steps"]}
    for path in sorted(glob.glob(os.path.join(a.dir, "*kernel_stats.csv"))):
        with open(path) as f:
            for row in csv.DictReader(f):
                if "step_kernel<6" not in row["Name"]:
                    continue
                mean_ns = float(row["AverageNs"])
                out["rocprof"][os.path.basename(path)] = {
                    "calls": int(row["Calls"]), "mean_us": mean_ns / 1e3, "min_us": float(row["MinNs"]) / 1e3,
                    "frac": bytes_launch / (mean_ns * 1e-9) / 1e9 / peak}
    k20 = [v["frac"] for k, v in out["hip_events"].items() if v["steps"] == 20]
    if k20:
        out["k20_event_frac_median"] = statistics.median(k20)
        for v in out["rocprof"].values():
            v["ratio_to_k20_event_frac"] = v["frac"] / out["k20_event_frac_median"]
    text = json.dumps(out, indent=1)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
