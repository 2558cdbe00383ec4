"""The step kernel's rocprofv3 kernel-trace duration of one bench.py command, stamped with the
kernel source hash, so that bench.py can quote it beside its own HIP-event time
(roofline.frac_rocprof) only while the kernel source is the same.

    rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o bench -- python bench.py ARGS > DIR/bench.json
    python tools/rocprof_step.py DIR --out profiles/r03/<tag>/rocprof_step_k<K>_n<N>.json
    (a bench.py --mode rollout line: --out .../rocprof_rollout_n<N>_t<T>_<dtype>.json, the collect kernel)

Reads DIR/**/*kernel_stats.csv (the step_kernel row: calls, mean / min / max ns) and the bench
line the same command printed (its HIP-event time under the profiler, N, K, bytes per launch).
"""
import argparse
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("--bench", help="bench JSON line file (default: RUN_DIR/bench.json)")
    ap.add_argument("--out")
    a = ap.parse_args()
    from rl_rocket_amd.build import kernel_isa_hashes, source_hash

    bench = a.bench or os.path.join(a.run_dir, "bench.json")
    with open(bench) as f:
        line = [json.loads(x) for x in f if x.startswith("{")][-1]
    stats = glob.glob(os.path.join(a.run_dir, "**", "*kernel_stats.csv"), recursive=True)
    if not stats:
        raise SystemExit("no *kernel_stats.csv under %s" % a.run_dir)
    model = 6 if "6DOF" in line["metric"] else 3
    rollout = "gpu_ms_per_collect" in line
    pat = (r"(?<![A-Za-z_])rollout_step_kernel<%d,\d+,\d+,true," if rollout else r"(?<![A-Za-z_])step_kernel<%d,") % model
    row = None
    for path in stats:
        with open(path) as f:
            for r in csv.DictReader(f):
                if re.search(pat, r["Name"].replace(" ", "")):
                    if row is None or int(r["Calls"]) > int(row["Calls"]):
                        row = r
    if row is None:
        raise SystemExit("no %s row in %s" % (pat, stats))
    rf = line["roofline"]
    mean = float(row["AverageNs"])
    if rollout:  # the collect kernel (bench.py --mode rollout): FLOPs against the MFMA peak
        res = {
            "kernel": "rollout_step_kernel<%d,MULTI>" % model, "kernel_name": row["Name"],
            "isa_hash": kernel_isa_hashes().get(row["Name"]), "n": line["config"]["envs_per_gpu"],
            "calls": int(row["Calls"]), "mean_ns": mean, "min_ns": float(row["MinNs"]), "max_ns": float(row["MaxNs"]),
            "flops_per_launch": rf["flops_per_launch"], "peak_tflops": rf["peak"],
            "achieved_tflops": rf["flops_per_launch"] / (mean * 1e-9) / 1e12,
            "frac": rf["flops_per_launch"] / (mean * 1e-9) / 1e12 / rf["peak"],
            "events_ms_per_collect_under_profiler": line["gpu_ms_per_collect"],
            "method": "rocprofv3 --kernel-trace --stats of bench.py --mode rollout (all dispatches of the collect "
                      "kernel in the process)", "source": a.run_dir, "source_hash": source_hash()}
        text = json.dumps(res, indent=1)
        print(text)
        if a.out:
            os.makedirs(os.path.dirname(a.out), exist_ok=True)
            with open(a.out, "w") as f:
                f.write(text + "\n")
        return
    res = {
        "kernel": "step_kernel<%d,%s>" % (model, line["config"]["integrator"].upper()),
        "kernel_name": row["Name"],
        "isa_hash": kernel_isa_hashes().get(row["Name"]),
        "n": line["config"]["envs_per_gpu"], "steps": line["steps"], "warmup": line["warmup"],
        "launch": line["config"]["launch"],
        "calls": int(row["Calls"]), "mean_ns": mean, "min_ns": float(row["MinNs"]), "max_ns": float(row["MaxNs"]),
        "stddev_ns": float(row.get("StdDev", 0) or 0),
        "bytes_per_launch": rf["bytes_per_launch"],
        "frac": rf["bytes_per_launch"] / (mean * 1e-9) / 1e9 / rf["peak"],
        "events_kernel_us": rf["kernel_us"],
        "events_frac_under_profiler": rf["frac"],
        "method": "rocprofv3 --kernel-trace --stats of the bench command (all dispatches of the kernel in the "
                  "process, warm-up included); events_* = the bench's own HIP-event time in the same run",
        "source": a.run_dir,
        "source_hash": source_hash(),
    }
    text = json.dumps(res, indent=1)
    print(text)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
