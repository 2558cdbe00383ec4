"""Per-launch HBM traffic of the step kernel from rocprofv3 PMC passes.

    python tools/pmc_traffic.py gpurun_out/<tag> [--out profiles/rNN/pmc_traffic.json] [--n 65536]

Reads the separate FETCH_SIZE and WRITE_SIZE passes (tools/gpu_check.sh, PMC=1),
takes the median over step_kernel dispatches and applies the gfx950 corrections of
/opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reports half the bytes of
a coalesced streaming read -> x2; WRITE_SIZE (KiB) reads exactly. Calibrated on this
kernel's own pattern: the loaded bytes are known (state 56 + action 12 + v0 4 +
counter 4 = 76 B per 6DOF env), so the x2 factor is checked, not assumed.
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


STEP = re.compile(r"(?<![A-Za-z_])step_kernel<")


def median_counter(d, name, names=None):
    f = glob.glob(os.path.join(d, "pmc_%s" % name, "*counter_collection.csv"))
    if not f:
        return None
    rows = [r for r in csv.DictReader(open(f[0])) if STEP.search(r["Kernel_Name"]) and r["Counter_Name"] == name]
    if names is not None:
        names.update(r["Kernel_Name"] for r in rows)
    vals = [float(r["Counter_Value"]) for r in rows]
    return statistics.median(vals) if vals else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("--out")
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--model", type=int, default=6)
    a = ap.parse_args()
    names = set()
    fetch = median_counter(a.run_dir, "FETCH_SIZE", names)
    write = median_counter(a.run_dir, "WRITE_SIZE", names)
    if len(names) != 1:
        raise SystemExit("expected one step_kernel instantiation in the passes, got %s" % sorted(names))
    from rl_rocket_amd.build import kernel_isa_hashes
    kname = names.pop()
    loaded = {6: 76, 3: 44}[a.model] * a.n
    stored = {6: 122, 3: 66}[a.model] * a.n
    res = {
        "kernel": "step_kernel<%d,RK4>" % a.model, "n": a.n,
        "kernel_name": kname, "isa_hash": kernel_isa_hashes().get(kname),
        "fetch_size_kib": fetch, "write_size_kib": write,
        "read_bytes": 2 * fetch * 1024, "write_bytes": write * 1024,
        "traffic_bytes": 2 * fetch * 1024 + write * 1024,
        "expected_read_bytes": loaded, "expected_write_bytes": stored,
        "read_ratio": 2 * fetch * 1024 / loaded, "write_ratio": write * 1024 / stored,
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), median over step_kernel "
                  "dispatches of bench.py; FETCH_SIZE x2 (gfx950 half-count), KiB = 1024 B",
        "source": a.run_dir,
        "source_hash": __import__("rl_rocket_amd.build", fromlist=["source_hash"]).source_hash(),
    }
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
