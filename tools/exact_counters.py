"""Counter summary of the exact-mode kernel (step_exact_kernel / step_exact_pair_kernel) from the
rocprofv3 passes of tools/gpu_r03.sh (exact_kt: kernel trace; exact_SQ, exact_SQ2: --pmc).

    python tools/exact_counters.py gpurun_out/<tag> [--out profiles/r03/<tag>/exact_counters.json]

Per dispatch medians, per-wave figures and the shares of wave cycles (SQ_WAVE_CYCLES and the
SQ_WAIT / SQ_ACTIVE counters count quad-cycles: x4 for cycles, MI355X_MICROARCH.md).
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys


def counters(d, grid=None):
    """Per-dispatch medians of the exact kernel's counters (only dispatches of `grid` threads when
    given: bench.py's N sweep runs the same kernel at other N in the same process)."""
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "step_exact" not in r["Kernel_Name"] or (grid and int(r["Grid_Size"]) != grid):
                continue
            out.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    res = {}
    n = None
    bench = os.path.join(a.run_dir, "bench_exact.json")
    if os.path.exists(bench):
        line = [json.loads(x) for x in open(bench) if x.startswith("{")][-1]
        n = line["config"]["envs_per_gpu"]
        res["bench"] = {"value": line["value"], "ms_per_step": line["ms_per_step"],
                        "kernel_us_events": line["roofline"]["kernel_us"], "n": n}
    # dispatches at the bench's N only (one thread per env)
    c = {}
    for sub in ("exact_SQ", "exact_SQ2"):
        c.update(counters(os.path.join(a.run_dir, sub), n))
    res["median_per_dispatch"] = c
    for f in glob.glob(os.path.join(a.run_dir, "exact_kt", "**", "*kernel_trace.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if "step_exact" in r["Kernel_Name"] and
                (n is None or int(r["Grid_Size_X"]) == n)]
        if rows:
            us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
            res["kernel_trace"] = {"name": rows[0]["Kernel_Name"], "calls": len(us), "grid": n,
                                   "mean_us": statistics.mean(us), "median_us": statistics.median(us),
                                   "min_us": min(us), "max_us": max(us)}
    w = c.get("SQ_WAVES")
    if w:
        d = {}
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                  "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_BRANCH", "SQ_INSTS_SMEM"):
            if k in c:
                d[k + "_per_wave"] = c[k] / w
        for k in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in c:
                d[k + "_cycles_per_wave"] = 4 * c[k] / w
        wc = c.get("SQ_WAVE_CYCLES")
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in c and wc:
                d[k + "_share_of_wave_cycles"] = c[k] / wc
        if "SQ_INSTS_VALU" in c and "SQ_ACTIVE_INST_VALU" in c:
            d["valu_cycles_per_valu_inst"] = 4 * c["SQ_ACTIVE_INST_VALU"] / c["SQ_INSTS_VALU"]
        res["derived"] = d
    # fp64 VALU FLOPs issued per dispatch (64 lanes per wave-instruction, masked lanes included: an
    # upper bound of the useful work) over the kernel-trace mean at the same N, against the fp64
    # vector peak (MI355X_MICROARCH.md: 78.6 TF)
    if all(k in c for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64")) and \
            "kernel_trace" in res:
        fl = 64 * (c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + 2 * c["SQ_INSTS_VALU_FMA_F64"])
        t = res["kernel_trace"]["mean_us"] * 1e-6
        res["fp64"] = {"flops_per_dispatch": fl, "achieved_tflops": fl / t / 1e12, "peak_tflops": 78.6,
                       "frac": fl / t / 1e12 / 78.6,
                       "what": "64 x (ADD_F64 + MUL_F64 + 2 FMA_F64) wave-instructions per dispatch over the "
                               "kernel-trace mean (masked lanes counted: issue rate, not useful work)"}
    if "kernel_trace" in res:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from rl_rocket_amd.build import kernel_isa_hashes

        res["kernel_name"] = res["kernel_trace"]["name"]
        res["isa_hash"] = kernel_isa_hashes().get(res["kernel_name"])
    res["source"] = a.run_dir
    text = json.dumps(res, indent=1)
    print(text)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
