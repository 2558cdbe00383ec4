"""Per-dispatch SQ / GRBM counter summary of one kernel from rocprofv3 --pmc passes.

    python tools/sq_summary.py gpurun_out/<tag> [--kernel step_kernel] [--out profiles/rNN/sq.json]

Reads every pmc_*/*counter_collection.csv under the run directory, keeps the dispatches
whose name contains --kernel, and reports the median per dispatch of each counter plus
derived per-wave figures. Units (MI355X_MICROARCH.md, 'SQ PMC units'): SQ_WAVE_CYCLES,
SQ_BUSY_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_* count quad-cycles (x4 = shader cycles);
SQ_INSTS_* count wave-instructions; WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES.
GRBM_GUI_ACTIVE is summed over the 8 XCDs (/8 = GPU-busy cycles of the dispatch).
"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("--kernel", default="step_kernel")
    ap.add_argument("--out")
    a = ap.parse_args()
    per = {}
    for f in glob.glob(os.path.join(a.run_dir, "pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if a.kernel not in r["Kernel_Name"]:
                continue
            key = (os.path.basename(os.path.dirname(f)), r["Dispatch_Id"])
            per.setdefault(r["Counter_Name"], {}).setdefault(key, 0.0)
            per[r["Counter_Name"]][key] += float(r["Counter_Value"])
            kname = r["Kernel_Name"]
    med = {c: statistics.median(v.values()) for c, v in per.items()}
    n_disp = {c: len(v) for c, v in per.items()}
    res = {"kernel": kname if per else None, "dispatches": n_disp, "median_per_dispatch": med}
    waves = med.get("SQ_WAVES")
    if waves:
        d = {}
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_LDS", "SQ_INSTS_SMEM",
                  "SQ_INSTS_BRANCH", "SQ_INSTS_VALU_TRANS_F32"):
            if c in med:
                d[c + "_per_wave"] = med[c] / waves
        for c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_SCA", "SQ_INST_CYCLES_VMEM"):
            if c in med:
                d[c + "_cycles_per_wave"] = 4 * med[c] / waves
        if "SQ_WAVE_CYCLES" in med:
            wc = med["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in med:
                    d[c + "_share_of_wave_cycles"] = med[c] / wc
        if "GRBM_GUI_ACTIVE" in med:
            d["gpu_busy_cycles"] = med["GRBM_GUI_ACTIVE"] / 8
        res["derived"] = d
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(dict(res, source=a.run_dir), open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
