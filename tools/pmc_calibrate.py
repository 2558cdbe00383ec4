"""Calibrate rocprofv3's FETCH_SIZE / WRITE_SIZE on the step kernel's OWN access pattern (VERDICT r5
weak 3: the guide's x2 FETCH_SIZE correction was measured for 16-B-per-lane reads; the step kernel
reads 4 B per lane per plane). The probe is tools/floor_probe.hip's `mem` kernel — the step's launch
shape and exact memory pattern with no compute: per env it loads the counter word, the 12-B action
row, 14 state planes and v0 through buffer descriptors (76 B; the helper waves re-load the counter
word, a line the main wave fetches too) and stores the 14 planes + counter (sc1), reward, done,
truncated and the obs row through the LDS tile as 16-B stores (122 B) — so its bytes are known.

    python tools/pmc_calibrate.py run [--n 65536] [--k 64]        # the probe launches (under rocprofv3 --pmc)
    python tools/pmc_calibrate.py parse DIR [--n 65536] [--step STEP_PMC_JSON] [--out F]

`parse` reads DIR/pmc_FETCH_SIZE and DIR/pmc_WRITE_SIZE (separate passes, as tools/pmc_traffic.py),
takes the median over the probe's dispatches and reports counter bytes / known bytes for reads and
writes; with --step (a tools/pmc_traffic.py JSON of the step kernel, same box or not) it applies those
factors to the step kernel's counters: its traffic calibrated on its own pattern.
"""
import argparse
import csv
import ctypes
import glob
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READ_B, WRITE_B = 76, 122  # per env: floor_probe.hip kind 1 (= step_kernel<6, RK4, HELP>'s pattern)


def run(a):
    import torch

    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libfloor_probe.so"))
    P = ctypes.c_void_p
    lib.fp_repeat.argtypes = [ctypes.c_int, ctypes.c_int64, P, P, ctypes.c_int64, P, P, P, P, P]
    n, dev = a.n, torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    state = torch.rand((17 * n,), device=dev, generator=g)
    action = torch.rand((n, 3), device=dev, generator=g) * 2 - 1
    obs = torch.empty((n, 14), device=dev)
    reward = torch.empty((n,), device=dev)
    done = torch.empty((n,), device=dev, dtype=torch.uint8)
    trunc = torch.empty((n,), device=dev, dtype=torch.uint8)
    p = lambda t: P(t.data_ptr())  # noqa: E731
    s = P(torch.cuda.current_stream(dev).cuda_stream)
    rc = lib.fp_repeat(1, a.k, p(state), p(action), n, p(obs), p(reward), p(done), p(trunc), s)
    torch.cuda.synchronize(dev)
    if rc != 0:
        raise SystemExit("fp_repeat failed: %d" % rc)
    print(json.dumps({"n": n, "launches": a.k, "kind": "mem"}))


def median_counter(d, name, kernel):
    f = glob.glob(os.path.join(d, "pmc_%s" % name, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return None, 0
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f[0]))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == name]
    return (statistics.median(vals), len(vals)) if vals else (None, 0)


def parse(a):
    kernel = "probe_kernel<1, 0>"
    fetch, nf = median_counter(a.run_dir, "FETCH_SIZE", kernel)
    write, nw = median_counter(a.run_dir, "WRITE_SIZE", kernel)
    if fetch is None or write is None:
        raise SystemExit("no %s rows under %s" % (kernel, a.run_dir))
    rb, wb = READ_B * a.n, WRITE_B * a.n
    out = {"what": "FETCH_SIZE / WRITE_SIZE (KiB, rocprofv3 --pmc, separate passes) of a kernel with the step "
                   "kernel's launch shape and memory pattern and known bytes (tools/floor_probe.hip kind 1)",
           "n": a.n, "dispatches": [nf, nw], "fetch_size_kib": fetch, "write_size_kib": write,
           "known_read_bytes": rb, "known_write_bytes": wb,
           "fetch_bytes_over_known_read": fetch * 1024 / rb, "write_bytes_over_known_write": write * 1024 / wb,
           "read_correction": rb / (fetch * 1024), "write_correction": wb / (write * 1024), "source": a.run_dir}
    if a.step:
        with open(a.step) as f:
            st = json.load(f)
        rd = st["fetch_size_kib"] * 1024 * out["read_correction"]
        wr = st["write_size_kib"] * 1024 * out["write_correction"]
        out["step"] = {"source": a.step, "isa_hash": st.get("isa_hash"), "read_bytes_calibrated": rd,
                       "write_bytes_calibrated": wr, "traffic_bytes_calibrated": rd + wr,
                       "read_ratio_calibrated": rd / st["expected_read_bytes"],
                       "write_ratio_calibrated": wr / st["expected_write_bytes"],
                       "traffic_bytes_guide_x2": st["traffic_bytes"]}
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--n", type=int, default=65536)
    r.add_argument("--k", type=int, default=64)
    q = sub.add_parser("parse")
    q.add_argument("run_dir")
    q.add_argument("--n", type=int, default=65536)
    q.add_argument("--step")
    q.add_argument("--out")
    a = ap.parse_args()
    run(a) if a.cmd == "run" else parse(a)


if __name__ == "__main__":
    main()
