"""The per-wave latency floor of the N = 65 536 step kernel.

    python tools/floor_probe.py run --graph [--n 65536] [--out FILE]  # events, back to back (hipGraph)
    rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o fp -- python tools/floor_probe.py run --reps 25
    python tools/floor_probe.py model RUN.json DIR/fp_kernel_stats.csv [--out FILE]

`run` launches, in one process, the probe kernels of tools/floor_probe.hip (the step kernel's
launch shape and memory pattern: empty, memory only, memory + 128 / 256 / 384 / 512 VALU of
dependent fma chains) and the real step kernel (rr_step through RocketBatch at N envs, auto-reset,
TimeLimit 800 — the bench's headline configuration), each `reps` times back to back after a
warm-up, and prints the per-launch time by HIP events around each back-to-back group (--graph:
replayed from a hipGraph, so the host does not pace them). Under
rocprofv3 the same command gives every kernel's kernel-trace duration. `model` fits
t(VALU) = t_mem + c * VALU over the probe chain (c = cycles per lone-wave VALU instruction at the
clock the chip held) and places the step kernel on it with the VALU count of its slowest wave
(the main role's compute block + the ground-event block, trans ops counted twice: a lone wave
issues a transcendental every 8 cycles, a plain VALU op every 4).
"""
import argparse
import csv
import ctypes
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "tools", "libfloor_probe.so")
KINDS = {0: "empty", 1: "mem", 2: "mem+128", 3: "mem+256", 4: "mem+384", 5: "mem+512"}
VALU_EXTRA = {1: 0, 2: 128, 3: 256, 4: 384, 5: 512}


def run(a):
    import numpy as np
    import torch

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF, MAX_EPISODE_STEPS

    lib = ctypes.CDLL(LIB)
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
    ptr = lambda t: P(t.data_ptr())  # noqa: E731
    out = {"n": n, "reps": a.reps, "launch": "hipGraph of reps launches" if a.graph else "direct launches",
           "events_us_per_launch": {}}

    def timed(fn):
        """Per-launch time of `reps` back-to-back launches by HIP events: replayed from one hipGraph
        (--graph: the host cannot pace them; the replay's fixed preamble is spread over the reps), or
        issued directly (host-paced for launches shorter than the ~3 us of host time each costs)."""
        stream = torch.cuda.current_stream(dev)
        fn(5)  # warm-up
        torch.cuda.synchronize(dev)
        if a.graph:
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(dev)
            s.wait_stream(stream)
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    fn(a.reps)
            stream.wait_stream(s)
            g.replay()
            torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        if a.graph:
            g.replay()
        else:
            fn(a.reps)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / a.reps * 1e3

    for kind, name in KINDS.items():
        def probe(k, kind=kind):
            rc = lib.fp_repeat(kind, k, ptr(state), ptr(action), n, ptr(obs), ptr(reward), ptr(done), ptr(trunc),
                               P(torch.cuda.current_stream(dev).cuda_stream))
            if rc:
                raise RuntimeError("fp_repeat(%d): %d" % (kind, rc))
        out["events_us_per_launch"][name] = timed(probe)
    env = RocketBatch(n, model=6, device=dev, max_episode_steps=MAX_EPISODE_STEPS, auto_reset=True,
                      episode_stats=False, **ENV_CONFIG_6DOF)
    env.reset()
    pool = torch.rand((8, n, 3), device=dev, generator=g) * 2 - 1
    for k in range(200):  # steady state: ~1 % of the envs end an episode per step
        env.step(pool[k % 8])

    def step(k):
        for t in range(k):
            env.step(pool[t % 8])
    out["events_us_per_launch"]["step"] = timed(step)
    env.close()
    print(json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


def _step_valu(lib_path=None):
    """(VALU, trans) of the step kernel's slowest main-wave path: the blocks of the main role's
    compute (the largest block) and the ground-event path, from the device assembly of the
    kernel this tree builds (tools/isa_count.py's classes)."""
    import subprocess
    import tempfile

    from rl_rocket_amd import build as B

    with tempfile.TemporaryDirectory() as d:
        s = os.path.join(d, "step.s")
        cmd = B.command(out=s, compile_only=True)
        cmd = [c for c in cmd if c not in ("-c", "-fPIC")] + ["--cuda-device-only", "-S"]
        subprocess.check_call(cmd, cwd=ROOT, stderr=subprocess.DEVNULL)
        text = open(s).read()
    m = re.search(r"^_Z\S*step_kernelILi6ELi0ELb0ELb1ELi4ELb0E\S*:", text, re.M)
    body = text[m.end():]
    body = body[:body.index(".Lfunc_end")]
    blocks, cur = [], {"valu": 0, "trans": 0}
    trans = re.compile(r"^v_(exp|log|rcp|rsq|sqrt|sin|cos)_")
    for line in body.splitlines():
        t = line.strip()
        if re.match(r"^\.LBB\d+_\d+:", t):
            blocks.append(cur)
            cur = {"valu": 0, "trans": 0}
            continue
        op = t.split()[0] if t and not t.startswith((";", ".")) else ""
        if trans.match(op):
            cur["trans"] += 1
        elif op.startswith("v_") and not op.startswith(("v_readfirstlane", "v_writelane", "v_readlane")):
            cur["valu"] += 1
    blocks.append(cur)
    return blocks


def model(a):
    with open(a.run) as f:
        run_ = json.load(f)
    rp = {}
    with open(a.stats) as f:
        for r in csv.DictReader(f):
            nm = r["Name"].replace(" ", "")
            m = re.search(r"probe_kernel<(\d+),(\d+)>", nm)
            if m:
                kind = 0 if m.group(1) == "0" else {0: 1, 32: 2, 64: 3, 96: 4, 128: 5}[int(m.group(2))]
                rp[KINDS[kind]] = float(r["AverageNs"]) / 1e3
            elif re.search(r"(?<![A-Za-z_])step_kernel<6,0,false,true,4,false>", nm):
                rp["step"] = float(r["AverageNs"]) / 1e3
    blocks = _step_valu()
    big = sorted(blocks, key=lambda b: b["valu"], reverse=True)
    # the main role's compute block and the ground-event block are the two largest main-role
    # blocks; the helper role's candidate draw (~200 VALU) runs on its own wave
    main, event = big[0], big[2] if big[1]["valu"] > 150 and big[2]["valu"] > 60 else big[1]
    res = {"events_us": run_["events_us_per_launch"], "rocprof_us": rp}
    for frame, t in (("events", run_["events_us_per_launch"]), ("rocprof", rp)):
        if not all(KINDS[k] in t for k in VALU_EXTRA):
            continue
        xs = [VALU_EXTRA[k] for k in VALU_EXTRA]
        ys = [t[KINDS[k]] for k in VALU_EXTRA]
        mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
        c = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
        t0 = my - c * mx
        res[frame] = {"us_per_valu": c, "t_mem_fit_us": t0, "t_empty_us": t[KINDS[0]],
                      "fit_residual_max_us": max(abs(t0 + c * x - y) for x, y in zip(xs, ys))}
        if "step" in t:
            for label, v in (("no_event", main["valu"] + 2 * main["trans"]),
                             ("with_event", main["valu"] + 2 * main["trans"] + event["valu"] + 2 * event["trans"])):
                fl = t0 + c * v
                res[frame]["floor_" + label] = {"valu_issue_slots": v, "floor_us": fl, "step_us": t["step"],
                                                "step_over_floor": t["step"] / fl}
    res["step_blocks"] = {"main_compute": main, "ground_event": event}
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--n", type=int, default=65536)
    r.add_argument("--reps", type=int, default=200)
    r.add_argument("--graph", action="store_true", help="time hipGraph replays (the unprofiled back-to-back frame)")
    r.add_argument("--out")
    m = sub.add_parser("model")
    m.add_argument("run")
    m.add_argument("stats")
    m.add_argument("--out")
    a = ap.parse_args()
    run(a) if a.cmd == "run" else model(a)


if __name__ == "__main__":
    main()
