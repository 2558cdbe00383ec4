"""Where one step's time goes, per wave: a diagnostic copy of the step kernel with
s_memrealtime stamps (100 MHz) at four points of every main wave, built OUTSIDE the product
source (the product kernel carries no diagnostic code).

    python tools/stamp_probe.py build          # here: writes .ab/stamp.so from a patched copy
    python tools/stamp_probe.py run [--k 20]   # GPU box: K graph launches, stamps of the last

Stamps per main wave: t0 wave start, t1 state / action / counter loads landed, t2 reward +
obs computed, t4 done mask / terminal rows / auto-reset done, t5 state planes and outputs
issued, t6 obs tile issued, t3 every store of the wave acknowledged (s_waitcnt vmcnt(0) after
the last store). Printed relative to the earliest t0 of the launch, with the HIP-event time of the
same launches for the launch floor around them.
"""
import argparse
import ctypes
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, ".ab", "stamp.so")


def patch(src, twice=False):
    def sub(pattern, repl, count=1):
        nonlocal src
        new, k = re.subn(pattern, repl.replace('\\"', '"'), src, count=count)
        if k != count:
            raise SystemExit("stamp_probe: pattern not found: %r" % pattern)
        src = new

    sub(r"(namespace \{\n)", r"\1__device__ unsigned long long g_stamps[8 * 65536];\n")
    if twice:  # diagnostic: the same integration code runs twice (a loop, so the same instruction
        # addresses) after every load has landed; stamp 7 = end of pass 0 (cold i-cache), 4 = end of pass 1
        sub(r"(    const bool event = physics_step<MODEL, INTEG>\(P, a, y0, y1\);\n)",
            r"    asm volatile(\"; all loads\" ::\"v\"(y0[1]), \"v\"(y0[2]), \"v\"(y0[3]), \"v\"(y0[4]), "
            r"\"v\"(y0[5]), \"v\"(y0[7]), \"v\"(y0[8]), \"v\"(y0[9]), \"v\"(y0[10]), \"v\"(y0[11]), "
            r"\"v\"(y0[12]), \"v\"(a[1]));\n"
            r"    const unsigned long long stw = __builtin_amdgcn_s_memrealtime();\n"
            r"    unsigned long long stx = 0;\n    bool event = false;\n"
            r"#pragma unroll 1\n    for (int pass = 0; pass < 2; ++pass) {\n"
            r"        float z = 0.0f;\n        asm volatile(\"\" : \"+v\"(z));\n        float yb[NS];\n"
            r"        for (int j = 0; j < NS; ++j) yb[j] = y0[j] + z;\n"
            r"        event = physics_step<MODEL, INTEG>(P, a, yb, y1);\n"
            r"        asm volatile(\"; pass\" ::\"v\"(y1[0]), \"v\"(y1[13]));\n"
            r"        if (pass == 0) stx = __builtin_amdgcn_s_memrealtime();\n    }\n"
            r"    const unsigned long long sty = __builtin_amdgcn_s_memrealtime();\n")
    sub(r"(    const bool valid = i < n;\n)",
        r"\1    const unsigned long long st0 = __builtin_amdgcn_s_memrealtime();\n")
    sub(r"(    const CounterLayout CL\(P\);\n)",
        r"\1    asm volatile(\"; loads used\" ::\"v\"(y0[0]), \"v\"(y0[6]), \"v\"(y0[13]), \"v\"(a[0]), \"v\"(a[2]), "
        r"\"v\"(v0), \"v\"(cw));\n    const unsigned long long st1 = __builtin_amdgcn_s_memrealtime();\n")
    sub(r"(    float o\[NS\];\n    normalize_obs<NS>\(y1, H.inv_norm, o\);\n)",
        r"\1    asm volatile(\"; computed\" ::\"v\"(o[0]), \"v\"(o[13]), \"v\"(r));\n"
        r"    const unsigned long long st2 = __builtin_amdgcn_s_memrealtime();\n")
    sub(r"(        if \(dv\) store_terminal<NS>\(B, i, vo, plane, o, ret, el\);\n)",
        r"\1        st7 = __builtin_amdgcn_s_memrealtime();\n")
    sub(r"(    const uint64_t m = __ballot\(dv\);\n)", r"\1    unsigned long long st7 = 0;\n")
    sub(r"(    cw = CL.with_elapsed\(cw, el\);\n)",
        r"\1    const unsigned long long st4 = __builtin_amdgcn_s_memrealtime();\n")
    sub(r"(        store_outputs<NT, !ROWS>\(io, i, vo, plane, n, r, done, trunc, t, bv, event\);\n    \}\n)",
        r"\1    const unsigned long long st5 = __builtin_amdgcn_s_memrealtime();\n")
    sub(r"(        store_obs_tile<NS, kWave>\(lds\[wv\], o, make_rsrc\(io.obs, \(uint64_t\)NS \* plane\), wave_base, lane, "
        r"nvalid,\n                                  io.obs_vec_ok\);\n    \}\n)",
        r"\1    const unsigned long long st6 = __builtin_amdgcn_s_memrealtime();\n"
        r"    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n"
        r"    const unsigned long long st3 = __builtin_amdgcn_s_memrealtime();\n"
        r"    if (lane == 0 && wave_idx < 65536u) {\n"
        r"        unsigned long long* g = g_stamps + 8 * wave_idx;\n"
        r"        g[0] = st0; g[1] = st1; g[2] = st2; g[3] = st3; g[4] = st4; g[5] = st5; g[6] = st6; g[7] = st7;\n"
        r"    }\n")
    if twice:
        src = src.replace("g[4] = st4;", "g[4] = sty;").replace("g[7] = st7;", "g[7] = stx;")
        src = src.replace("g[1] = st1;", "g[1] = stw;")
    sub(r"(extern \"C\" \{\n)", r"\1void* rr_diag_stamps() { void* p = nullptr; "
        r"(void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_stamps)); return p; }\n")
    return src


def build(twice=False):
    from rl_rocket_amd import build as b

    src = patch(open(b.SRC).read(), twice)
    tmp = os.path.join(ROOT, ".ab", "stamp_src")
    os.makedirs(tmp, exist_ok=True)
    for f in [os.path.basename(p) for p in b.DEPS]:
        with open(os.path.join(b.HERE, "csrc", f)) as fi, open(os.path.join(tmp, f), "w") as fo:
            fo.write(fi.read())
    path = os.path.join(tmp, "rocket_hip.hip")
    with open(path, "w") as f:
        f.write(src)
    cmd = b.command(out=OUT)
    cmd[-1] = path
    subprocess.check_call(cmd, cwd=ROOT)
    print(OUT)


def run(k, n, twice=False):
    os.environ["RR_LIB_PATH"] = OUT
    import numpy as np
    import torch

    from rl_rocket_amd import _lib
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF

    lib = _lib.load()
    lib.rr_diag_stamps.restype = ctypes.c_void_p
    dev = torch.device("cuda", 0)
    env = RocketBatch(n, model=6, device=dev, max_episode_steps=800, auto_reset=True, episode_stats=False,
                      **ENV_CONFIG_6DOF)
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    pool = torch.rand((8, n, 3), device=dev, generator=g) * 2 - 1
    for j in range(30):
        env.step(pool[j % 8])
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        with torch.cuda.graph(gr, stream=s):
            for j in range(k):
                env.step(pool[j % 8])
    torch.cuda.current_stream(dev).wait_stream(s)
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gr.replay()
    e1.record()
    torch.cuda.synchronize()
    waves = n // 64
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    buf = np.zeros(8 * waves, dtype=np.uint64)
    rc = hip.hipMemcpy(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(lib.rr_diag_stamps()),
                       ctypes.c_size_t(buf.nbytes), ctypes.c_int(2))
    if rc != 0:
        raise SystemExit("hipMemcpy failed: %d" % rc)
    st = buf.reshape(waves, 8).astype(np.int64)
    t = (st[:, :7] - st[:, 0].min()) * 10  # ns
    has_done = st[:, 7] > 0
    q = lambda a: {p: float(np.percentile(a, p)) for p in (0, 50, 90, 99, 100)}  # noqa: E731
    if twice:  # slot 7 = end of the first integration, slot 4 = end of the second
        print(json.dumps({"k": k, "n": n, "twice": True,
                          "ns_first_integration": q((st[:, 7] - st[:, 1]) * 10),
                          "ns_second_integration": q((st[:, 4] - st[:, 7]) * 10)}, indent=1))
        return
    print(json.dumps({
        "k": k, "n": n, "event_us_per_launch": e0.elapsed_time(e1) * 1e3 / k,
        "ns_start": q(t[:, 0]), "ns_loads_landed": q(t[:, 1] - t[:, 0]), "ns_compute": q(t[:, 2] - t[:, 1]),
        "ns_tail_to_ack": q(t[:, 3] - t[:, 2]), "ns_wave_total": q(t[:, 3] - t[:, 0]),
        "ns_done_reset": q(t[:, 4] - t[:, 2]), "ns_state_output_issue": q(t[:, 5] - t[:, 4]),
        "ns_obs_tile_issue": q(t[:, 6] - t[:, 5]), "ns_ack_wait": q(t[:, 3] - t[:, 6]),
        "waves_with_done": int(has_done.sum()),
        "ns_terminal_rows_done_waves": q((st[has_done, 7] - st[has_done, 2]) * 10) if has_done.any() else None,
        "ns_reset_after_terminal_done_waves": q((st[has_done, 4] - st[has_done, 7]) * 10) if has_done.any() else None,
        "ns_last_ack_after_first_start": float(t[:, 3].max()),
        "slowest_wave": {"index": int(np.argmax(t[:, 3])), "stamps_ns": t[int(np.argmax(t[:, 3]))].tolist()},
    }, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["build", "run"])
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--twice", action="store_true", help="diagnostic: integrate twice (cold vs warm i-cache)")
    a = ap.parse_args()
    build(a.twice) if a.what == "build" else run(a.k, a.n, a.twice)


if __name__ == "__main__":
    main()
