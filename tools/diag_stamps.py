"""Per-wave phase timeline of the step kernel (RR_DIAG=4 build, s_memtime stamps).

    python tools/diag_stamps.py [--n 65536] [--steps 40]

Phases (cycles, shader clock): 0->1 load burst landed, 1->2 RK4, 2->3 event path,
3->4 reward/done, 4->5 done mask + reset, 5->6 stores issued, 6->7 stores drained.
Diagnostic only: the stamps' waits serialise the wave, so read shares, not totals.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "diag"))
    ap.add_argument("--graph", action="store_true", help="replay the steps back to back from a hipGraph")
    ap.add_argument("--raw", help="save every sampled wave record (npz) for offline analysis")
    ap.add_argument("--defines", default="", help="extra -D defines for the stamp build, comma separated")
    ap.add_argument("--diag", type=int, default=4, choices=[4, 12],
                    help="4: phase stamps (the waits serialise the wave); 12: start / end only (product code "
                         "inside the wave; stamp slots 0 / 1 = event / done lanes of the wave)")
    a = ap.parse_args()
    from rl_rocket_amd import build as b

    os.makedirs(a.out, exist_ok=True)
    lib_path = os.path.join(a.out, "librocket_hip_diag%d.so" % a.diag)
    subprocess.check_call(b.command(out=lib_path, defines=("RR_DIAG=%d" % a.diag,) + tuple(d for d in a.defines.split(",") if d)))
    os.environ["RR_LIB_PATH"] = lib_path
    import torch

    from rl_rocket_amd import _lib
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF

    _lib.LIB_PATH = lib_path
    lib = _lib.load()
    lib.rr_debug_stamps.restype = ctypes.c_int64
    lib.rr_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    env = RocketBatch(a.n, model=6, device="cuda:0", max_episode_steps=800, episode_stats=False, **ENV_CONFIG_6DOF)
    env.reset()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(3)
    nw = (a.n + 63) // 64
    buf = np.zeros(nw * 12, np.uint64)
    rows = []
    pool = [torch.rand((a.n, 3), device="cuda:0", generator=g) * 2 - 1 for _ in range(8)]
    if a.graph:
        for k in range(30):
            env.step(pool[k % 8])
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(graph, stream=s):
                for k in range(16):
                    env.step(pool[k % 8])
        torch.cuda.current_stream().wait_stream(s)
        for k in range(a.steps):
            graph.replay()
            if k >= a.steps - 10:  # stamps of the last step of the replay (after 15 back-to-back launches)
                lib.rr_debug_stamps(env._h, buf.ctypes.data_as(ctypes.c_void_p), buf.size)
                rows.append(buf.reshape(nw, 12).astype(np.int64).copy())
    else:
        for k in range(a.steps):
            env.step(pool[k % 8])
            if k >= a.steps - 10:
                lib.rr_debug_stamps(env._h, buf.ctypes.data_as(ctypes.c_void_p), buf.size)
                rows.append(buf.reshape(nw, 12).astype(np.int64).copy())
    allst = np.concatenate(rows)
    st = allst[:, :8]
    names = ["load", "rk4", "event", "reward", "done+reset", "store_issue", "store_drain"]
    d = np.diff(st, axis=1)
    out = {"n": a.n, "waves": int(nw), "samples": int(st.shape[0])}
    for j, nm in enumerate(names):
        out[nm] = {"median": float(np.median(d[:, j])), "p90": float(np.percentile(d[:, j], 90)),
                   "max": float(d[:, j].max())}
    per = allst.reshape(len(rows), nw, 12)
    if a.raw:
        np.savez_compressed(a.raw, stamps=per)
    # realtime stamps: 100 MHz, one clock for every XCD -> dispatch skew and tail in us
    rt = [(p[:, 8] - p[:, 8].min()) / 100.0 for p in per]
    rte = [(p[:, 9] - p[:, 8].min()) / 100.0 for p in per]
    out["start_us_p50_p90_max"] = [float(np.median([np.percentile(r, q) for r in rt])) for q in (50, 90, 100)]
    out["end_us_p50_p90_max"] = [float(np.median([np.percentile(r, q) for r in rte])) for q in (50, 90, 100)]
    out["wave_life_us_median"] = float(np.median([np.median(e - s) for s, e in zip(rt, rte)]))
    out["wave_life_cycles_median"] = float(np.median(per[:, :, 7] - per[:, :, 0]))
    out["clock_ghz"] = out["wave_life_cycles_median"] / out["wave_life_us_median"] / 1e3
    # the wave that finishes last sets the kernel time: its start and phase breakdown
    crit = []
    for p in per:
        w = int(np.argmax(p[:, 9]))
        ph = np.diff(p[w, :8])
        crit.append([(p[w, 8] - p[:, 8].min()) / 100.0, (p[w, 9] - p[w, 8]) / 100.0] + list(ph))
    crit = np.median(np.array(crit, np.float64), axis=0)
    out["critical_wave"] = {"start_us": crit[0], "life_us": crit[1],
                            "phases_cycles": dict(zip(names, [float(x) for x in crit[2:]]))}
    ev = d[:, 2] > 400  # waves that ran the event path
    rs = d[:, 4] > 400  # waves that ran the reset path
    out["frac_waves_event"] = float(ev.mean())
    out["frac_waves_reset"] = float(rs.mean())
    print(json.dumps(out, indent=1))
    env.close()


if __name__ == "__main__":
    main()
