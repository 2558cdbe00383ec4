"""Driver of tools/coissue_probe.hip (measurement only): per-launch time of the three roles by
HIP events over hipGraph replays, for a few MFMA / VALU stream lengths. Prints one JSON line.

    python tools/coissue_probe.py [--out FILE]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tools", "libcoissue_probe.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import torch

    lib = ctypes.CDLL(LIB)
    P = ctypes.c_void_p
    lib.cp_launch.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, P]
    dev = torch.device("cuda", 0)
    out = torch.zeros((256 * 512,), device=dev)
    res = {"what": "2 waves per SIMD (256 workgroups x 8 waves); role 0 MFMA only, 1 VALU only, 2 one of each per "
                   "SIMD; m rounds of 4 fp32 32x32x2 MFMAs, v rounds of 4 v_fma_f32; role 3 v rounds of 4 v_exp_f32, "
                   "4 one MFMA wave + one exp wave per SIMD, 5 one stream with 2 v_exp_f32 after each MFMA",
           "runs": []}

    def timed(role, m, v):
        def go():
            rc = lib.cp_launch(role, 256, P(out.data_ptr()), m, v, P(torch.cuda.current_stream(dev).cuda_stream))
            if rc:
                raise RuntimeError("cp_launch: %d" % rc)
        go()
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(a.reps):
                    go()
        torch.cuda.current_stream(dev).wait_stream(s)
        g.replay()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / a.reps * 1e3

    for m, v in ((32, 512), (64, 1024), (128, 2048), (64, 0), (0, 1024)):
        row = {"m": m, "v": v}
        for role in (0, 1, 2):
            row["role%d_us" % role] = timed(role, m, v)
        res["runs"].append(row)
        print(json.dumps(row), flush=True)
    # transcendentals (v_exp_f32) beside / between fp32 MFMAs: role 3 exp alone, 4 one MFMA wave and
    # one exp wave per SIMD, 5 both in one stream (2 exps after each MFMA); role 0 / 3 at the same m / v
    # are the references (role 5 issues 8 exps per round of 4 MFMAs: v = 2 m rounds of 4 exps)
    for m in (32, 64, 128):
        v = 2 * m
        row = {"m": m, "v_exp": v}
        for role in (0, 3, 4, 5):
            row["role%d_us" % role] = timed(role, m, v)
        res["runs"].append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    sys.exit(main())
