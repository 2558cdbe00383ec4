"""Time rr_policy_act alone (hipGraph of 64 launches, HIP events) for one or more library
builds, interleaved (diagnostics for the fused rollout policy kernel).

    python tools/policy_bench.py lib1.so [lib2.so ...] [--n 65536] [--rounds 3] [--prec fp32,bf16]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(n, reps, prec):
    import torch

    from rl_rocket_amd import _lib
    from rl_rocket_amd.batch import _ptr
    from rl_rocket_amd.rollout import MlpActorCritic, PolicyPack

    lib = _lib.load()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    pol = MlpActorCritic(14, 3).to(dev)
    pk = PolicyPack(pol, 14, 3, dev, precision=prec)
    params = pk.pack()
    obs = torch.randn((n, 14), device=dev)
    it = torch.zeros((1,), dtype=torch.int64, device=dev)
    outs = [torch.empty((n, 3), device=dev), torch.empty((n, 3), device=dev), torch.empty((n,), device=dev),
            torch.empty((n,), device=dev), torch.empty((n, 14), device=dev)]

    def call(t):
        _lib.check(lib.rr_policy_act(_ptr(params), 14, 3, pk.prec, n, 0, _ptr(obs), 1, _ptr(it), t, *[_ptr(o) for o in outs],
                                     None, None, None, 0.0, None, None, None,
                                     __import__("ctypes").c_void_p(torch.cuda.current_stream().cuda_stream)),
                   "rr_policy_act")

    for t in range(8):
        call(t)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for t in range(64):
                call(t)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"us_per_call": e0.elapsed_time(e1) * 1e3 / (64 * reps)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--prec", default="fp32", help="comma list of policy precisions (fp32, bf16)")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a.n, a.reps, a.prec)
    keys = [(l, p) for l in (a.libs or [os.path.join(ROOT, "rl_rocket_amd", "librocket_hip.so")])
            for p in a.prec.split(",")]
    res = {k: [] for k in keys}
    for _ in range(a.rounds):
        for l, p in keys:
            env = dict(os.environ, RR_LIB_PATH=os.path.abspath(l))
            out = subprocess.run([sys.executable, __file__, "--child", "--n", str(a.n), "--reps", str(a.reps),
                                  "--prec", p], env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:])
                sys.exit(out.returncode)
            res[(l, p)].append(json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])["us_per_call"])
    print(json.dumps({"n": a.n, "libs": {"%s [%s]" % (os.path.relpath(l, ROOT), p): {"median_us": statistics.median(v),
                                                                                   "runs": v}
                                        for (l, p), v in res.items()}}, indent=1))


if __name__ == "__main__":
    main()
