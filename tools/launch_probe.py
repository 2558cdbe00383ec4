"""Per-launch cost of back-to-back tiny kernels (launch + inter-kernel floor), HIP events.

    python tools/launch_probe.py [--k 2000] [--graph]

Runs K launches of a one-element torch kernel (x.add_(1)) back to back, from a hipGraph
(--graph) or issued directly, and prints the per-launch device time by HIP events. Run it
plain and under `rocprofv3 --kernel-trace --stats` to price the profiler's per-dispatch
overhead on a kernel with no work (rocprof vs HIP events).
"""
import argparse
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=2000)
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args()
    x = torch.zeros(1, device="cuda")
    for _ in range(50):
        x.add_(1)
    torch.cuda.synchronize()
    if a.graph:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(a.k):
                    x.add_(1)
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    if a.graph:
        g.replay()
    else:
        for _ in range(a.k):
            x.add_(1)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"k": a.k, "graph": a.graph, "us_per_launch": e0.elapsed_time(e1) * 1e3 / a.k}))


if __name__ == "__main__":
    main()
