"""Achievable HBM bandwidth of the box this runs on, next to the step kernel's HBM-bound
point (the N = 4 194 304 spread between boxes).

    python tools/hbm_probe.py [--gib 2] [--reps 10]

Times, with HIP events, a device-to-device copy of a --gib GiB fp32 buffer (read + write,
like the step) and a read-only reduction (torch.sum) of it; prints GB/s (1e9 B/s) as the
median over --reps. Both buffers are far past the 256 MiB MALL.
"""
import argparse
import json
import statistics

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=2.0)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    n = int(a.gib * (1 << 30)) // 4
    x = torch.rand(n, device="cuda")
    y = torch.empty_like(x)
    out = {}
    for name, fn, nbytes in (("copy", lambda: y.copy_(x), 2 * 4 * n), ("read", lambda: x.sum(), 4 * n)):
        fn()
        torch.cuda.synchronize()
        rates = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            rates.append(nbytes / (e0.elapsed_time(e1) * 1e-3) / 1e9)
        out[name + "_gbs"] = statistics.median(rates)
    props = torch.cuda.get_device_properties(0)
    out.update({"gib": a.gib, "device": props.name, "cus": props.multi_processor_count,
                "mem_gib": round(props.total_memory / (1 << 30), 1)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
