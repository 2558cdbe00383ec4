"""Time the ways to draw a PPO epoch's permutation of n = 1 M rows on the device with torch:
randperm and sorts of random keys (profiles/r06/perm_native/ also holds a native attempt's row)."""
import json
import sys

import torch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
dev = "cuda:0"
g = torch.Generator(dev).manual_seed(1)
torch.randperm(n, device=dev, generator=g)


def t(name, fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return name, e0.elapsed_time(e1) / reps * 1e3


rows = [
    t("randperm", lambda: torch.randperm(n, device=dev, generator=g)),
    t("argsort_i64_keys", lambda: torch.argsort(torch.randint(-2**63, 2**63 - 1, (n,), device=dev, generator=g))),
    t("sort_i64_keys_unstable", lambda: torch.sort(torch.randint(-2**63, 2**63 - 1, (n,), device=dev, generator=g))[1]),
    t("sort_f32_keys", lambda: torch.sort(torch.rand(n, device=dev, generator=g))[1]),
    t("sort_i32_keys", lambda: torch.sort(torch.randint(0, 2**31 - 1, (n,), device=dev, generator=g,
                                                         dtype=torch.int32))[1]),
    t("batched10_sort_i64_keys_per_epoch", lambda: torch.sort(torch.randint(-2**63, 2**63 - 1, (10, n), device=dev,
                                                                            generator=g), dim=1)[1], reps=5),
]
print(json.dumps({k: round(v, 2) for k, v in rows}))
