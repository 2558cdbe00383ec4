"""Probe: ways to take a Linear's bias gradient (the column sum of g [rows, cols]) on MI355X —
device time per call (HIP events over 200 back-to-back calls) and correctness on hipGraph replays
after a GEMM in the same graph (see tools/probe_graph_reduce.py).

  sum0        g.sum(0)                                   (wrong on graph replays after a GEMM)
  ones_mm     ones(1, rows) @ g
  ones_mm2    two stages: ones(1, 256) @ g.view(256, -1), then ones(1, rows/256) @ that
  aug_gemm    the weight-gradient GEMM with a ones column appended to x: g.T @ [x, 1]
              (the cost beyond the plain weight GEMM g.T @ x, which is timed as weight_gemm)
"""
import torch

dev = "cuda"
torch.manual_seed(0)


def timed(fn, reps=200):
    for _ in range(10):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def variants(x, g, rows):
    xa = torch.cat([x, x.new_ones(rows, 1)], 1)
    return {
        "sum0": lambda: g.sum(0),
        "ones_mm": lambda: (g.new_ones(1, rows) @ g)[0],
        "ones_mm2": lambda: (g.new_ones(1, rows // 256) @ (g.new_ones(1, 256) @ g.view(256, -1)).view(rows // 256, -1))[0],
        "weight_gemm": lambda: g.t() @ x,
        "aug_gemm": lambda: (g.t() @ xa)[:, -1],
        "aug_cat_gemm": lambda: (g.t() @ torch.cat([x, x.new_ones(rows, 1)], 1))[:, -1],
    }


def graph_check(name, rows, cin, cols):
    x = torch.randn(rows, cin, device=dev)
    W = torch.randn(cin, cols, device=dev)
    xin = torch.randn(rows, cin, device=dev)
    out = torch.zeros(cols, device=dev)

    def body():
        g = torch.tanh(xin @ W)  # the summed tensor comes from a GEMM in the graph
        out.copy_(variants(x, g, rows)[name]() if name != "weight_gemm" else g.sum(0))

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            body()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        body()
    err = []
    for _ in range(3):
        xin.copy_(torch.randn_like(xin))
        gr.replay()
        torch.cuda.synchronize()
        err.append(round((out - torch.tanh(xin @ W).sum(0)).abs().max().item() / max(1.0, torch.tanh(xin @ W).sum(0).abs().max().item()), 7))
    return err


for rows, cin, cols in ((65536, 64, 64), (65536, 14, 64), (65536, 64, 3), (65536, 64, 1), (8192, 64, 64)):
    x = torch.randn(rows, cin, device=dev)
    g = torch.randn(rows, cols, device=dev)
    res = {k: round(timed(f), 2) for k, f in variants(x, g, rows).items()}
    ref = g.sum(0)
    acc = {k: float((f().reshape(-1)[:cols] - ref).abs().max()) if k not in ("weight_gemm",) else 0.0
           for k, f in variants(x, g, rows).items()}
    print("rows %d cin %d cols %d  us per call:" % (rows, cin, cols), res, flush=True)
    print("   max |err| vs sum0 (eager):", {k: round(v, 5) for k, v in acc.items()}, flush=True)
    print("   graph replays rel err:", {k: graph_check(k, rows, cin, cols) for k in ("sum0", "ones_mm", "ones_mm2", "aug_gemm")}, flush=True)
