"""Probe: column sums and Linear bias gradients on hipGraph replays (PyTorch on ROCm).

Each case captures a region after a side-stream warm-up, replays it 4 times with new inputs and
prints the max error per replay against the same computation run eagerly.
  colsum_static   out = x.sum(0), x a static input
  colsum_internal out = tanh(x @ W).sum(0), the summed tensor produced inside the graph
  mm_only         out = (x @ W)[:, 0]
  colsum_elementwise  out = tanh(x).sum(0)
  colsum_mm       out = (x @ W).sum(0)
  mm_full         out = x @ W (every column)
  colsum_mm_ones  out = ones(1, rows) @ (x @ W): the column sum as a GEMM
  colsum_mm_t     out = (x @ W).t().sum(1)
  colsum_mm_clone out = (x @ W).clone().sum(0)
  colsum_mm_2048  out = (x @ W)[:2048].sum(0)
  mlp_bias        grad of the first bias of x -> Linear(14, 64) -> tanh -> Linear(64, 3),
                  torch.autograd.grad into static buffers
"""
import torch

torch.manual_seed(0)
dev = "cuda"


def capture(body):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            body()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    return g


def run(case, rows, cols=64):
    x = torch.randn(rows, 14 if case != "colsum_static" else cols, device=dev)
    W = torch.randn(14, cols, device=dev) * 0.3
    out = torch.zeros(rows if case == "mm_only" else cols, device=dev)
    if case == "mm_full":
        out = torch.zeros(rows, cols, device=dev)
    if case == "colsum_elementwise":
        x = torch.randn(rows, cols, device=dev)
    l1, l2 = torch.nn.Linear(14, cols).to(dev), torch.nn.Linear(cols, 3).to(dev)
    gw = torch.randn(rows, 3, device=dev)
    params = list(l1.parameters()) + list(l2.parameters())
    static = [torch.zeros_like(p) for p in params]

    def eager():
        if case == "colsum_static":
            return [x.sum(0)]
        if case == "colsum_internal":
            return [torch.tanh(x @ W).sum(0)]
        if case == "mm_only":
            return [(x @ W)[:, 0].contiguous()]
        if case == "colsum_elementwise":
            return [torch.tanh(x).sum(0)]
        if case == "colsum_mm":
            return [(x @ W).sum(0)]
        if case == "mm_full":
            return [(x @ W)]
        if case == "colsum_mm_ones":
            return [(torch.ones(1, rows, device=dev) @ (x @ W))[0]]
        if case == "colsum_mm_t":
            return [(x @ W).t().sum(1)]
        if case == "colsum_mm_clone":
            return [(x @ W).clone().sum(0)]
        if case == "colsum_mm_2048":
            return [(x @ W)[:2048].sum(0)]
        loss = (l2(torch.tanh(l1(x))) * gw).mean()
        return list(torch.autograd.grad(loss, params))

    def body():
        r = eager()
        if case == "mlp_bias":
            for b, g in zip(static, r):
                b.copy_(g)
        else:
            out.copy_(r[0])

    g = capture(body)
    errs = []
    for _ in range(4):
        x.copy_(torch.randn_like(x))
        gw.copy_(torch.randn_like(gw))
        g.replay()
        torch.cuda.synchronize()
        ref = eager()
        got = static if case == "mlp_bias" else [out]
        errs.append(max(round((a - b).abs().max().item(), 6) for a, b in zip(got, ref)))
    print(case, rows, cols, "max error per replay:", errs, flush=True)


for rows in (8192, 65536):
    for case in ("colsum_static", "colsum_internal", "mm_only", "colsum_elementwise", "colsum_mm", "mlp_bias",
                 "mm_full", "colsum_mm_ones", "colsum_mm_t", "colsum_mm_clone", "colsum_mm_2048"):
        run(case, rows)
run("colsum_static", 65536, 3)
run("colsum_static", 65536, 1)
