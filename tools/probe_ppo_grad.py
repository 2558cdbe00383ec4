"""Time the PPO learner pieces on synthetic data of the configs[4] shape (16 x 65 536 samples,
minibatch 65 536, 6DOF MlpPolicy): rr_ppo_grad per call, rr_clip_adam per call, and the graphed
fused update (GraphedPPOUpdate: one graph per epoch, reported per minibatch), by HIP events over
back-to-back calls.

    python tools/probe_ppo_grad.py [--calls 50] [--only grad]   (--only grad: the rocprofv3 --pmc runs)
"""
import argparse
import json
import os
import sys
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rl_rocket_amd.rollout import ClipAdam, GraphedPPOUpdate, MlpActorCritic, PPOGrad


def events(fn, calls):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(calls):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--only", default="")
    ap.add_argument("--T", type=int, default=16)
    ap.add_argument("--n", type=int, default=65536)
    a = ap.parse_args()
    dev = "cuda:0"
    torch.manual_seed(0)
    ns, na, T, n = 14, 3, a.T, a.n
    pol = MlpActorCritic(ns, na).to(dev)
    f = dict(device=dev, dtype=torch.float32)
    ro = types.SimpleNamespace(n_steps=T, env=types.SimpleNamespace(num_envs=n, state_dim=ns, action_dim=na),
                               obs=torch.randn((T, n, ns), **f), actions=torch.randn((T, n, na), **f),
                               log_probs=-4.0 + 0.3 * torch.randn((T, n), **f), advantages=torch.randn((T, n), **f),
                               returns=torch.randn((T, n), **f))
    grad = PPOGrad(pol, ro, n)
    idx = torch.randperm(T * n, device=dev)[:n].contiguous()
    out = {"samples_per_minibatch": n, "grad_us": events(lambda: grad(idx), a.calls)}
    if a.only != "grad":
        opt = torch.optim.Adam(pol.parameters(), lr=3e-4, eps=1e-5, capturable=True)
        adam = ClipAdam(opt, list(pol.parameters()), 0.5)
        out["clip_adam_us"] = events(adam, a.calls)
        opt2 = torch.optim.Adam(pol.parameters(), lr=3e-4, eps=1e-5, capturable=True)
        g = GraphedPPOUpdate(pol, opt2, ro, batch_size=n, fused=True)
        out["graphed_minibatch_us"] = events(g.graph.replay, max(3, a.calls // g.n_mb)) / g.n_mb
        gt = GraphedPPOUpdate(pol, opt2, ro, batch_size=n, fused=False)
        out["graphed_autograd_minibatch_us"] = events(gt.graph.replay, 3) / gt.n_mb
    print(json.dumps(out))


if __name__ == "__main__":
    main()
