import copy, sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
from rl_rocket_amd.batch import RocketBatch
from rl_rocket_amd.params import ENV_CONFIG_6DOF
from rl_rocket_amd.rollout import DeviceRollout, GraphedPPOUpdate, ppo_update
from test_gpu_rollout import _policy
n, T, bs = 8192, 8, 8192
env = RocketBatch(n, model=6, device="cuda:0", max_episode_steps=30, **ENV_CONFIG_6DOF)
pol = _policy(14, 3, seed=7)
ro = DeviceRollout(env, pol, n_steps=T, seed=3)
ro.collect(); torch.cuda.synchronize()
pa, pb, pc = copy.deepcopy(pol), copy.deepcopy(pol), copy.deepcopy(pol)
oa = torch.optim.Adam(pa.parameters(), lr=3e-4, eps=1e-5, capturable=True)
ob = torch.optim.Adam(pb.parameters(), lr=3e-4, eps=1e-5, capturable=True)
oc = torch.optim.Adam(pc.parameters(), lr=3e-4, eps=1e-5, capturable=True)
MG = float(os.environ.get("MG", "0.5"))
g = GraphedPPOUpdate(pb, ob, ro, batch_size=bs, max_grad_norm=MG, fused=False)
# eager, with the graph object's own _step on a third copy through an eager GraphedPPOUpdate-like loop
perm = torch.randperm(n * T, device="cuda:0", generator=torch.Generator("cuda:0").manual_seed(5))
for s in range(0, n * T, bs):
    idx = perm[s:s + bs]
    # eager a
    mean, value = pa(ro.obs.reshape(n*T,-1)[idx]); lp = pa.log_prob(mean, ro.actions.reshape(n*T,-1)[idx])
    adv = ro.advantages.reshape(-1)[idx]; adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    ratio = torch.exp(lp - ro.log_probs.reshape(-1)[idx])
    pg = -torch.min(adv * ratio, adv * torch.clamp(ratio, 0.8, 1.2)).mean()
    vf = torch.nn.functional.mse_loss(ro.returns.reshape(-1)[idx], value)
    ent = -pa.entropy(bs).mean(); loss = pg + 0.01 * ent + 0.5 * vf
    oa.zero_grad(set_to_none=True); loss.backward(); torch.nn.utils.clip_grad_norm_(pa.parameters(), MG); oa.step()
    g.idx.copy_(idx); g.graph.replay()
    torch.cuda.synchronize()
    da = max((x - y).abs().max().item() for x, y in zip(pa.parameters(), pb.parameters()))
    ga = max((x.grad - y.grad).abs().max().item() for x, y in zip(pa.parameters(), pb.parameters()))
    names = [k for k, _ in pa.named_parameters()]
    per = {k: round((x.grad - y.grad).abs().max().item(), 6) for k, x, y in zip(names, pa.parameters(), pb.parameters())}
    if s // bs in (1, 2):
        print(per)
    print(s // bs, "param diff", da, "grad diff", ga, "loss", float(pg), float(g.stats["policy_loss"]), float(vf), float(g.stats["value_loss"]),
          "step", float(oa.state[next(pa.parameters())]["step"]), float(ob.state[next(pb.parameters())]["step"]))
