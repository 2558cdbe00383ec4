"""Per-XCD wave start / end (s_memrealtime) and per-wave phase cycles of the headline step from the
RR_DIAG_STAMPS build, for the LAST launch of a K-launch hipGraph replay (K = 1 and 20), the env
restored to the same state before each replay: RR_LIB_PATH=<diag lib> python tools/step_stamps_graph.py OUT.json"""
import os, sys, json
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from rl_rocket_amd.batch import RocketBatch
from rl_rocket_amd.params import ENV_CONFIG_6DOF, MAX_EPISODE_STEPS
dev = torch.device("cuda", 0)
n = 65536
gen = torch.Generator(device=dev).manual_seed(42)
pool = torch.rand((8, n, 3), device=dev, generator=gen) * 2 - 1
out = []
for K in (1, 20):
    env = RocketBatch(n, model=6, device=dev, max_episode_steps=MAX_EPISODE_STEPS, auto_reset=True, episode_stats=False, **ENV_CONFIG_6DOF)
    env.reset()
    for t in range(5):
        env.step(pool[t % 8])
    torch.cuda.synchronize()
    ck = {k: v.clone() for k, v in env.checkpoint().items()}
    s = torch.cuda.Stream(dev); s.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for t in range(K):
                env.step(pool[(5 + t) % 8])
    torch.cuda.current_stream(dev).wait_stream(s)
    for rep in range(6):
        env.restore(ck); torch.cuda.synchronize()
        g.replay(); torch.cuda.synchronize()
        if rep < 2:
            continue
        r = env.reward.cpu().numpy().reshape(-1, 64)
        bits = r[:, 4:6].copy().view(np.uint32).astype(np.int64)
        s0 = bits[:, 0].min()
        st, en = bits[:, 0] - s0, bits[:, 1] - s0
        wave = np.arange(len(st)); xcd = (wave // 4) % 8
        rec = {"graph_launches": K, "start_by_xcd_median_ticks": [float(np.median(st[xcd == x])) for x in range(8)],
               "end_by_xcd_max_ticks": [float(en[xcd == x].max()) for x in range(8)],
               "end_max_us": float(en.max()) / 100.0, "start_spread_us": float(st.max()) / 100.0,
               "cycles_median": [float(v) for v in np.median(r[:, :4], axis=0)],
               "cycles_total_median": float(np.median(r[:, :4].sum(axis=1)))}
        out.append(rec)
        print(json.dumps(rec))
    env.close()
json.dump(out, open(sys.argv[1], "w"), indent=1)
