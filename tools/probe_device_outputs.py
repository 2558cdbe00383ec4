import time, json, sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from rl_rocket_amd.vec_env import RocketVecEnv
from rl_rocket_amd.params import ENV_CONFIG_6DOF
dev = torch.device("cuda", 0); n = 65536
pool = torch.rand((8, n, 3), device=dev, generator=torch.Generator(device=dev).manual_seed(1)) * 2 - 1
for mon in (True, False):
    v = RocketVecEnv(n, model="6DOF", device=dev, monitor=mon, device_outputs=True, **ENV_CONFIG_6DOF)
    v.reset()
    ts = []
    for k in range(300):
        t0 = time.perf_counter(); v.step(pool[k % 8]); ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    ts = np.array(ts) * 1e6
    print(json.dumps({"monitor": mon, "mean": ts.mean(), "p50": np.median(ts), "p90": np.percentile(ts, 90), "max": ts.max(),
                      "first50": ts[:50].mean(), "mid": ts[50:150].mean(), "last": ts[150:].mean()}))
    v.close()
