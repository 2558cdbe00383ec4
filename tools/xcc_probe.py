"""Diagnostic: is the round-robin block -> XCD deal stable enough for an XCD-affine map?
Steps N envs with a library built with the XCD-affine block map (RR_LIB_PATH) and checks
that the step outputs equal a reference library's bit for bit (every env group stepped once)."""
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(lib, n, steps):
    code = r'''
import torch, sys
sys.path.insert(0, %r)
from rl_rocket_amd.batch import RocketBatch
from rl_rocket_amd.params import ENV_CONFIG_6DOF
b = RocketBatch(%d, model=6, device="cuda:0", max_episode_steps=800, **ENV_CONFIG_6DOF)
b.reset()
g = torch.Generator(device="cuda:0"); g.manual_seed(3)
for _ in range(%d):
    o, r, d, t = b.step(torch.rand((%d, 3), device="cuda:0", generator=g) * 2 - 1)
torch.save([o.cpu(), r.cpu(), d.cpu(), b.get_state()[0].cpu()], %r)
''' % (ROOT, n, steps, n, "/tmp/xcc_%s.pt" % os.path.basename(lib))
    subprocess.check_call([sys.executable, "-c", code], env=dict(os.environ, RR_LIB_PATH=lib))
    return torch.load("/tmp/xcc_%s.pt" % os.path.basename(lib))


if __name__ == "__main__":
    a = run(sys.argv[1], 65536, 50)
    b = run(sys.argv[2], 65536, 50)
    print("bitwise equal:", all(torch.equal(x, y) for x, y in zip(a, b)))
