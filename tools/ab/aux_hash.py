"""A/B helper for the aux deconv kernels: hashes of forward_deconv outputs (174x174 and 84x84)
and of the parameters after a few A2C updates with the fused aux loss, so two builds can be
compared bit for bit."""
import hashlib
import os
import sys

import numpy as np
import torch

R = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "a2cat-vn-pytorch_amd"))
import vnav  # noqa: E402


def h(t):
    return hashlib.sha1(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()[:12]


for hw in ((174, 174), (84, 84)):
    torch.manual_seed(1)
    pol = vnav.GoalNavPolicy(3, 4, hw, aux=True)
    g = torch.Generator().manual_seed(2)
    img = torch.randint(0, 256, (3, 2) + hw + (3,), dtype=torch.uint8, generator=g).cuda()
    gl = torch.randint(0, 256, (3, 2) + hw + (3,), dtype=torch.uint8, generator=g).cuda()
    heads, _ = pol.forward_deconv(((img, gl), None))
    print(hw, "heads", [h(x) for x in heads], flush=True)

rng = np.random.default_rng(0)
maze = np.ones((5, 5), dtype=bool)
X, Y = maze.shape
obs = rng.integers(0, 256, size=(X, Y, 4, 174, 174, 3), dtype=np.uint8)
dep = rng.integers(0, 256, size=(X, Y, 4, 174, 174, 1), dtype=np.uint8)
seg = rng.integers(0, 256, size=(X, Y, 4, 174, 174, 3), dtype=np.uint8)
scene = vnav.oriented_scene(maze, obs, goals=[(2, 2, 0)], depths=dep, segmentations=seg)
env = vnav.VectorEnv([scene], 64, seed=3, max_episode_steps=50)
tr = vnav.A2CTrainer(env, num_steps=20, seed=0, max_time_steps=1e9, recurrent=True, aux_weight=0.1)
for u in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    m = tr.step(sync=True)
print("params after updates", h(tr.params), "aux_loss %.6f" % m["aux_loss"], flush=True)
