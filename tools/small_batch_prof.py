"""The logged run's shape (174x174, LSTM + aux heads, 4 envs x 20 steps) for a few updates:
run under rocprofv3 --kernel-trace to see per-kernel costs at tiny batch."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "a2cat-vn-pytorch_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import vnav  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 4
graph = len(sys.argv) > 2 and sys.argv[2] == "graph"
torch.cuda.set_device(0)
sc = bench.aux_scenes(4, (174, 174, 3))
env = vnav.VectorEnv(sc, E, seed=3)
tr = vnav.A2CTrainer(env, num_steps=20, seed=1, max_time_steps=1e12, recurrent=True, aux_weight=0.1, cuda_graph=graph)
for _ in range(8):
    tr.step(sync=False)
torch.cuda.synchronize()
print("done")
