"""A/B helper: a few recurrent A2C updates on the small test scene; prints a hash of the
parameters and the episode-length curve, so two builds can be compared bit for bit."""
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "a2cat-vn-pytorch_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import vnav  # noqa: E402
from oracle.graph import h5_tables  # noqa: E402
from oracle.frames import synth_frames  # noqa: E402

graph, spd, _ = h5_tables(np.ones((3, 3), dtype=bool))
frames = synth_frames(3, np.arange(len(graph)), (84, 84, 3))
scene = vnav.scene_from_arrays(graph, spd, frames)
U = int(sys.argv[1]) if len(sys.argv) > 1 else 400
SEED = int(sys.argv[2]) if len(sys.argv) > 2 else 0
LR = float(sys.argv[3]) if len(sys.argv) > 3 else 2e-3
E = int(sys.argv[4]) if len(sys.argv) > 4 else 256
env = vnav.VectorEnv([scene], E, seed=1, max_episode_steps=60, tasks=[(0, 5)])
tr = vnav.A2CTrainer(env, num_steps=20, seed=SEED, max_time_steps=1e9, recurrent=True, learning_rate=LR)
lengths = []
for u in range(U):
    m = tr.step(sync=(u < 20 or u >= U - 10 or u % 20 == 19))
    lengths.append(m.get("episode_length", float("nan")) if "raw" not in m else float("nan"))
    if u % 20 == 19:
        h = hashlib.sha1(tr.params.detach().cpu().numpy().tobytes()).hexdigest()[:12]
        print(u, h, "%.2f" % np.nanmean(lengths[-20:]), flush=True)
