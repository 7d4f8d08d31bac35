"""A/B helper: a few recurrent A2C updates with the aux deconv heads on a synthetic 174x174
scene with depth + segmentation, printing every update's metric dict exactly (float.hex) and a hash
of the parameters, so two builds' metric paths can be compared bit for bit.
usage: train_metrics.py ROOT [updates] [envs]  (ROOT: the tree whose vnav is imported)"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.abspath(sys.argv[1])
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "a2cat-vn-pytorch_amd"))
import vnav  # noqa: E402

U = int(sys.argv[2]) if len(sys.argv) > 2 else 12
E = int(sys.argv[3]) if len(sys.argv) > 3 else 4
rng = np.random.default_rng(5)
scene = vnav.synthetic_scene(0, frame_shape=(174, 174, 3))
scene.depth = rng.integers(0, 256, size=(scene.n_states, 174, 174, 1), dtype=np.uint8)
scene.segmentation = rng.integers(0, 256, size=(scene.n_states, 174, 174, 3), dtype=np.uint8)
scene.__post_init__()
env = vnav.VectorEnv([scene], E, seed=1, max_episode_steps=60)
tr = vnav.A2CTrainer(env, num_steps=20, seed=3, max_time_steps=1e9, recurrent=True, learning_rate=2e-3,
                     aux_weight=0.1)
for u in range(U):
    m = tr.step(sync=True)
    print(u, " ".join("%s=%s" % (k, float(v).hex()) for k, v in sorted(m.items()) if isinstance(v, float)))
print("params", hashlib.sha1(tr.params.detach().cpu().numpy().tobytes()).hexdigest()[:12])
