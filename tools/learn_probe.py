"""Print A2C learning curves on tiny synthetic scenes (diagnostic)."""
import sys, os, time
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))), os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "a2cat-vn-pytorch_amd")]
import numpy as np
import vnav
from oracle.graph import h5_tables
from oracle.frames import synth_frames

maze = np.ones((3, 3), dtype=bool)
graph, spd, _ = h5_tables(maze)
frames = synth_frames(3, np.arange(len(graph)), (84, 84, 3))
scene = vnav.scene_from_arrays(graph, spd, frames)
for tasks in ([(0, 5)], None):
    env = vnav.VectorEnv([scene], 256, seed=1, max_episode_steps=60, tasks=tasks)
    tr = vnav.A2CTrainer(env, num_steps=20, seed=0, max_time_steps=1e9)
    t0 = time.time()
    for u in range(150):
        m = tr.step(sync=(u % 10 == 0))
        if "raw" not in m:
            print(tasks, u, {k: round(v, 4) for k, v in m.items() if k in ("episode_length", "reward", "entropy", "value_loss", "action_loss", "grad_norm", "fps")}, flush=True)
    print("time", time.time() - t0)
