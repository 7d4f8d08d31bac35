"""A/B: A2CTrainer with and without goal-frame deduplication, same seeds, U updates each,
never re-synchronised. Per reported update: the largest parameter difference relative to the
parameter scale, whether the two rollouts sampled the same actions, and both runs' episode
lengths. Usage: python tools/ab/dedup_drift.py [updates] [envs] [hw] [aux|noaux] [control]
control: both runs WITHOUT deduplication, the second with VN_WGRAD_GENERIC=1 (the generic
split-K weight-gradient products: the same gradients in another summation order) — the
drift any fp32 reordering shows, the baseline for the deduplicated run's."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
for p in (ROOT, os.path.join(ROOT, "a2cat-vn-pytorch_amd")):
    sys.path.insert(0, p)
import vnav  # noqa: E402
from bench import aux_scenes  # noqa: E402

U = int(sys.argv[1]) if len(sys.argv) > 1 else 40
E = int(sys.argv[2]) if len(sys.argv) > 2 else 256
HW = int(sys.argv[3]) if len(sys.argv) > 3 else 84
AUX = len(sys.argv) > 4 and sys.argv[4] == "aux"
CONTROL = len(sys.argv) > 5 and sys.argv[5] == "control"
scenes = aux_scenes(2, (HW, HW, 3)) if AUX else [vnav.synthetic_scene(k, frame_shape=(HW, HW, 3)) for k in range(2)]
runs = []
for dedup in ((False, False) if CONTROL else (True, False)):
    env = vnav.VectorEnv(scenes, E, seed=5, max_episode_steps=12)
    runs.append(vnav.A2CTrainer(env, num_steps=20, seed=3, max_time_steps=1e9, recurrent=True,
                                aux_weight=0.1 if AUX else 0.0, dedup_goals=dedup, learning_rate=2e-3))
a, b = runs
print("hw %d envs %d aux %s dedup %s / %s%s" % (HW, E, AUX, a.dedup_goals, b.dedup_goals,
                                               "  (control: second run on the generic weight-gradient products)"
                                               if CONTROL else ""))
same_actions = True
for u in range(U):
    ma = a.step(sync=True)
    if CONTROL:
        os.environ["VN_WGRAD_GENERIC"] = "1"
    mb = b.step(sync=True)
    os.environ.pop("VN_WGRAD_GENERIC", None)
    same_actions = same_actions and bool(torch.equal(a.actions, b.actions))
    scale = float(b.params.abs().max())
    d = float((a.params - b.params).abs().max()) / scale
    T = a.num_steps
    g = a.goal_count.cpu().numpy() if a.dedup_goals else np.full(T + 1, E)
    if u < 5 or u % 5 == 4:
        print("update %3d  param diff %.3g of scale  actions identical so far: %s  ep.len %.2f / %.2f  "
              "goal frames computed %.3f" % (u + 1, d, same_actions, ma["episode_length"], mb["episode_length"],
                                              g[:T].sum() / (T * E)), flush=True)
