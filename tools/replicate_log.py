#!/usr/bin/env python3
"""Replay the reference's one logged training run (outputs/output.txt, thor-cached-auxiliary)
with the engine at the same shape and hyper-parameters, and print both learning curves.

Reference run (experiments/thor_cached_auxiliary.py:26-84, outputs/output.txt): 4 envs of
AuxiliaryGraph-v0 (GoalGymGraphAuxiliaryEnv over the 174x174 scene thor-cached-212-174,
fixed goal (10, 14, 0), TimeLimit 900), hardness set_complexity(0.01), num_steps 20,
gamma 0.99, RMSprop(alpha .99, eps 1e-5), lr 7e-4 -> 0 over max_time_steps 2e6, grad-norm
clip 0.5, AuxiliaryBigGoalHouseModel (LSTM + deconv heads), auxiliary_weight 0.1; 1e6
env-steps (12,500 updates of 80).

Here: the same settings on a synthetic 174x174 oriented grid scene (the pickled THOR scene
is a download, not in the image) whose frames, depth and segmentation are fixed random
images per (cell, rotation); the UNREAL replay losses (pixel control, reward prediction,
value replay) are deep_rl's and not part of the engine. What is compared is the shape of
the curve: episode length from the random-walk level down to a few steps, reward -> 1.

    python tools/replicate_log.py [updates] [out.csv] [--entropy-coef C] [--seed S] [--aux-weight W]
    python tools/replicate_log.py [updates] [out.csv] --experiment [--seed S]   # vnav.train's trainer

The options exist for the late-entropy investigation (DESIGN.md "End-to-end check"): the same
run with another entropy coefficient / seed / aux weight. Each 10k-step row also carries the
mean pre-clip gradient norm and the fraction of updates the 0.5 clip scaled down.
"""
import csv
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "a2cat-vn-pytorch_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import vnav  # noqa: E402

# the reference log's rows sampled every 10k env-steps (outputs/output.txt, extracted in the
# build container; the reference tree is not on the GPU box)
REF_CURVE = os.path.join(REPO, "tools", "data", "reference_log_curve.csv")


def reference_curve():
    """(step, reward, episode_length, entropy, aux_loss) rows of the reference log."""
    if not os.path.exists(REF_CURVE):
        return []
    with open(REF_CURVE) as f:
        return [(int(r["step"]), float(r["reward"]), float(r["episode_length"]), float(r["entropy"]),
                 float(r["aux_loss"])) for r in csv.DictReader(f)]


def make_scene(seed=0, grid=(16, 16), frame=(174, 174)):
    rng = np.random.default_rng(seed)
    maze = rng.random(grid) >= 0.25
    maze[10, 14] = True
    # keep the goal's 4-connected component
    from scipy.ndimage import label
    lab, _ = label(maze)
    maze = lab == lab[10, 14]
    X, Y = grid
    h, w = frame
    obs = rng.integers(0, 256, size=(X, Y, 4, h, w, 3), dtype=np.uint8)
    depth = rng.integers(0, 256, size=(X, Y, 4, h, w, 1), dtype=np.uint8)
    seg = rng.integers(0, 256, size=(X, Y, 4, h, w, 3), dtype=np.uint8)
    return vnav.oriented_scene(maze, obs, goals=[(10, 14, 0)], name="synthetic-oriented-174",
                               depths=depth, segmentations=seg)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("updates", nargs="?", type=int, default=12500)
    ap.add_argument("out", nargs="?", default=None)
    ap.add_argument("--entropy-coef", type=float, default=0.01)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--aux-weight", type=float, default=0.1)
    ap.add_argument("--experiment", action="store_true",
                    help="the trainer of vnav.train's thor-cached-auxiliary as registered (UNREAL losses, replayed "
                         "aux batches, its entropy cost; the other options are ignored)")
    a = ap.parse_args()
    updates, out = a.updates, a.out
    torch.cuda.set_device(0)
    if a.experiment:
        from vnav.train import make_trainer
        exp = make_trainer("thor-cached-auxiliary", seed=a.seed, save=False, logger=None)
        tr = exp._setup()
        print("experiment thor-cached-auxiliary: envs %d, entropy %g, aux %g (%s), unreal %s, dedup %s"
              % (tr.env.num_envs, tr.entropy_coefficient, tr.aux_weight, tr.aux_source, tr.unreal, tr.dedup_goals),
              flush=True)
    else:
        scene = make_scene()
        env = vnav.VectorEnv([scene], 4, seed=1 + a.seed, max_episode_steps=900)
        env.set_complexity(0.01)
        tr = vnav.A2CTrainer(env, num_steps=20, seed=a.seed, max_time_steps=2e6, recurrent=True,
                             aux_weight=a.aux_weight, entropy_coefficient=a.entropy_coef)
    ref = reference_curve()
    rows = []
    t0 = time.time()
    window = []
    for u in range(updates):
        m = tr.step(sync=True)
        window.append(m)
        if (u + 1) % 125 == 0:  # every 10k env-steps
            eps = sum(x["episodes"] for x in window)
            rsum = sum(x["reward"] * x["episodes"] for x in window if x["episodes"])
            lsum = sum(x["episode_length"] * x["episodes"] for x in window if x["episodes"])
            row = dict(step=m["step"], episodes=eps, reward=rsum / eps if eps else float("nan"),
                       episode_length=lsum / eps if eps else float("nan"),
                       entropy=float(np.mean([x["entropy"] for x in window])),
                       aux_loss=float(np.mean([x.get("aux_loss", 0.0) for x in window])),
                       grad_norm=float(np.mean([x["grad_norm"] for x in window])),
                       clipped=float(np.mean([x["grad_norm"] > tr.max_gradient_norm for x in window])),
                       wall_s=time.time() - t0)
            if tr.unreal:
                for k in ("pc_loss", "rp_loss", "vr_loss"):
                    row[k] = float(np.mean([x[k] for x in window]))
            rr = [r for r in ref if r[0] <= row["step"]]
            if rr:
                row.update(ref_reward=rr[-1][1], ref_episode_length=rr[-1][2], ref_entropy=rr[-1][3],
                           ref_aux_loss=rr[-1][4])
            rows.append(row)
            print({k: (round(v, 4) if isinstance(v, float) else v) for k, v in row.items()}, flush=True)
            window = []
    if out:
        with open(out, "w", newline="") as f:
            wr = csv.DictWriter(f, fieldnames=list(rows[-1].keys()))
            wr.writeheader()
            for r in rows:
                wr.writerow({k: r.get(k, "") for k in rows[-1].keys()})
    print("done: %d updates in %.1f s" % (updates, time.time() - t0))


if __name__ == "__main__":
    main()
