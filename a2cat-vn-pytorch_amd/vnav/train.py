"""The reference's experiment entry points over vnav: ``register_trainer`` / ``make_trainer``
/ ``Trainer.run()`` / ``Trainer.test()`` and the ``train.py NAME`` / ``test-train.py NAME``
command line (train.py:10-25, test-train.py:11-26; the Trainer surface is deep_rl's,
driven by experiments/thor_cached_auxiliary.py:26-84).

    python -m vnav.train thor-cached-auxiliary [--scene thor-cached-212-174.pkl] [--save-dir D]
    python -m vnav.train thor-cached-auxiliary --test [--episodes 100]      # test-train.py
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m vnav.train cached-thor --envs 4096

An experiment is a class registered under its name with the deep_rl trainer arguments
(max_time_steps, validation_period, validation_episodes, episode_log_interval,
saving_period, save) and the reference's hyper-parameters as attributes; ``create_env``
builds the batched VectorEnv (one process per GPU instead of one per env) and
``create_trainer`` the A2CTrainer. ``run()`` trains to max_time_steps, prints deep_rl's
metric table every ``episode_log_interval`` finished episodes and saves a checkpoint every
``saving_period`` env-steps (and at the end); ``test()`` loads that checkpoint and runs
``validation_episodes`` episodes of the policy. Scenes the reference downloads (the pickled
THOR grids) are loaded from ``--scene`` when given; otherwise a synthetic scene of the same
geometry stands in (no network in this image).
"""
import argparse
import os
import time

import numpy as np
import torch

from . import dist as vdist
from .a2c import A2CTrainer
from .envs import VectorEnv
from .scenes import load_graph_pickle, load_h5, load_npz, oriented_scene, synthetic_scene

_TRAINERS = {}


def register_trainer(name, max_time_steps=None, validation_period=None, validation_episodes=None,
                     episode_log_interval=None, saving_period=None, save=True):
    """deep_rl's ``@register_trainer(...)`` (experiments/thor_cached_auxiliary.py:26): the
    decorated experiment class is made by ``make_trainer(name)`` with these attributes."""
    def wrap(cls):
        cls.name = name
        cls.max_time_steps = max_time_steps
        cls.validation_period = validation_period
        cls.validation_episodes = validation_episodes
        cls.episode_log_interval = episode_log_interval
        cls.saving_period = saving_period
        cls.save = save
        _TRAINERS[name] = cls
        return cls
    return wrap


def make_trainer(name, env_kwargs=None, model_kwargs=None, **kwargs):
    """deep_rl's ``make_trainer(name, **default_args())`` (train.py:24)."""
    if name not in _TRAINERS:
        raise KeyError("unknown experiment %r (registered: %s)" % (name, sorted(_TRAINERS)))
    return _TRAINERS[name](env_kwargs=env_kwargs or {}, model_kwargs=model_kwargs or {}, **kwargs)


def registered():
    return sorted(_TRAINERS)


def _format_table(metrics):
    """deep_rl's logger table (outputs/output.txt)."""
    keys = ["step"] + sorted(k for k in metrics if k != "step")
    rows = []
    for k in keys:
        v = metrics[k]
        if isinstance(v, float):
            v = "%.3g" % v
        rows.append((k, str(v)))
    w1 = max(len(k) for k, _ in rows) + 2
    w2 = max(8, max(len(v) for _, v in rows))
    line = "-" * (w1 + w2 + 6)
    return "\n".join([line] + ["| %-*s| %-*s |" % (w1, k, w2, v) for k, v in rows] + [line])


class Experiment:
    """Base of the registered experiments: hyper-parameters as attributes (the deep_rl
    Trainer fields the reference sets), create_env / create_trainer hooks, run / test."""

    name = None
    max_time_steps = 2e6
    validation_period = None
    validation_episodes = None
    episode_log_interval = 10
    saving_period = 100000
    save = True
    # A2C / RMSprop (experiments/thor_cached_auxiliary.py:29-37)
    num_processes = 4
    num_steps = 20
    gamma = 0.99
    learning_rate = 7e-4
    rms_alpha = 0.99
    rms_epsilon = 1e-5
    max_gradient_norm = 0.5
    # loss coefficients (deep_rl's, absent: A2C's 0.5 / 0.01; see ThorCachedAuxiliary)
    value_coefficient = 0.5
    entropy_coefficient = 0.01
    recurrent = True
    auxiliary_weight = 0.0
    hardness = None
    cuda_graph = False
    capture_collectives = False  # cuda_graph at world > 1 (captured RCCL): explicit opt-in only
    aux_source = "rollout"
    # UnrealTrainer's pixel-control / reward-prediction / value-replay losses (deep_rl, absent:
    # parity unpinned) on the UNREAL heads of BigGoalHouseModel (goal.py:94-137)
    unreal = False
    unreal_source = "rollout"
    rp_weight = 1.0
    pc_weight = 0.05
    vr_weight = 1.0

    def __init__(self, env_kwargs=None, model_kwargs=None, save_dir=None, seed=0, device=None, logger=print,
                 **overrides):
        for k, v in overrides.items():
            if not hasattr(type(self), k):
                raise TypeError("unknown experiment attribute %r" % k)
            setattr(self, k, v)
        self.env_kwargs = dict(env_kwargs or {})
        self.model_kwargs = dict(model_kwargs or {})
        self.seed = int(seed)
        self.rank, self.world, local = vdist.env_rank()
        if device is None:
            device = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
        self.device = torch.device(device)
        self.save_dir = save_dir or os.path.join(os.path.expanduser("~/.visual_navigation/models"), self.name)
        self.logger = logger
        self.env = None
        self.trainer = None

    # --- hooks (deep_rl names)
    def create_env(self, kwargs):
        raise NotImplementedError

    def create_trainer(self):
        return A2CTrainer(self.env, num_steps=self.num_steps, gamma=self.gamma, learning_rate=self.learning_rate,
                          max_time_steps=self.max_time_steps, rms_alpha=self.rms_alpha,
                          rms_epsilon=self.rms_epsilon, max_gradient_norm=self.max_gradient_norm,
                          value_coefficient=self.value_coefficient, entropy_coefficient=self.entropy_coefficient,
                          seed=self.seed, recurrent=self.recurrent,
                          aux_weight=self.auxiliary_weight, aux_source=self.aux_source,
                          # the 42x42 pixel-control map crops 168 px (goal.py:72, 112): smaller
                          # stand-in frames train without the UNREAL losses
                          unreal=self.unreal and min(self.env.frame_shape[:2]) >= 168,
                          pc_weight=self.pc_weight, rp_weight=self.rp_weight,
                          vr_weight=self.vr_weight, unreal_source=self.unreal_source,
                          # world > 1: only on explicit opt-in (the captured RCCL path is unvalidated)
                          cuda_graph=self.cuda_graph and (self.world == 1 or self.capture_collectives),
                          capture_collectives=self.capture_collectives)

    def _setup(self):
        if self.trainer is None:
            torch.cuda.set_device(self.device)
            self.env = self.create_env(self.env_kwargs)
            if self.hardness is not None:
                # experiments/thor_cached_auxiliary.py:68-70 sets it before the first reset;
                # the VectorEnv constructor already reset, so draw the starts again
                self.env.set_hardness(self.hardness)
                self.env.reset()
            self.trainer = self.create_trainer()
        return self.trainer

    @property
    def checkpoint_path(self):
        """save_dir/checkpoint.pt. One process: the whole trainer state. world > 1: the
        world-agnostic parameters + RMSprop state that rank 0 writes once every rank's own
        state is on disk (what ``test()`` in a single process loads); the per-rank states
        (env shard, running returns, recurrent carry) live in ``rank_checkpoint_path()``."""
        return os.path.join(self.save_dir, "checkpoint.pt")

    def _generation_dir(self, total_steps):
        return os.path.join(self.save_dir, "ckpt-%012d" % int(total_steps))

    def rank_checkpoint_path(self, total_steps=None):
        """This rank's file of the last complete checkpoint set (world > 1), or of the set
        at ``total_steps``. None when no complete set exists."""
        if total_steps is None:
            latest = self._latest()
            if latest is None:
                return None
            total_steps = latest["total_steps"]
        return os.path.join(self._generation_dir(total_steps), "rank%d.pt" % self.rank)

    def _latest(self):
        """latest.json: the complete per-rank checkpoint set (written by rank 0 after every
        rank has saved)."""
        import json
        p = os.path.join(self.save_dir, "latest.json")
        if not os.path.exists(p):
            return None
        with open(p) as f:
            return json.load(f)

    @staticmethod
    def _atomic_save(obj, path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tmp = path + ".tmp"
        torch.save(obj, tmp)
        os.replace(tmp, path)

    def save_checkpoint(self, path=None):
        """One process: checkpoint.pt. world > 1 (collective: every rank calls it): each rank
        writes its state into the generation directory ckpt-<total_steps>/rank<r>.pt; after a
        barrier rank 0 writes the world-agnostic checkpoint.pt and then latest.json (the
        commit point: a crash before it leaves the previous complete set in force) and drops
        older generations. Resume therefore never mixes ranks of different updates."""
        tr = self.trainer
        if self.world == 1:
            path = path or self.checkpoint_path
            self._atomic_save(tr.state_dict(), path)
            return path
        step = tr.total_steps
        self._atomic_save(tr.state_dict(), self.rank_checkpoint_path(step))
        torch.distributed.barrier()
        if self.rank == 0:
            import json
            import shutil
            self._atomic_save(tr.params_state_dict(), self.checkpoint_path)
            tmp = os.path.join(self.save_dir, "latest.json.tmp")
            with open(tmp, "w") as f:
                json.dump({"total_steps": step, "num_updates": tr.num_updates, "world": self.world}, f)
            os.replace(tmp, os.path.join(self.save_dir, "latest.json"))
            keep = os.path.basename(self._generation_dir(step))
            for d in os.listdir(self.save_dir):
                if d.startswith("ckpt-") and d != keep:
                    shutil.rmtree(os.path.join(self.save_dir, d), ignore_errors=True)
        torch.distributed.barrier()
        return self.rank_checkpoint_path(step)

    def has_checkpoint(self):
        if self.world == 1:
            return os.path.exists(self.checkpoint_path)
        latest = self._latest()
        return latest is not None and os.path.exists(self.rank_checkpoint_path(latest["total_steps"]))

    def _resume_decision(self):
        """Whether run(resume=True) loads: this rank's has_checkpoint(), agreed by all ranks
        (load_checkpoint is collective). Ranks that disagree — a save_dir that is not shared,
        one rank's file missing — raise on every rank instead of leaving some ranks in the
        load's collectives and others in the first gradient all-reduce."""
        have = self.has_checkpoint()
        if self.world == 1:
            return have
        self._setup()
        vdist.check_ranks_agree([int(have)], "whether a checkpoint exists to resume from (has_checkpoint)")
        return have

    def load_checkpoint(self, path=None):
        """One process: checkpoint.pt (or ``path``). world > 1 (collective): this rank's file
        of the complete set named by latest.json; then the ranks check that they agree on the
        update and step counters (all-reduce min / max: a mismatch would leave one rank
        blocked in the gradient all-reduce) and take rank 0's parameters and RMSprop state."""
        tr = self._setup()
        if self.world == 1:
            tr.load_state_dict(torch.load(path or self.checkpoint_path, map_location="cpu", weights_only=True))
            return self
        latest = self._latest()
        if latest is None:
            raise FileNotFoundError("no complete checkpoint set in %s (latest.json missing)" % self.save_dir)
        if int(latest["world"]) != self.world:
            raise ValueError("checkpoint set of world %d resumed at world %d" % (int(latest["world"]), self.world))
        tr.load_state_dict(torch.load(path or self.rank_checkpoint_path(latest["total_steps"]), map_location="cpu",
                                      weights_only=True))
        vdist.check_ranks_agree([tr.num_updates, tr.total_steps], "checkpoint counters (num_updates, total_steps)")
        vdist.broadcast_params_(tr.params)
        vdist.broadcast_params_(tr.square_avg)
        return self

    def _log(self, m):
        """deep_rl's console table, and the same row appended to save_dir/metrics.jsonl."""
        if self.rank != 0:
            return
        if self.logger:
            self.logger(_format_table(m))
        if self.save:
            import json
            os.makedirs(self.save_dir, exist_ok=True)
            with open(os.path.join(self.save_dir, "metrics.jsonl"), "a") as f:
                f.write(json.dumps(m) + "\n")

    def run(self, resume=False):
        """Train to max_time_steps: deep_rl's Trainer.run() (train.py:25). resume=True
        continues from save_dir's checkpoint when there is one (parameters, RMSprop state,
        per-env state and running returns, recurrent carry, update / step counters)."""
        if resume and self._resume_decision():
            self.load_checkpoint()
        tr = self._setup()
        window = dict(episodes=0.0, rsum=0.0, lsum=0.0)
        last = None
        next_save = (tr.total_steps // self.saving_period + 1) * self.saving_period if self.saving_period else None
        t0, s0 = time.perf_counter(), tr.total_steps
        while tr.total_steps < self.max_time_steps:
            m = tr.step(sync=True)
            last = m
            if m["episodes"]:
                window["episodes"] += m["episodes"]
                window["rsum"] += m["reward"] * m["episodes"]
                window["lsum"] += m["episode_length"] * m["episodes"]
            if self.episode_log_interval and window["episodes"] >= self.episode_log_interval:
                now = time.perf_counter()
                row = {k: m[k] for k in ("step", "updates", "value_loss", "action_loss", "entropy", "loss")}
                if "aux_loss" in m:
                    row["aux_loss"] = m["aux_loss"]
                row.update(episodes=int(window["episodes"]), reward=window["rsum"] / window["episodes"],
                           episode_length=window["lsum"] / window["episodes"],
                           fps=int((tr.total_steps - s0) / max(now - t0, 1e-9)))
                self._log(row)
                window = dict(episodes=0.0, rsum=0.0, lsum=0.0)
                t0, s0 = now, tr.total_steps
            if self.save and next_save is not None and tr.total_steps >= next_save:
                self._saving(self.save_checkpoint())
                next_save += self.saving_period
        if self.save:
            self._saving(self.save_checkpoint())
        return last

    def _saving(self, path):
        if self.rank == 0 and self.logger:
            self.logger("Saving %s (step %d)" % (path, self.trainer.total_steps))  # outputs/output.txt:462

    def test(self, episodes=None, checkpoint=None):
        """deep_rl's Trainer.test() (test-train.py:26): the saved policy over ``episodes``
        (default validation_episodes, else 100) episodes. Reads save_dir/checkpoint.pt (or
        ``checkpoint``), whichever world wrote it: the policy parameters are world-agnostic,
        a single-process file also restores its env state. Raises FileNotFoundError when
        there is no checkpoint (evaluating untrained weights would be silent nonsense)."""
        path = checkpoint or self.checkpoint_path
        if not os.path.exists(path):
            raise FileNotFoundError("no checkpoint to test: %s (train first, or pass checkpoint=)" % path)
        sd = torch.load(path, map_location="cpu", weights_only=True)
        tr = self._setup()
        if sd.get("params_only") or (int(sd.get("world", 1)), int(sd.get("rank", 0))) != (self.world, self.rank):
            tr.load_params_state_dict(sd)
        else:
            tr.load_state_dict(sd)
        n = episodes or self.validation_episodes or 100
        res = self.trainer.evaluate(episodes=n)
        self._log(dict(step=self.trainer.total_steps, **res))
        return res


def _synthetic_oriented(grid, frame, goal, seed=0, aux=True):
    """A random oriented grid whose frames (and depth / segmentation) are fixed random
    images per (cell, rotation): the stand-in for a pickled THOR scene."""
    rng = np.random.default_rng(seed)
    maze = rng.random(grid) >= 0.25
    maze[goal[0], goal[1]] = True
    from scipy.ndimage import label
    lab, _ = label(maze)
    maze = lab == lab[goal[0], goal[1]]
    X, Y = grid
    h, w = frame
    obs = rng.integers(0, 256, size=(X, Y, 4, h, w, 3), dtype=np.uint8)
    kw = {}
    if aux:
        kw = dict(depths=rng.integers(0, 256, size=(X, Y, 4, h, w, 1), dtype=np.uint8),
                  segmentations=rng.integers(0, 256, size=(X, Y, 4, h, w, 3), dtype=np.uint8))
    return oriented_scene(maze, obs, goals=[tuple(goal)], name="synthetic-oriented-%dx%d" % (h, w), **kw)


@register_trainer("thor-cached-auxiliary", max_time_steps=2e6, validation_period=None, validation_episodes=None,
                  episode_log_interval=10, saving_period=100000, save=True)
class ThorCachedAuxiliary(Experiment):
    """experiments/thor_cached_auxiliary.py: AuxiliaryGraph-v0 on thor-cached-212-174 with the
    fixed goal (10, 14, 0), 4 envs, hardness 0.01, LSTM policy + deconv heads with
    auxiliary_weight 0.1 (:42), frames 174x174 (screen_size is not forwarded).
    env_kwargs: scene (a ThorGridWorld pickle path) or grid / frame / goal of the synthetic
    stand-in. The UNREAL losses run with the weights of :39-41 (rp 1.0, pc 0.05, vr 1.0) on
    sequences of a stored rollout, as deep_rl's UnrealTrainer samples them from its replay buffer
    (absent: the buffer's capacity, sequence shape and initial states are parity unpinned)."""

    num_processes = 4
    auxiliary_weight = 0.1
    hardness = 0.01
    # The trainer is deep_rl's UnrealTrainer (absent); its entropy cost is inferred from the
    # logged curve, parity unpinned: outputs/output.txt ends at entropy 0.0014, which the replay
    # of this run reproduces with 0.001 (0.0013 at 1M steps, episode length at the optimum)
    # and not with A2C's 0.01 (0.27-0.36: with reward 1 only at the goal and gamma 0.99 an
    # extra step costs ~0.01 of return, the same order as the 0.01 entropy bonus, so the
    # policy settles stochastic). profiles/r03/entropy/, DESIGN.md "End-to-end check".
    entropy_coefficient = 0.001
    # AuxiliaryTrainer computes the deconv loss on self.replay.sample_sequence()
    # (experiments/ai2_auxiliary/trainer.py:27-31), not on the on-policy batch: the aux batch
    # is a stored rollout drawn from the last replay_size rollouts. deep_rl's replay buffer
    # (its capacity and sequence shape) is absent, so the sequence shape is parity unpinned.
    aux_source = "replay"
    unreal = True
    # UnrealTrainer draws the pixel-control / value-replay / reward-prediction sequences from
    # its replay buffer too: the first 16 envs of the stored rollout drawn for the aux batch
    unreal_source = "replay"
    # the replay ring is pushed and drawn on the device (vn_replay_push_draw), so the update of
    # this 4-env batch is one captured hipGraph (bit-identical to eager, tests/test_replay_gpu.py;
    # single process only unless capture_collectives)
    cuda_graph = True

    def create_env(self, kwargs):
        goal = tuple(kwargs.get("goal", (10, 14, 0)))
        if kwargs.get("scene"):
            scene = load_graph_pickle(kwargs["scene"], goals=[goal], auxiliary=True)
        else:
            scene = _synthetic_oriented(tuple(kwargs.get("grid", (16, 16))), tuple(kwargs.get("frame", (174, 174))),
                                        goal, seed=kwargs.get("scene_seed", 0))
        return VectorEnv([scene], kwargs.get("num_envs", self.num_processes),
                         seed=vdist.rank_seed(self.seed + 1, self.rank), device=self.device, max_episode_steps=900)


@register_trainer("cached-thor", max_time_steps=1e9, validation_period=None, validation_episodes=None,
                  episode_log_interval=1000, saving_period=int(5e7), save=True)
class CachedThor(Experiment):
    """CachedThor-v0 (environments/gym_ai2thor/envs/cached.py) at the north-star shape: h5 /
    npz scene caches (env_kwargs scenes=[paths]) or synthetic 24x24 scenes (n_scenes), 84x84
    frames, num_envs envs per GPU (4096), the LSTM policy without deconv heads."""

    num_processes = 4096

    def create_env(self, kwargs):
        paths = kwargs.get("scenes") or []
        if paths:
            scenes = [load_h5(p) if p.endswith((".h5", ".hdf5")) else load_npz(p) for p in paths]
        else:
            scenes = [synthetic_scene(k) for k in range(int(kwargs.get("n_scenes", 20)))]
        return VectorEnv(scenes, kwargs.get("num_envs", self.num_processes),
                         seed=vdist.rank_seed(self.seed + 1, self.rank), device=self.device, max_episode_steps=900)


def main(argv=None):
    p = argparse.ArgumentParser(description="train.py / test-train.py over vnav")
    p.add_argument("name", help="experiment name (%s)" % ", ".join(registered()))
    p.add_argument("--test", action="store_true", help="test-train.py: evaluate the saved policy")
    p.add_argument("--scene", action="append", default=[], help="scene file(s): .pkl (ThorGridWorld), .h5 or .npz")
    p.add_argument("--envs", type=int, default=None, help="envs per GPU (default: the experiment's num_processes)")
    p.add_argument("--max-time-steps", type=float, default=None)
    p.add_argument("--save-dir", default=None)
    p.add_argument("--episodes", type=int, default=None, help="--test: episodes to run")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--cuda-graph", action="store_true", help="replay each update as a captured hipGraph (1 GPU)")
    p.add_argument("--resume", action="store_true", help="continue from the checkpoint in --save-dir")
    a = p.parse_args(argv)
    vdist.init_distributed()
    env_kwargs = {}
    if a.envs:
        env_kwargs["num_envs"] = a.envs
    if a.scene:
        if a.name == "thor-cached-auxiliary":
            env_kwargs["scene"] = a.scene[0]
        else:
            env_kwargs["scenes"] = a.scene
    over = {}
    if a.max_time_steps is not None:
        over["max_time_steps"] = a.max_time_steps
    if a.cuda_graph:
        over["cuda_graph"] = True
    exp = make_trainer(a.name, env_kwargs=env_kwargs, save_dir=a.save_dir, seed=a.seed, **over)
    if a.test:
        exp.test(episodes=a.episodes)
    else:
        exp.run(resume=a.resume)
    if vdist.world_of()[0] > 1:
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
