"""The experiment surface (vnav.train): register_trainer / make_trainer / run / test and the
train.py / test-train.py command line (reference train.py:10-25, test-train.py:11-26,
experiments/thor_cached_auxiliary.py:26-84)."""
import os

import numpy as np
import pytest
import torch


def _train():
    from vnav import train
    return train


def test_registry_and_hyperparameters():
    train = _train()
    assert {"thor-cached-auxiliary", "cached-thor"} <= set(train.registered())
    cls = train._TRAINERS["thor-cached-auxiliary"]
    # experiments/thor_cached_auxiliary.py:26-42
    assert (cls.max_time_steps, cls.episode_log_interval, cls.saving_period, cls.save) == (2e6, 10, 100000, True)
    assert (cls.num_processes, cls.num_steps, cls.gamma, cls.learning_rate) == (4, 20, 0.99, 7e-4)
    assert (cls.rms_alpha, cls.rms_epsilon, cls.max_gradient_norm) == (0.99, 1e-5, 0.5)
    assert (cls.value_coefficient, cls.entropy_coefficient) == (0.5, 0.001)
    assert (cls.auxiliary_weight, cls.hardness, cls.recurrent) == (0.1, 0.01, True)
    assert (cls.unreal, cls.rp_weight, cls.pc_weight, cls.vr_weight) == (True, 1.0, 0.05, 1.0)  # :39-41
    # replayed aux / UNREAL batches with the ring on the device: the update is a captured hipGraph
    assert (cls.aux_source, cls.unreal_source, cls.cuda_graph) == ("replay", "replay", True)
    with pytest.raises(KeyError):
        train.make_trainer("no-such-experiment")
    with pytest.raises(TypeError):
        train.make_trainer("cached-thor", not_an_attribute=1)


def test_metric_table_format():
    t = _train()._format_table({"step": 2240, "reward": 0.9, "episodes": 10, "fps": 32})
    lines = t.split("\n")
    assert lines[0].startswith("---") and lines[-1].startswith("---")
    assert lines[1].startswith("| step") and "2240" in lines[1]
    assert len({len(x) for x in lines}) == 1


@pytest.mark.gpu
def test_run_saves_and_test_reloads(tmp_path):
    """run() trains to max_time_steps with periodic + final checkpoints, test() reloads the
    saved policy into a fresh experiment and runs evaluation episodes."""
    train = _train()
    logs = []
    kw = dict(env_kwargs=dict(grid=(6, 6), frame=(84, 84), goal=(3, 3, 0), num_envs=8), save_dir=str(tmp_path),
              max_time_steps=8 * 20 * 3, saving_period=160, episode_log_interval=1, logger=logs.append)
    exp = train.make_trainer("thor-cached-auxiliary", **kw)
    m = exp.run()
    assert m["step"] == 480 and m["updates"] == 3 and np.isfinite(m["loss"])
    assert os.path.exists(exp.checkpoint_path)
    sd = torch.load(exp.checkpoint_path, weights_only=True)
    assert torch.equal(sd["params"], exp.trainer.params.cpu()) and sd["total_steps"] == 480
    tables = [x for x in logs if x.startswith("---")]
    saves = [x for x in logs if x.startswith("Saving")]
    assert tables and len(saves) >= 3 and len(tables) + len(saves) == len(logs)
    ev = train.make_trainer("thor-cached-auxiliary", **kw)
    res = ev.test(episodes=5)
    assert torch.equal(ev.trainer.params.cpu(), sd["params"])
    assert res["episodes"] >= 5 and 0.0 < res["reward"] <= 1.0 and res["episode_length"] >= 1
    # evaluation does not advance the learning-rate schedule
    assert int(ev.trainer.sched[1]) == 480
    rows = [l for l in open(os.path.join(str(tmp_path), "metrics.jsonl"))]
    assert len(rows) == len(tables) + 1  # + the test() row


@pytest.mark.gpu
def test_resume_continues_exactly(tmp_path):
    """run(resume=True) from a checkpoint reaches the same parameters as an uninterrupted
    run of the same length (deep_rl saving_period checkpoints)."""
    train = _train()
    kw = dict(env_kwargs=dict(grid=(6, 6), frame=(84, 84), goal=(3, 3, 0), num_envs=8), saving_period=0,
              episode_log_interval=0, logger=None)
    full = train.make_trainer("thor-cached-auxiliary", save_dir=str(tmp_path / "a"), max_time_steps=640, **kw)
    full.run()
    # the same experiment interrupted after two updates (the LinearSchedule horizon is
    # max_time_steps, so the interrupted run keeps it), checkpointed, then resumed
    part = train.make_trainer("thor-cached-auxiliary", save_dir=str(tmp_path / "b"), max_time_steps=640, **kw)
    tr = part._setup()
    tr.step()
    tr.step()
    part.save_checkpoint()
    rest = train.make_trainer("thor-cached-auxiliary", save_dir=str(tmp_path / "b"), max_time_steps=640, **kw)
    rest.run(resume=True)
    assert rest.trainer.total_steps == 640
    assert torch.equal(rest.trainer.params, full.trainer.params)


def test_checkpoint_paths_per_rank(tmp_path, monkeypatch):
    """checkpoint.pt is the single-process state (world 1) or the world-agnostic policy
    state (world > 1); the per-rank files (env shard, running returns, recurrent carry) sit
    in the generation directory of the last complete set (tests/test_dist_cpu.py covers the
    protocol at world 2)."""
    train = _train()
    exp = train.make_trainer("cached-thor", save_dir=str(tmp_path))
    assert exp.checkpoint_path == os.path.join(str(tmp_path), "checkpoint.pt")
    assert not exp.has_checkpoint()
    for r in range(2):
        monkeypatch.setenv("RANK", str(r))
        monkeypatch.setenv("WORLD_SIZE", "2")
        monkeypatch.setenv("LOCAL_RANK", str(r))
        exp = train.make_trainer("cached-thor", save_dir=str(tmp_path))
        assert exp.checkpoint_path == os.path.join(str(tmp_path), "checkpoint.pt")
        assert exp.rank_checkpoint_path() is None
        assert exp.rank_checkpoint_path(4800) == os.path.join(str(tmp_path), "ckpt-%012d" % 4800, "rank%d.pt" % r)


def test_test_without_checkpoint_raises(tmp_path):
    """test() refuses to evaluate when there is no checkpoint (no silent random policy)."""
    train = _train()
    exp = train.make_trainer("cached-thor", save_dir=str(tmp_path))
    with pytest.raises(FileNotFoundError):
        exp.test(episodes=1)
