"""Multi-process data parallelism on the CPU (gloo, world_size 2): the product's DP
helpers (vnav/dist.py) average gradients so that the per-rank A2C gradients of two env
shards equal the single-process gradient over the concatenated batch (computed with the
CPU oracle model), and reduce the metrics as the trainer expects."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import sys
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from oracle import a2c
    from oracle.policy import GoalNetOracle
    from vnav import dist as vdist
    r, w, _ = vdist.init_distributed(backend="gloo")
    assert (r, w) == (rank, world)
    torch.manual_seed(0)
    net = GoalNetOracle((84, 84))
    g = torch.Generator().manual_seed(1)
    N = 8
    img = torch.rand(N, 3, 84, 84, generator=g)
    goal = torch.rand(N, 3, 84, 84, generator=g)
    acts = torch.randint(0, 4, (N,), generator=g)
    rets = torch.randn(N, generator=g)
    start, count = vdist.shard(N, world, rank)
    sl = slice(start, start + count)
    lg, v = net(img[sl], goal[sl])
    loss, parts = a2c.loss(lg, v.view(-1), acts[sl], rets[sl])
    loss.backward()
    flat = torch.cat([p.grad.reshape(-1) for p in net.parameters()])
    scale = vdist.allreduce_gradients_(flat)
    m = torch.tensor([parts["value_loss"].item(), 0.0, 0.0, 0.0, 1.0, float(count), 2.0, 3.0])
    vdist.reduce_metrics_(m, 5)
    seeds = [vdist.rank_seed(5, rr) for rr in range(world)]
    q.put((rank, (flat * scale).numpy(), m.numpy(), len(set(seeds))))
    dist.destroy_process_group()


def test_gloo_world2_gradient_average_equals_full_batch():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    g0, g1 = res[0][1], res[1][1]
    np.testing.assert_array_equal(g0, g1)  # every rank holds the same averaged gradient
    # single process, concatenated batch
    from oracle import a2c
    from oracle.policy import GoalNetOracle
    torch.manual_seed(0)
    net = GoalNetOracle((84, 84))
    g = torch.Generator().manual_seed(1)
    N = 8
    img = torch.rand(N, 3, 84, 84, generator=g)
    goal = torch.rand(N, 3, 84, 84, generator=g)
    acts = torch.randint(0, 4, (N,), generator=g)
    rets = torch.randn(N, generator=g)
    lg, v = net(img, goal)
    loss, _ = a2c.loss(lg, v.view(-1), acts, rets)
    loss.backward()
    full = torch.cat([p.grad.reshape(-1) for p in net.parameters()]).numpy()
    np.testing.assert_allclose(g0, full, rtol=1e-4, atol=1e-7)
    m = res[0][2]
    assert m[4] == 1.0 and m[5] == 8.0 and m[6] == 4.0  # means averaged, counters summed
    assert res[0][3] == world


def test_shard_covers_all_envs():
    from vnav.dist import shard
    for n, w in ((32768, 8), (10, 3), (4096, 1)):
        spans = [shard(n, w, r) for r in range(w)]
        assert spans[0][0] == 0 and sum(c for _, c in spans) == n
        for (s0, c0), (s1, _) in zip(spans, spans[1:]):
            assert s0 + c0 == s1


def _bcast_worker(rank, world, port, q):
    import sys
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from vnav import dist as vdist
    vdist.init_distributed(backend="gloo")
    sub = dist.new_group([1, 2])  # a subgroup without global rank 0: every rank must call new_group
    flat = torch.full((16,), float(rank))
    if rank in (1, 2):
        vdist.broadcast_params_(flat, group=sub)  # src = the subgroup's rank 0 = global rank 1
        trainer_world = vdist.world_of(sub)
    else:
        trainer_world = None
    q.put((rank, flat.numpy(), trainer_world))
    dist.destroy_process_group()


def test_gloo_subgroup_broadcast_uses_group_rank():
    """broadcast_params_(group=g) sends from g's first member, not from global rank 0."""
    world = 3
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bcast_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.all(res[0][1] == 0.0)            # rank 0 is not in the group: untouched
    assert np.all(res[1][1] == 1.0) and np.all(res[2][1] == 1.0)
    assert res[1][2] == (2, 0) and res[2][2] == (2, 1)


class _StubTrainer:
    """The parts of A2CTrainer the checkpoint protocol uses (CPU tensors, no GPU)."""

    def __init__(self, rank, world):
        self.rank, self.world = rank, world
        self.params = torch.zeros(6)
        self.square_avg = torch.zeros(6)
        self.env_state = torch.zeros(3)
        self.num_updates = self.total_steps = 0

    def advance(self, n, rank_value):
        self.num_updates += n
        self.total_steps += 10 * n
        self.params.fill_(float(self.num_updates))
        self.square_avg.fill_(2.0 * self.num_updates)
        self.env_state.fill_(rank_value)

    def state_dict(self):
        return {"params": self.params.clone(), "square_avg": self.square_avg.clone(), "env": self.env_state.clone(),
                "num_updates": self.num_updates, "total_steps": self.total_steps, "rank": self.rank,
                "world": self.world}

    def params_state_dict(self):
        return {"params": self.params.clone(), "square_avg": self.square_avg.clone(), "num_updates": self.num_updates,
                "total_steps": self.total_steps, "world": self.world, "params_only": True}

    def load_state_dict(self, sd):
        self.params.copy_(sd["params"])
        self.square_avg.copy_(sd["square_avg"])
        self.env_state.copy_(sd["env"])
        self.num_updates, self.total_steps = int(sd["num_updates"]), int(sd["total_steps"])


def _ckpt_worker(rank, world, port, save_dir, q):
    import sys
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import json
    import torch.distributed as dist
    from vnav import dist as vdist
    from vnav import train
    vdist.init_distributed(backend="gloo")
    out = {}
    exp = train.make_trainer("cached-thor", save_dir=save_dir, device="cpu", logger=None)
    exp.trainer = _StubTrainer(rank, world)
    exp.trainer.advance(10, 100 + rank)
    exp.save_checkpoint()                                    # set at step 100
    exp.trainer.advance(10, 200 + rank)
    exp.save_checkpoint()                                    # set at step 200 (replaces 100)
    out["gens"] = sorted(d for d in os.listdir(save_dir) if d.startswith("ckpt-"))
    out["latest"] = json.load(open(os.path.join(save_dir, "latest.json")))
    # a crash after rank 0 (only) wrote the next generation: latest.json still names step 200
    exp.trainer.advance(10, 300 + rank)
    if rank == 0:
        exp._atomic_save(exp.trainer.state_dict(), exp.rank_checkpoint_path(exp.trainer.total_steps))
    dist.barrier()
    fresh = train.make_trainer("cached-thor", save_dir=save_dir, device="cpu", logger=None)
    fresh.trainer = _StubTrainer(rank, world)
    fresh.load_checkpoint()
    out["resumed"] = (fresh.trainer.num_updates, fresh.trainer.total_steps, float(fresh.trainer.env_state[0]),
                      float(fresh.trainer.params[0]))
    # rank 1's file of the complete set disagrees (a hand-edited / foreign file): every rank refuses
    dist.barrier()
    if rank == 1:
        p = fresh.rank_checkpoint_path()
        sd = torch.load(p, weights_only=True)
        sd["num_updates"] += 1
        sd["params"].fill_(-1.0)
        torch.save(sd, p)
    dist.barrier()
    bad = train.make_trainer("cached-thor", save_dir=save_dir, device="cpu", logger=None)
    bad.trainer = _StubTrainer(rank, world)
    try:
        bad.load_checkpoint()
        out["mismatch"] = "loaded"
    except RuntimeError as e:
        out["mismatch"] = "refused" if "disagree" in str(e) else str(e)
    # run(resume=True)'s decision is collective: agreed while both files exist, refused on
    # every rank once rank 1's file of the set is gone (instead of a hang in the collectives)
    out["resume_agreed"] = bad._resume_decision()
    dist.barrier()
    if rank == 1:
        os.remove(bad.rank_checkpoint_path())
    dist.barrier()
    try:
        bad._resume_decision()
        out["resume_split"] = "decided"
    except RuntimeError as e:
        out["resume_split"] = "refused" if "disagree" in str(e) else str(e)
    q.put((rank, out))
    dist.destroy_process_group()


def test_gloo_world2_checkpoint_sets_are_complete_and_consistent(tmp_path):
    """world > 1 checkpoints (vnav/train.py): per-rank files in a generation directory
    committed by rank 0's latest.json after a barrier, a world-agnostic checkpoint.pt for a
    single-process test(), resume from the last complete set after a partial save, and a
    refusal on every rank when the ranks' counters disagree."""
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ckpt_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        o = res[r]
        assert o["latest"] == {"total_steps": 200, "num_updates": 20, "world": 2}
        assert o["resumed"] == (20, 200, 200.0 + r, 20.0)   # own env state, rank 0's params
        assert o["mismatch"] == "refused"
        assert o["resume_agreed"] is True and o["resume_split"] == "refused"
    assert res[0]["gens"] == ["ckpt-%012d" % 200]
    sd = torch.load(os.path.join(str(tmp_path), "checkpoint.pt"), weights_only=True)
    assert sd["params_only"] and sd["num_updates"] == 20 and float(sd["params"][0]) == 20.0
