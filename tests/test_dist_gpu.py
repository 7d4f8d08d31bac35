"""The multi-GPU update math on the HIP path: the trainer's RCCL all-reduce is a
SUM of the flat gradient with the 1/world scale folded into vn_grad_norm and
vn_rmsprop_step_dev (vnav/a2c.py update, vnav/dist.py). Two checks:

* single process: two half-batch gradients summed, then norm + RMSprop with scale 0.5,
  equal the update over the concatenated batch (params and square_avg);
* world 2 (gloo, both ranks on cuda:0 — the box has one GPU; RCCL refuses two ranks on
  one device): A2CTrainer.update() on identical rollouts on both ranks gives exactly the
  single-process update, the two-bucket all-reduce (heads + LSTM + aux heads issued after
  the LSTM backward, overlapped with the trunk backward) equals the one-bucket update
  bitwise, and per-rank checkpoints restore each rank's own shard.
"""
import ctypes
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _norm_rmsprop(lib, _lib, params, grads, sq, scale, lr_dev):
    st = _lib.stream_ptr(params.device)
    part = torch.zeros(512, dtype=torch.float64, device=params.device)
    sc = torch.zeros(2, device=params.device)
    _lib.check(lib.vn_grad_norm(_lib.ptr(grads), grads.numel(), ctypes.c_float(scale), ctypes.c_float(0.5),
                                _lib.ptr(part), _lib.ptr(sc), st), "vn_grad_norm")
    _lib.check(lib.vn_rmsprop_step_dev(_lib.ptr(params), _lib.ptr(grads), _lib.ptr(sq), params.numel(),
                                       ctypes.c_float(scale), _lib.ptr(sc), _lib.ptr(lr_dev), ctypes.c_float(0.99),
                                       ctypes.c_float(1e-5), st), "vn_rmsprop_step_dev")
    return sc


def test_half_batch_sum_with_scale_equals_full_batch_update():
    import vnav
    from vnav import _lib
    from vnav.policy import PolicyNet, frames_from_batch
    from test_prod_oracle_gpu import _loss_grad
    lib = _lib.load()
    net = PolicyNet((84, 84), 4)
    p0 = net.init_params(1)
    n = 512
    g = torch.Generator(device="cuda").manual_seed(3)
    img = torch.randint(0, 256, (n, 84, 84, 3), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (n, 84, 84, 3), dtype=torch.uint8, device="cuda", generator=g)
    actions = torch.randint(0, 4, (n,), dtype=torch.int32, device="cuda", generator=g)
    rets = torch.randn(n, device="cuda", generator=g)

    def grad(lo, hi):
        m = hi - lo
        acts = net.new_acts(m)
        out = torch.zeros((m, 8), device="cuda")
        fr = frames_from_batch(img[lo:hi], gl[lo:hi])
        net.forward(p0, fr, m, acts, m, 0, out)
        dout = _loss_grad(out, actions[lo:hi].contiguous(), rets[lo:hi].contiguous())
        gr = torch.zeros_like(p0)
        net.backward(p0, fr, m, acts, m, dout, gr, torch.empty(net.workspace_floats(m), device="cuda"))
        return gr

    lr = torch.full((1,), 7e-4, device="cuda")
    sq_init = torch.rand(p0.shape, device="cuda", generator=g) * 1e-6  # a carried square_avg
    full = grad(0, n)
    pa, sa = p0.clone(), sq_init.clone()
    na = _norm_rmsprop(lib, _lib, pa, full, sa, 1.0, lr)
    summed = grad(0, n // 2) + grad(n // 2, n)     # the all-reduce (SUM) of two ranks' gradients
    pb, sb = p0.clone(), sq_init.clone()
    nb = _norm_rmsprop(lib, _lib, pb, summed, sb, 0.5, lr)
    torch.cuda.synchronize()
    assert abs(float(na[0]) - float(nb[0])) <= 1e-5 * float(na[0])
    assert float((sa - sb).abs().max() / sa.abs().max()) <= 1e-5
    step_a, step_b = pa - p0, pb - p0
    assert float((step_a - step_b).abs().max() / step_a.abs().max()) <= 1e-4


def _worker(rank, world, port, tmp, q):
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    try:
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import vnav
        from vnav import dist as vdist
        solo = dist.new_group([0])
        res = {}
        sc = [vnav.synthetic_scene(k) for k in range(2)]
        orig_seed = vdist.rank_seed

        # (1) identical rollouts on both ranks (same env seed, sampling seed of rank 0)
        vdist.rank_seed = lambda seed, r: orig_seed(seed, 0)

        def make(group, env_seed=4, recurrent=True, buckets=2, aux=0.0):
            scn = aux_sc if aux else sc
            env = vnav.VectorEnv(scn, 16, seed=env_seed, max_episode_steps=10)
            return vnav.A2CTrainer(env, num_steps=5, seed=2, max_time_steps=0, process_group=group,
                                   recurrent=recurrent, allreduce_buckets=buckets, time_collectives=True,
                                   aux_weight=aux)
        from bench import aux_scenes
        aux_sc = aux_scenes(2, (84, 84, 3))
        a = make(None)                       # two buckets: heads + LSTM overlapped with the trunk backward
        a1 = make(None, buckets=1)           # one flat bucket after the whole backward
        ax = make(None, aux=0.1)             # + the aux heads in the first bucket
        ax1 = make(None, aux=0.1, buckets=1)
        b = make(solo) if rank == 0 else None
        for _ in range(3):
            for t in (a, a1, ax, ax1):
                t.step(sync=True)
            if b is not None:
                b.step(sync=True)
        res["buckets_equal"] = bool(torch.equal(a.params, a1.params) and torch.equal(a.square_avg, a1.square_avg))
        res["buckets_equal_aux"] = bool(torch.equal(ax.params, ax1.params))
        res["split"] = (a._buckets_split(), a1._buckets_split())
        res["collective_ms"] = a.collective_ms()
        if rank == 0:
            res["world"] = a.world
            res["same_params"] = bool(torch.equal(a.params, b.params))
            res["same_sq"] = bool(torch.equal(a.square_avg, b.square_avg))
        vdist.rank_seed = orig_seed

        # (2) per-rank shards (different env seeds and sampling streams): a checkpoint of each
        # rank restores that rank exactly; another rank's checkpoint is refused
        c = make(None, env_seed=vdist.rank_seed(9, rank))
        for _ in range(2):
            c.step(sync=True)
        path = os.path.join(tmp, "ckpt.rank%d.pt" % rank)
        torch.save(c.state_dict(), path)
        for _ in range(2):
            c.step(sync=True)
        dist.barrier()
        d = make(None, env_seed=vdist.rank_seed(9, rank))
        d.load_state_dict(torch.load(path, weights_only=True))
        for _ in range(2):
            d.step(sync=True)
        res["resume_exact"] = bool(torch.equal(c.params, d.params) and torch.equal(c.square_avg, d.square_avg)
                                   and torch.equal(c.env.get_state(), d.env.get_state()))
        other = torch.load(os.path.join(tmp, "ckpt.rank%d.pt" % (1 - rank)), weights_only=True)
        try:
            d.load_state_dict(other)
            res["refused_other"] = False
        except ValueError:
            res["refused_other"] = True
        res["shards_differ"] = not torch.equal(torch.load(path, weights_only=True)["env_state"],
                                               other["env_state"])
        q.put((rank, res))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, {"error": "%s\n%s" % (e, traceback.format_exc())}))


def test_world2_trainer_update_and_per_rank_checkpoints(tmp_path):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=240) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert "error" not in res[r], res[r]["error"]
        assert res[r]["resume_exact"] and res[r]["refused_other"] and res[r]["shards_differ"], res[r]
        # the bucketed all-reduce (heads + LSTM first, overlapped with the trunk backward)
        # equals the single flat bucket bitwise, with and without the aux heads
        assert res[r]["split"] == (True, False), res[r]
        assert res[r]["buckets_equal"] and res[r]["buckets_equal_aux"], res[r]
        assert res[r]["collective_ms"] is not None and res[r]["collective_ms"] >= 0.0
    assert res[0]["world"] == 2
    assert res[0]["same_params"] and res[0]["same_sq"], res[0]


def test_bench_world2_line_carries_dist_record(tmp_path):
    """bench.py at world 2 as the driver launches it (torch.distributed.run, one rank per
    process), here with gloo and both ranks on the box's one GPU, short legs: rank 0's JSON line
    carries the dist record (world, ranks seen) and per training leg the all-reduce bytes,
    buckets and the exposed collective time; the run exits 0 (bench.py exits non-zero when a
    rank is missing, or under RCCL when two ranks share a device)."""
    import json
    import subprocess
    port = _free_port()
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "20",
           "--warmup", "5", "--envs", "64", "--scenes", "2", "--train-steps", "2", "--train-warmup", "1",
           "--no-train-ref", "--no-c5", "--dist-backend", "gloo", "--allreduce-buckets", "2"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-4000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0
    d = line["dist"]
    assert d["world"] == 2 and d["ranks_seen"] == 2 and d["backend"] == "gloo", d
    for leg in ("train", "train_feedforward"):
        ld = line[leg]["dist"]
        assert ld["world"] == 2 and ld["allreduce_bytes"] > 0, ld
        assert ld["allreduce_exposed_ms_per_update"] is not None and ld["allreduce_exposed_ms_per_update"] >= 0, ld
        assert sum(b for b, _ in ld["buckets"]) == ld["allreduce_bytes"], ld
    assert len(line["train"]["dist"]["buckets"]) == 2           # LSTM: heads + LSTM bucket, trunk bucket
    assert len(line["train_feedforward"]["dist"]["buckets"]) == 1
