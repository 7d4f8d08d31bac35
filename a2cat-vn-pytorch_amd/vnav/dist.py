"""Data parallelism: one process per GPU, torch.distributed over RCCL ("nccl" on ROCm).

Envs are independent, so each rank owns its own env shard and a full replica of the
scene cache; the only data-path exchange is the all-reduce of the flat
fp32 gradient buffer per update (0.96 MB for the 84x84 feed-forward policy; 9.4-19.8 MB
with the LSTM / aux / UNREAL heads), one flat bucket by default (A2CTrainer
allreduce_buckets=1). allreduce_buckets=2 is opt-in: heads + LSTM + aux heads as soon as the
LSTM backward ends, overlapped with the trunk backward, then the trunk — bitwise equal to
one bucket in the gloo world-2 test, not yet run under RCCL across distinct GPUs. Plus one
tiny all-reduce of the episode/loss statistics.
The reference has no distributed code at all (it runs 4 SubprocVecEnv processes on
one GPU, experiments/thor_cached_auxiliary.py:58-71).
"""
import os

import torch
import torch.distributed as dist


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_distributed(backend=None):
    """Initialise from torchrun's environment. Returns (rank, world, local_rank)."""
    rank, world, local = env_rank()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return rank, world, local


def world_of(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def capturable(group=None):
    """Whether the group's collectives can be captured in a hipGraph (RCCL can, gloo not)."""
    world, _ = world_of(group)
    return world == 1 or dist.get_backend(group) == "nccl"


def allreduce_gradients_(flat, group=None):
    """SUM-all-reduce the flat gradient in place; returns the 1/world scale the update
    kernels fold into the gradient norm and the RMSprop step (no extra pass)."""
    world, _ = world_of(group)
    if world > 1:
        dist.all_reduce(flat, group=group)
    return 1.0 / world


def allreduce_async_(flat, group=None):
    """Start a SUM all-reduce of ``flat`` in place and return its work handle (None at world
    1). With RCCL the collective runs on the communicator's own stream once the current
    stream reaches this point, so later kernels on the current stream overlap it; ``wait()``
    makes the current stream wait for it."""
    world, _ = world_of(group)
    if world == 1:
        return None
    return dist.all_reduce(flat, group=group, async_op=True)


def reduce_metrics_(m, n_mean, group=None):
    """m = [mean stats (n_mean entries) | summed counters]: average the first n_mean
    entries over ranks and sum the rest."""
    world, _ = world_of(group)
    if world > 1:
        dist.all_reduce(m, group=group)
        m[:n_mean] /= world
    return m


def broadcast_params_(flat, src=0, group=None):
    """Broadcast from the group's rank `src` (a rank WITHIN `group`, translated to the global
    rank torch.distributed.broadcast expects, so subgroups without global rank 0 work)."""
    world, _ = world_of(group)
    if world > 1:
        gsrc = src if group is None else dist.get_global_rank(group, src)
        dist.broadcast(flat, src=gsrc, group=group)
    return flat


def check_ranks_agree(values, what, group=None):
    """Raise on every rank unless all ranks hold the same integer ``values`` (an all-reduce
    of [v, -v] with MAX gives max and -min in one call)."""
    world, rank = world_of(group)
    if world == 1:
        return
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    v = torch.tensor([float(x) for x in values], dtype=torch.float64, device=dev)
    t = torch.cat([v, -v])
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    n = len(values)
    hi, lo = t[:n].cpu(), -t[n:].cpu()
    if not torch.equal(hi, lo):
        raise RuntimeError("ranks disagree on %s: min %s, max %s (rank %d has %s)"
                           % (what, lo.tolist(), hi.tolist(), rank, list(values)))


def rank_seed(seed, rank):
    """Distinct, reproducible per-rank seeds for env resets and policy sampling."""
    return (int(seed) * 1000003 + int(rank) * 7919 + 1) & (2**63 - 1)


def shard(n_total, world, rank):
    """Contiguous env shard [start, start+count) of rank (envs e -> GPU e // per)."""
    per, extra = divmod(int(n_total), int(world))
    start = rank * per + min(rank, extra)
    return start, per + (1 if rank < extra else 0)
