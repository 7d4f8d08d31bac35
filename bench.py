#!/usr/bin/env python3
"""Benchmark: env-steps/sec (whole node) of the batched cached-THOR VectorEnv.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs 4096] [--scenes 20]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One bench step = one batched VectorEnv.step over all local envs: vn_step (transition,
reward/done masking, auto-reset, gather of the image frame and goal frame into the output
batch) on synthetic uniform actions that are generated on the device (vn_random_actions)
before the timed region. Each rank owns
--envs envs and a full replica of the scene cache (weak scaling, no data-path
collective: envs are independent). The timed region is bracketed by
barrier + synchronize; the max over ranks is reported. The vn_step kernel's average
duration comes from HIP events around each launch on the launch stream.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "a2cat-vn-pytorch_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
FP32_MFMA_PEAK_TFLOPS = 157.3  # dense f32 MFMA = f32 vector peak (MI355X_MICROARCH.md)
# the reference's only throughput record: deep_rl fps of thor-cached-auxiliary (174x174, LSTM +
# aux deconv, 4 envs, 1 GPU), steady-state median, BASELINE.md §2 / outputs/output.txt
REFERENCE_LOG_FPS = 106.0
# auxiliary_weight of the logged experiment (experiments/thor_cached_auxiliary.py:42; 0.05 is only
# AuxiliaryTrainer's default, experiments/ai2_auxiliary/trainer.py:25)
AUX_WEIGHT_LOGGED = 0.1


def alg_bytes_per_env_step(frame_bytes):
    """read image + goal frame, write both into the batch, + 32 B of state."""
    return 4 * frame_bytes + 32


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--warmup", type=int, default=500)
    p.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    p.add_argument("--scenes", type=int, default=20)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--train-steps", type=int, default=6, help="timed A2C updates (0 = skip the train leg)")
    p.add_argument("--train-warmup", type=int, default=2)
    p.add_argument("--no-train-ff", action="store_true", help="skip the feed-forward (no LSTM) train leg")
    p.add_argument("--no-train-84", action="store_true", help="skip the 84x84 LSTM train leg")
    p.add_argument("--no-train-ref", action="store_true",
                   help="skip the 174x174 LSTM + aux-deconv train leg (the reference's logged experiment shape)")
    p.add_argument("--no-train-ref4", action="store_true",
                   help="skip the 4-env (the logged run's batch) 174x174 leg")
    p.add_argument("--no-train-174", action="store_true",
                   help="skip the 4096-env 174x174 leg only (the 4-env leg still runs)")
    p.add_argument("--no-c5", action="store_true",
                   help="skip the 300x400 + goal + aux-depth train leg (config C5, 512 envs per GPU)")
    p.add_argument("--num-steps", type=int, default=20, help="A2C rollout length (reference: 20)")
    p.add_argument("--no-short", action="store_true",
                   help="skip the 2-step-episode legs (goal-frame deduplication at the logged run's operating point)")
    p.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    p.add_argument("--dist-backend", default="nccl", help="torch.distributed backend (nccl = RCCL on ROCm)")
    p.add_argument("--allreduce-buckets", type=int, choices=(1, 2), default=1,
                   help="gradient all-reduce buckets at world > 1 (2: heads + LSTM overlapped with the trunk backward)")
    p.add_argument("--pmc-leg", choices=sorted(LEGS), default=None,
                   help="(child of the PMC pass) run only this training leg: one warmup update, then exactly one "
                        "update between two vn_trace_marker launches; no env leg, no JSON line")
    p.add_argument("--cpu-sweep", default="1,16,all",
                   help="CPU-baseline process counts (comma list; 'all' = every CPU of this process's affinity)")
    return p.parse_args()


def _pmc_pass(counter, out_dir, envs, scenes):
    """One rocprofv3 --pmc pass (a single counter, no tracing) over a short child bench run;
    returns the median per-dispatch value of `counter` for the vn_step kernel (KB)."""
    import csv
    import glob
    import shutil
    import subprocess
    if shutil.which("rocprofv3") is None:
        return None
    d = os.path.join(out_dir, counter.lower())
    cmd = ["rocprofv3", "--pmc", counter, "--kernel-include-regex", "env_kernel", "--output-format", "csv",
           "-d", d, "-o", "run", "--", sys.executable, os.path.abspath(__file__), "--steps", "10", "--warmup", "2",
           "--no-cpu-baseline", "--train-steps", "0", "--no-pmc", "--envs", str(envs), "--scenes", str(scenes)]
    env = dict(os.environ, TMPDIR="/tmp")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=240)
    if r.returncode != 0:
        return None
    vals = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") == counter and "env_kernel<0" in row.get("Kernel_Name", ""):
                    vals.append(float(row["Counter_Value"]))
    return sorted(vals)[len(vals) // 2] if vals else None


def pmc_traffic(envs, scenes):
    """HBM bytes per vn_step launch from PMC counters, separate passes, gfx950 correction
    (MI355X_MICROARCH.md §HBM): read = 2 x FETCH_SIZE (half-counted for 16-B/lane streaming
    reads), write = WRITE_SIZE; both in KB."""
    import tempfile
    out_dir = tempfile.mkdtemp(prefix="vnav_pmc_", dir="/tmp")
    try:
        f_kb = _pmc_pass("FETCH_SIZE", out_dir, envs, scenes)
        w_kb = _pmc_pass("WRITE_SIZE", out_dir, envs, scenes)
    except Exception:
        return None, None
    if f_kb is None or w_kb is None:
        return None, None
    return (2 * f_kb + w_kb) * 1024, {"fetch_size_kb": f_kb, "write_size_kb": w_kb,
                                       "source": "live rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes"}


def pmc_train_mfma(args, leg):
    """Measured matrix-core utilisation of exactly one training update of ``leg`` (rollout +
    update): a rocprofv3 --pmc pass (SQ_VALU_MFMA_BUSY_CYCLES summed over the SIMDs,
    GRBM_GUI_ACTIVE summed over the 8 XCDs; no tracing) over a child run of this script with
    --pmc-leg, which runs one warmup update and then one update between two vn_trace_marker
    launches. Only the dispatches between the markers are counted. Busy fraction =
    sum(MFMA busy) / (SIMDs x sum(GRBM) / 8). The split-bf16 products issue 3-6 bf16 MFMAs
    per fp32 product, so this is pipe occupancy, not the algorithmic fraction."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    if shutil.which("rocprofv3") is None:
        return None
    d = tempfile.mkdtemp(prefix="vnav_pmc_mfma_%s_" % leg, dir="/tmp")
    cmd = ["rocprofv3", "--pmc", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "--output-format", "csv", "-d", d,
           "-o", "run", "--", sys.executable, os.path.abspath(__file__), "--pmc-leg", leg, "--envs", str(args.envs),
           "--scenes", str(args.scenes), "--num-steps", str(args.num_steps)]
    env = dict(os.environ, TMPDIR="/tmp")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    try:
        r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           timeout=300)
    except Exception:
        return None
    if r.returncode != 0:
        return None
    rows = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                rec = rows.setdefault(int(row["Dispatch_Id"]), {"name": row.get("Kernel_Name", "")})
                rec[row["Counter_Name"]] = rec.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    marks = sorted(i for i, v in rows.items() if "trace_marker" in v["name"])
    shutil.rmtree(d, ignore_errors=True)
    if len(marks) != 2:
        return None
    win = [v for i, v in rows.items() if marks[0] < i < marks[1]]
    mfma = sum(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for v in win)
    grbm = sum(v.get("GRBM_GUI_ACTIVE", 0.0) for v in win)
    if grbm <= 0:
        return None
    return {"mfma_busy_cycles": mfma, "grbm_gui_active": grbm, "dispatches": len(win), "updates": 1,
            "source": "live rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE, the dispatches of exactly one "
                      "%s update (between two vn_trace_marker launches of a --pmc-leg child)" % leg}


def aux_flops_per_sample(o3):
    """Algorithmic FLOPs of the deconv heads per sample (forward + both gradients): first
    layer 32 -> 3x16 over 2x2 taps per output pixel, second layer 16 -> (1, 3, 3) per head."""
    ah, aw = 2 * o3[0] + 2, 2 * o3[1] + 2
    ph, pw = 2 * ah + 2, 2 * aw + 2
    l1 = ah * aw * 48 * 4 * 32                      # MACs, forward (= dX4 = wgrad)
    l2 = ph * pw * 7 * 4 * 16                       # MACs, forward (= dA1 = wgrad)
    return 2 * 3 * (l1 + l2)


BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)
# fp32-equivalent ceilings of the MFMA forms the kernels issue per exact fp32 product
# (DESIGN.md "bf16 MFMA with exact operand splits"): x3 = 3 bf16 MFMAs (u8 frame x split
# weight / split dZ), x6 = 6 (split x split), f32 = the f32 MFMA / VALU rate
CEIL_TFLOPS = {"x3": BF16_MFMA_PEAK_TFLOPS / 3, "x6": BF16_MFMA_PEAK_TFLOPS / 6, "f32": FP32_MFMA_PEAK_TFLOPS}


def train_flops_terms(h=84, w=84, A=4, T=20, recurrent=False, aux=False, goal_fwd=1.0, goal_bwd=1.0, unreal=0.0):
    """FLOPs of one A2C env-step by (part, MFMA form): policy forward (kept activations serve
    the backward), weight gradients of every layer, input gradients of all but conv1, the
    bootstrap forward amortised over the rollout, and the aux deconv heads.
    The form is the one the kernels issue at these geometries (conv1 forward / weight gradient
    on u8 frames: x3; the aux heads' second layer: f32 VALU forward, f32 MFMA backward;
    everything else x6). goal_fwd / goal_bwd: the fraction of the goal frames whose
    shared_base (conv1, conv2) the rollout forward / the update's backward computes — 1 is
    the reference's algorithm (goal.py:88 runs it on every goal frame); with goal-frame
    deduplication the measured fractions give the executed FLOPs. unreal: the fraction S / E of
    the envs whose sequences the UNREAL losses use (pixel control on their T + 1 LSTM rows,
    reward prediction on their T - 2 three-frame samples), amortised per env-step; the pixel
    control's second layer counts its A + 1 live channels."""
    o1 = ((h - 7) // 4 + 1, (w - 7) // 4 + 1)
    o2 = ((o1[0] - 4) // 2 + 1, (o1[1] - 4) // 2 + 1)
    o3 = ((o2[0] - 4) // 2 + 1, (o2[1] - 4) // 2 + 1)
    p1, p2, p3 = o1[0] * o1[1], o2[0] * o2[1], o3[0] * o3[1]
    # FLOPs of conv1, conv2 over a sample's two frames (image and goal); MACs of the rest
    c1, c2 = 2 * 2 * p1 * 32 * 147, 2 * 2 * p2 * 32 * 512
    macs = [p3 * 64 * 1024, p3 * 32 * 64, 512 * 32 * p3, (A + 1) * 512]
    if recurrent:  # LSTM gates GEMM [xcat=512+A+1 padded to 4, +512] x 2048: fwd, dgrad, wgrad
        macs.append(2048 * ((512 + A + 1 + 3) // 4 * 4 + 512))
    fr = 2 * sum(macs)
    ff, fb = (1 + goal_fwd) / 2, (1 + goal_bwd) / 2  # frames computed per 2 frames
    terms = [("forward conv1", "x3", c1 * (ff + 1.0 / T)), ("forward conv2", "x6", c2 * (ff + 1.0 / T)),
             ("forward rest", "x6", fr * (1 + 1.0 / T)),
             ("wgrad conv1", "x3", c1 * fb), ("wgrad conv2", "x6", c2 * fb), ("wgrad rest", "x6", fr),
             ("dgrad conv2", "x6", c2 * fb), ("dgrad rest", "x6", fr)]
    if aux:
        ah, aw = 2 * o3[0] + 2, 2 * o3[1] + 2
        ph, pw = 2 * ah + 2, 2 * aw + 2
        l1 = 2 * ah * aw * 48 * 4 * 32
        l2 = 2 * ph * pw * 7 * 4 * 16
        terms += [("aux layer 1 (fwd, dX4, dW1)", "x6", 3 * l1), ("aux layer 2 forward", "f32", l2),
                  ("aux layer 2 backward", "f32", 2 * l2)]
    if unreal:
        rows, samples = unreal * (T + 1) / T, unreal * (T - 2) / T
        base, d1, d2 = 2 * 512 * 2592, 2 * 20 * 20 * 64 * 4 * 32, 2 * 42 * 42 * (A + 1) * 4 * 32
        rp = 2 * 3 * 3 * 32 * p3
        terms += [("unreal pc forward", "x6", (base + d1) * rows), ("unreal pc layer 2 forward", "f32", d2 * rows),
                  ("unreal pc backward", "x6", 2 * (base + d1 + d2) * rows), ("unreal rp", "f32", 3 * rp * samples)]
    return terms


def train_flops_per_env_step(h=84, w=84, A=4, T=20, recurrent=False, aux=False, goal_fwd=1.0, goal_bwd=1.0,
                             unreal=0.0):
    """(total FLOPs per env-step, forward FLOPs per sample)."""
    terms = train_flops_terms(h, w, A, T, recurrent, aux, goal_fwd, goal_bwd, unreal)
    total = sum(f for _, _, f in terms)
    fwd = sum(f for name, _, f in terms if name.startswith("forward")) / (1 + 1.0 / T)
    return total, fwd


def issued_ceiling_tflops(h=84, w=84, A=4, T=20, recurrent=False, aux=False, goal_fwd=1.0, goal_bwd=1.0, unreal=0.0):
    """The update's fp32-equivalent ceiling when every part runs at the peak of the MFMA form
    it issues: total FLOPs / sum(FLOPs_i / ceiling_i)."""
    terms = train_flops_terms(h, w, A, T, recurrent, aux, goal_fwd, goal_bwd, unreal)
    total = sum(f for _, _, f in terms)
    return total / sum(f / CEIL_TFLOPS[form] for _, form, f in terms)


def aux_scenes(n, frame, seed=0):
    """Synthetic scenes with depth + segmentation frames (AuxiliaryGraph / config C5 data)."""
    import vnav
    out = []
    rng = np.random.default_rng(seed)
    for k in range(n):
        sc = vnav.synthetic_scene(k, frame_shape=frame)
        sc.depth = rng.integers(0, 256, size=(sc.n_states,) + frame[:2] + (1,), dtype=np.uint8)
        sc.segmentation = rng.integers(0, 256, size=(sc.n_states,) + frame[:2] + (3,), dtype=np.uint8)
        sc.__post_init__()
        out.append(sc)
    return out


def bench_train(args, scenes, dev, world, rank, recurrent, aux_weight=0.0, envs=None, updates=None, warmup=None,
                model=None, cuda_graph=False, marker=False, unreal=False, hardness=None, max_episode_steps=900,
                replay_sources=False):
    """A2C training throughput: one step = rollout of num_steps on every local env (policy
    forward + sampling + env step) + backward + one RCCL all-reduce of the flat gradient +
    clip + RMSprop. recurrent: the full BigGoalHouseModel (LSTM core, BPTT over the rollout);
    else the feed-forward trunk + heads. aux_weight > 0 adds the deconv heads + aux loss;
    unreal the pixel-control / reward-prediction / value-replay losses (UnrealTrainer)."""
    import vnav
    E, T = envs or args.envs, args.num_steps
    updates = updates or args.train_steps
    warmup = args.train_warmup if warmup is None else warmup
    env = vnav.VectorEnv(scenes, E, seed=2000 + rank, device=dev, max_episode_steps=max_episode_steps)
    if hardness is not None:  # experiments/thor_cached_auxiliary.py:68-70 (before the first reset)
        env.set_hardness(hardness)
        env.reset()
    tr = vnav.A2CTrainer(env, num_steps=T, seed=7, max_time_steps=1e12, recurrent=recurrent, aux_weight=aux_weight,
                         cuda_graph=cuda_graph, time_collectives=world > 1 and not cuda_graph, unreal=unreal,
                         allreduce_buckets=args.allreduce_buckets,
                         **(dict(aux_source="replay", unreal_source="replay") if replay_sources else {}))
    for _ in range(warmup):
        tr.step(sync=False)
    torch.cuda.synchronize(dev)
    tr.collective_ms()  # drop the warmup updates' collective timings
    if marker:  # the PMC child's window: exactly the timed updates between two marker kernels
        from vnav import _lib
        _lib.check(_lib.load().vn_trace_marker(1, _lib.stream_ptr(dev)), "vn_trace_marker")
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(updates):
        tr.step(sync=False)
    if marker:
        _lib.check(_lib.load().vn_trace_marker(2, _lib.stream_ptr(dev)), "vn_trace_marker")
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    coll_ms = tr.collective_ms() if world > 1 else None
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t[0])
    steps = E * T * updates * world
    h, w = env.frame_shape[:2]
    ax = aux_weight > 0
    # goal frames whose shared_base ran (the last update's goal runs; 1 without deduplication)
    gf = gb = 1.0
    if tr.dedup_goals:
        cnt = tr.goal_count.cpu().tolist()
        gf, gb = sum(cnt[:T]) / (E * T), cnt[T] / (E * T)
    un = tr.unreal_S / E if tr.unreal else 0.0
    alg, fwd = train_flops_per_env_step(h, w, T=T, recurrent=recurrent, aux=ax, unreal=un)
    flops, _ = train_flops_per_env_step(h, w, T=T, recurrent=recurrent, aux=ax, goal_fwd=gf, goal_bwd=gb, unreal=un)
    tflops = E * T * updates * flops / el / 1e12
    ceil = issued_ceiling_tflops(h, w, T=T, recurrent=recurrent, aux=ax, goal_fwd=gf, goal_bwd=gb, unreal=un)
    if model is None:
        model = "BigGoalHouseModel (LSTM core)" if recurrent else "BigGoalHouseModel trunk + heads (no LSTM)"
    res = {"model": model, "frame": [h, w, 3],
           **({"episodes": {"hardness": hardness, "max_episode_steps": max_episode_steps}}
              if hardness is not None or max_episode_steps != 900 else {}),
           "value": steps / el, "unit": "env-steps/s", "updates": updates, "envs_per_gpu": E,
           **({"cuda_graph": True} if cuda_graph else {}),
           "num_steps": T, "ms_per_update": el / updates * 1e3, "dtype": "f32",
           # peak = the ceiling of the MFMA forms the kernels issue (x3 / x6 split-bf16 products of
           # exact fp32 values, f32 MFMA elsewhere): frac = achieved / that ceiling, comparable with
           # the measured matrix-pipe busy fraction (mfma_busy_measured.busy_frac). The ratio to the
           # native fp32 MFMA peak (157.3 TF) is speed_vs_native_fp32_mfma: how much faster than an
           # exact-fp32 MFMA implementation at full rate, not a utilisation
           "roofline": {"bound": "mfma", "achieved": tflops, "peak": ceil, "unit": "TFLOP/s",
                        "frac": tflops / ceil, "peak_kind": "issued split-bf16 / f32 MFMA ceiling of these kernels",
                        "speed_vs_native_fp32_mfma": tflops / FP32_MFMA_PEAK_TFLOPS,
                        "flops_per_env_step": flops,
                        "scope": "whole update (all kernels), executed FLOPs (fp32-equivalent): the reference's "
                                 "algorithm minus the goal frames' shared_base skipped by goal-run deduplication",
                        # the reference's algorithm (shared_base on every goal frame) at the same time
                        "algorithmic_flops_per_env_step": alg, "algorithmic_tflops": E * T * updates * alg / el / 1e12,
                        "goal_frames_computed": {"rollout_forward": gf, "update_backward": gb},
                        **({"algorithmic_note": "algorithmic_tflops counts the reference's shared_base on every goal "
                                                "frame; goal-run deduplication ran it on the fraction "
                                                "goal_frames_computed, so it can exceed the 157.3 TF fp32 peak"}
                           if E * T * updates * alg / el / 1e12 > FP32_MFMA_PEAK_TFLOPS else {}),
                        # the same FLOPs against the ceiling of the MFMA forms the kernels issue
                        # (x3 / x6 split-bf16, f32): frac_issued = achieved / that ceiling
                        "issued_ceiling_tflops": ceil, "frac_issued": tflops / ceil,
                        "issued_ceiling_terms": [[n, f, fl] for n, f, fl in
                                                 train_flops_terms(h, w, T=T, recurrent=recurrent, aux=ax,
                                                                   goal_fwd=gf, goal_bwd=gb, unreal=un)]}}
    if tr.unreal:
        res["unreal"] = {"sequences_per_update": tr.unreal_S, "pc_weight": tr.pc_weight, "rp_weight": tr.rp_weight,
                         "vr_weight": tr.vr_weight,
                         "source": ("the first S envs' sequences of a rollout drawn from the device replay ring "
                                    "(deep_rl's replay buffer; capacity and sequence shape parity unpinned)")
                         if tr.unreal_source == "replay" else
                         "the first S envs' on-policy sequences (deep_rl samples replayed ones; parity unpinned)"}
    if world > 1:
        P = tr.net.n_params
        hw = tr.net.offsets["head"][0]
        res["dist"] = {"backend": torch.distributed.get_backend(tr.group), "world": world,
                       "allreduce_bytes": 4 * P,
                       "buckets": [[4 * (P - hw), "heads + LSTM + aux heads (overlaps the trunk backward)"],
                                   [4 * hw, "trunk"]] if tr._buckets_split() else [[4 * P, "flat"]],
                       # compute-stream time from the end of the backward to the all-reduced
                       # gradient (HIP events): the exposed, not overlapped, collective time
                       "allreduce_exposed_ms_per_update": coll_ms}
    del tr, env
    return res


# training legs: name -> (bench_train keyword arguments, scene geometry, default updates / warmup)
LEGS = {
    "84": dict(recurrent=True),
    "ff": dict(recurrent=False),
    # thor-cached-auxiliary as logged (outputs/output.txt): 174x174 scenes, LSTM policy, aux
    # deconv loss with the experiment's weight 0.1 (experiments/thor_cached_auxiliary.py:42
    # overrides AuxiliaryTrainer's 0.05 default, ai2_auxiliary/trainer.py:25), 4 scenes
    # (AuxiliaryTrainer is an UnrealTrainer: the pixel-control / reward-prediction / value-replay
    # losses with the weights of :39-41 run too, on the first 16 envs' sequences)
    "174": dict(recurrent=True, aux_weight=AUX_WEIGHT_LOGGED, frame=(174, 174, 3), updates=3, warmup=1, unreal=True,
                model="AuxiliaryBigGoalHouseModel (LSTM + deconv + UNREAL heads), 174x174"),
    # the logged run's exact batch: 4 envs x 20 steps per update, one captured hipGraph per update
    "ref4": dict(recurrent=True, aux_weight=AUX_WEIGHT_LOGGED, frame=(174, 174, 3), envs=4, updates=400, warmup=3,
                 cuda_graph=True, unreal=True,
                 model="AuxiliaryBigGoalHouseModel (LSTM + deconv + UNREAL heads), 174x174, 4 envs (the logged "
                       "run's batch), hipGraph per update"),
    "c5": dict(recurrent=True, aux_weight=AUX_WEIGHT_LOGGED, frame=(300, 400, 3), envs=512, updates=3, warmup=1,
               unreal=True, model="AuxiliaryBigGoalHouseModel (LSTM + deconv + UNREAL heads), 300x400 (config C5)"),
}
# the logged run's operating point for goal-frame deduplication: a trained policy at hardness
# 0.01 ends its episodes in ~2 steps (outputs/output.txt), so about half the goal frames are new
# (the legs above, with a fresh policy, run to the 900-step TimeLimit: 5 % new). Here the
# episodes are cut at 2 steps by the TimeLimit, which reproduces that goal-frame turnover with
# the same kernels (the env step costs the same); the starts follow hardness 0.01.
_SHORT = dict(hardness=0.01, max_episode_steps=2)
LEGS["84_short"] = dict(LEGS["84"], **_SHORT, model="BigGoalHouseModel (LSTM core), episodes of <= 2 steps")
LEGS["174_short"] = dict(LEGS["174"], **_SHORT,
                         model="AuxiliaryBigGoalHouseModel (LSTM + deconv + UNREAL heads), 174x174, episodes of "
                               "<= 2 steps")
LEG_ORDER = ("84", "ff", "174", "ref4", "c5", "84_short", "174_short")
LEG_KEYS = {"84": "train", "ff": "train_feedforward", "174": "train_174_lstm_aux", "ref4": "train_174_lstm_aux_4env",
            "c5": "train_c5_300x400", "84_short": "train_84_short_episodes",
            "174_short": "train_174_lstm_aux_short_episodes"}


def leg_enabled(args, leg, world):
    return {"84": not args.no_train_84, "ff": not args.no_train_ff, "174": not args.no_train_ref and not args.no_train_174,
            "ref4": not args.no_train_ref and not args.no_train_ref4 and world == 1, "c5": not args.no_c5,
            "84_short": not args.no_train_84 and not args.no_short,
            "174_short": not args.no_train_ref and not args.no_train_174 and not args.no_short}[leg]


def run_leg(leg, args, scenes, dev, world, rank, updates=None, warmup=None, marker=False):
    kw = dict(LEGS[leg])
    frame = kw.pop("frame", None)
    sc = aux_scenes(4, frame) if frame else scenes
    up, wu = kw.pop("updates", None), kw.pop("warmup", None)
    updates = updates if updates is not None else up
    warmup = warmup if warmup is not None else wu
    res = bench_train(args, sc, dev, world, rank, updates=updates, warmup=warmup, marker=marker, **kw)
    if leg in ("174", "ref4"):
        # the same losses as the logged run (A2C + aux deconv + UNREAL pc / rp / vr), but deep_rl
        # ran the aux and UNREAL losses on sequences drawn from its replay buffer (extra trunk /
        # LSTM passes over them), this leg on the rollout's own sequences
        res["reference_log_fps"] = REFERENCE_LOG_FPS
        res["reference_log_note"] = ("the logged 106 env-steps/s ran the same losses (A2C + aux deconv + UNREAL pc / "
                                     "rp / vr) with the aux and UNREAL batches drawn from deep_rl's replay buffer; "
                                     "this leg computes them on the rollout's own sequences (no extra trunk passes)")
    if leg == "ref4" and not marker:
        eager = bench_train(args, sc, dev, world, rank, updates=100, warmup=3, recurrent=True,
                            aux_weight=AUX_WEIGHT_LOGGED, envs=4, model="eager", unreal=True)
        res["eager_value"] = eager["value"]
        res["eager_ms_per_update"] = eager["ms_per_update"]
        # the logged experiment's loss mix as thor-cached-auxiliary runs it: the aux deconv batch
        # and the UNREAL sequences drawn from the replay ring (their own trunk / LSTM passes), the
        # ring pushed and drawn on the device (vn_replay_push_draw), so the update is one hipGraph
        mix = bench_train(args, sc, dev, world, rank, updates=400, warmup=3, recurrent=True,
                          aux_weight=AUX_WEIGHT_LOGGED, envs=4, model="replay sources", unreal=True,
                          replay_sources=True, cuda_graph=True)
        mix_e = bench_train(args, sc, dev, world, rank, updates=100, warmup=3, recurrent=True,
                            aux_weight=AUX_WEIGHT_LOGGED, envs=4, model="replay sources, eager", unreal=True,
                            replay_sources=True)
        res["replay_sources"] = {"aux_source": "replay", "unreal_source": "replay", "cuda_graph": True,
                                 "value": mix["value"], "ms_per_update": mix["ms_per_update"],
                                 "eager_value": mix_e["value"], "eager_ms_per_update": mix_e["ms_per_update"]}
    return res


def ranks_seen(dev, world):
    """Which devices the ranks ran on (all-gather of rank, host, PCI bus / uuid): the first
    multi-GPU run shows that RCCL saw N ranks on N distinct GPUs."""
    import socket
    p = torch.cuda.get_device_properties(dev)
    ident = "%s:%s" % (socket.gethostname(), getattr(p, "pci_bus_id", None) if hasattr(p, "pci_bus_id")
                       else str(getattr(p, "uuid", dev.index)))
    seen = [None] * world
    torch.distributed.all_gather_object(seen, (int(os.environ.get("RANK", "0")), ident))
    return {"backend": torch.distributed.get_backend(), "world": world, "ranks_seen": len({r for r, _ in seen}),
            "distinct_devices": len({i for _, i in seen}), "devices": [i for _, i in sorted(seen)]}


def device_copy_rate(dev, nbytes, reps=20):
    """The chip's device-to-device copy rate at the env step's byte count: one copy of
    nbytes (= the step's frame reads, = its frame writes) moves 2 x nbytes through HBM.
    Context for roofline.frac: the env step is a gather + copy of the same volume."""
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    src.fill_(1)
    for _ in range(3):
        dst.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    e0.record()
    for _ in range(reps):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    del src, dst
    torch.cuda.empty_cache()
    return 2 * nbytes / (ms * 1e-3) / 1e9


# ---------------------------------------------------------------- CPU baseline
_CPU_SHARED = {}


def resize_standin(frame):
    """The cost of the reference's per-frame preprocessing at equal size
    (environments/gym_ai2thor/envs/cached.py:62-64: skimage 0.18 ``resize(image, (84, 84),
    anti_aliasing=True)``, 99.9 % of its step time) without skimage, which the bench's python
    lacks: float64 in [0, 1], an identity bilinear warp per channel (skimage's ``warp`` at
    factor 1, mode 'reflect' = ndimage 'mirror'), clip. Timed in the build container: 1007 us
    per 84x84x3 frame against 988 us for skimage's own call (DESIGN.md "Measurement")."""
    from scipy import ndimage as ndi
    x = frame.astype(np.float64) / 255.0
    out = np.empty_like(x)
    for c in range(x.shape[2]):
        ndi.affine_transform(x[:, :, c], np.eye(2), order=1, mode="mirror", output=out[:, :, c])
    return np.clip(out, 0.0, 1.0, out=out)


def _cpu_worker(args):
    n_envs, seconds, seed, frame_bytes, resize = args
    from oracle.envs import VectorEnvOracle
    sd = [dict(graph=g, spd=s, rewards=(1.0, -0.0, 0.0)) for g, s in _CPU_SHARED["scenes"]]
    o = VectorEnvOracle(sd, n_envs, seed, max_steps=900)
    arena = _CPU_SHARED["arena"]  # inherited copy-on-write from the parent, read only
    shape = _CPU_SHARED["frame_shape"]
    out_img = np.empty((n_envs, frame_bytes), dtype=np.uint8)
    out_goal = np.empty((n_envs, frame_bytes), dtype=np.uint8)
    rng = np.random.RandomState(seed)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        r = o.step(rng.randint(0, 4, size=n_envs))
        np.take(arena, r["img_row"], axis=0, out=out_img)
        np.take(arena, r["goal_row"], axis=0, out=out_goal)
        if resize:  # the reference preprocesses the image and the goal frame of every step
            for i in range(n_envs):
                resize_standin(out_img[i].reshape(shape))
                resize_standin(out_goal[i].reshape(shape))
        steps += 1
    return steps * n_envs, time.perf_counter() - t0


def host_cpu_info():
    """The host the CPU baseline ran on: logical CPUs of the machine (os.cpu_count / nproc),
    the CPUs this process may use (its affinity: the box's share), and the CPU model."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)), "model": model}


def _cpu_quota():
    """The cgroup CPU quota of this process (cpu.max 'quota period' -> CPUs), if any."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


def _cpu_run(workers, seconds, per, fb, resize=False):
    import multiprocessing as mp
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, [(per, seconds, 100 + i, fb, resize) for i in range(workers)])
    wall = time.perf_counter() - t0
    return sum(r[0] / r[1] for r in res), sum(r[0] for r in res), wall


def cpu_baseline(scenes, seconds, sweep="1,16,all"):
    """The oracle ('port') batched VectorEnv in numpy, one process per core (fork, before
    any GPU initialisation), each stepping 256 envs incl. the two-frame gather, at each
    process count of ``sweep`` ('all' = every CPU of this process's affinity). ``value`` /
    ``cores`` are the largest count; ``sweep`` holds every point (and the cgroup quota, when
    one limits the CPUs the box gives this job)."""
    fb = int(np.prod(scenes[0].frame_shape))
    rows = sum(s.n_states for s in scenes)
    _CPU_SHARED["scenes"] = [(s.graph, s.spd) for s in scenes]
    # frame contents do not change the cost of a gather; fill (not hash) the arena
    _CPU_SHARED["arena"] = np.full((rows, fb), 7, dtype=np.uint8)
    _CPU_SHARED["frame_shape"] = tuple(scenes[0].frame_shape)
    per = 256
    ncpu = len(os.sched_getaffinity(0))
    counts = []
    for tok in str(sweep).split(","):
        n = ncpu if tok.strip() == "all" else int(tok)
        n = max(1, min(n, ncpu))
        if n not in counts:
            counts.append(n)
    points = []
    for n in counts:
        rate, total, wall = _cpu_run(n, seconds, per, fb)
        points.append({"procs": n, "value": rate, "env_steps": total, "wall_s": wall})
    # the reference as written: the same port plus the per-frame resize's cost (stand-in), at
    # 1 process and at the fastest count above, 16 envs per process, half the time
    ras = []
    for n in sorted({1, max(points, key=lambda p: p["value"])["procs"]}):
        rate, total, wall = _cpu_run(n, seconds / 2, 16, fb, resize=True)
        ras.append({"procs": n, "value": rate, "env_steps": total, "wall_s": wall})
    _CPU_SHARED.clear()
    # value / cores: the fastest point (the box's cgroup quota can cap the CPUs this job gets
    # below its affinity mask: more processes than the quota only timeshare it)
    top = max(points, key=lambda p: p["value"])
    host = host_cpu_info()
    host["cgroup_cpu_quota"] = _cpu_quota()
    ra_top = max(ras, key=lambda p: p["value"])
    reference_as_written = {
        "value": ra_top["value"], "unit": "env-steps/s", "cores": ra_top["procs"], "sweep": ras,
        "sample": "the port above plus resize_standin() on both frames of every env-step (the cost of "
                  "cached.py:62-64's skimage resize, 1.02x of it per frame in the build container), 16 envs per "
                  "process, %.0f s" % (seconds / 2),
        "survey_measured": {"value_1_core": 592.0, "value_8_procs": 3177.0, "unit": "env-steps/s",
                            "source": "SURVEY.md §8d: the reference's own THORDiscreteCachedEnv (skimage resize "
                                      "included) timed in the build container (8 Xeon cores), not on this host"}}
    return dict(value=top["value"], unit="env-steps/s", cores=top["procs"], kind="port", host=host,
                sweep=points, reference_as_written=reference_as_written,
                note="value is the numpy port without the resize, a much faster CPU path than the reference as "
                     "written; reference_as_written times the port with the resize's cost",
                sample="oracle VectorEnvOracle (numpy), %s processes x %d envs, %.0f s each (incl. 2-frame gather "
                       "from a %d-row arena); value = the fastest point, %d processes"
                       % ("/".join(str(c) for c in counts), per, seconds, rows, top["procs"]))


# ---------------------------------------------------------------- GPU bench
def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import vnav

    scenes = [vnav.synthetic_scene(k) for k in range(args.scenes)]
    if args.pmc_leg:  # child of pmc_train_mfma: one leg, one warmup + one marked update
        torch.cuda.set_device(0)
        run_leg(args.pmc_leg, args, scenes, torch.device("cuda", 0), 1, 0, updates=1, warmup=1, marker=True)
        return
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(scenes, args.cpu_seconds, args.cpu_sweep)
    traffic, traffic_info = None, None
    mfma_pmc = {}
    if rank == 0 and world == 1 and not args.no_pmc:  # child rocprofv3 runs, before this process touches the GPU
        traffic, traffic_info = pmc_traffic(args.envs, args.scenes)
        if args.train_steps > 0:
            for leg in ("84", "174", "c5"):
                if leg_enabled(args, leg, world):
                    mfma_pmc[leg] = pmc_train_mfma(args, leg)

    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist
        kw = {"device_id": dev} if args.dist_backend == "nccl" else {}
        dist.init_process_group(args.dist_backend, rank=rank, world_size=world, **kw)

    E = args.envs
    env = vnav.VectorEnv(scenes, E, seed=1000 + rank, device=dev)
    fb = int(np.prod(env.frame_shape))
    out = dict(image=torch.empty((E,) + env.frame_shape, dtype=torch.uint8, device=dev),
               goal=torch.empty((E,) + env.frame_shape, dtype=torch.uint8, device=dev),
               reward=torch.empty(E, dtype=torch.float32, device=dev),
               done=torch.empty(E, dtype=torch.bool, device=dev),
               state=torch.empty(E, dtype=torch.int32, device=dev))
    # synthetic uniform actions for every warmup and timed step, generated on the device
    # before the timed region (the step's inputs are resident in HBM when timing starts)
    actions = torch.empty((args.warmup + args.steps, E), dtype=torch.int32, device=dev)
    for t in range(args.warmup + args.steps):
        env.random_actions(t, out=actions[t])

    # the device-copy reference rate runs before the warmup steps: ~3 ms of HBM-saturating
    # copies, so the timed window does not start on a GPU that has been idle since the scene
    # synthesis (the driver's 5-step warmup alone is 0.3 ms of work)
    copy_gbs = device_copy_rate(dev, E * 2 * fb)
    step = 0
    for _ in range(args.warmup):
        env.step(actions[step], out=out)
        step += 1

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    K = args.steps
    step_actions = list(actions.unbind(0))  # per-step views made before the timed region
    # one HIP event pair around the K launches (vn_step runs on torch's current stream): the
    # per-launch duration is the region's device time / K, inter-kernel gaps included. Event
    # records between every launch cost ~5 us of device time each step and slowed the
    # region itself by that much.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record()
    for k in range(K):
        env.step(step_actions[step], out=out)
        step += 1
    ev1.record()
    # poll the end event before the synchronize: a blocking wait that outlasts the runtime's
    # spin phase sleeps and is woken by an interrupt, which can add ~0.1-0.2 ms to a short
    # window (the driver's 20-step run measured 0.2 ms outside the kernels' event pair)
    while not ev1.query():
        pass
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / K
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    flags = env.error_flags()
    del env, out
    legs = {}
    if args.train_steps > 0:
        torch.cuda.empty_cache()
        for leg in LEG_ORDER:
            if not leg_enabled(args, leg, world):
                continue
            legs[leg] = run_leg(leg, args, scenes, dev, world, rank)
            torch.cuda.empty_cache()
    dist_info = None
    if world > 1:
        dist_info = ranks_seen(dev, world)
    if rank == 0:
        simds = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
        for leg, pm in mfma_pmc.items():
            if pm is None or legs.get(leg) is None:
                continue
            pm["simds"] = simds
            pm["busy_frac"] = pm["mfma_busy_cycles"] / (simds * pm["grbm_gui_active"] / 8.0)
            legs[leg]["roofline"]["mfma_busy_measured"] = pm
        env_steps = E * K * world
        value = env_steps / elapsed
        bpe = alg_bytes_per_env_step(fb)
        achieved = bpe * E / (kern_ms * 1e-3) / 1e9
        cache_mb = sum(s.n_states for s in scenes) * fb / 1e6
        line = {
            "metric": "env-steps/sec (whole node), 4096 parallel cached-THOR envs at 1/2/4/8 GPUs",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": "cached-THOR VectorEnv.step, %d synthetic 24x24 scenes (%.0f MB frame cache, "
                                   "%s), %d envs/GPU, 84x84x3 frames, uniform random actions, auto-reset, "
                                   "TimeLimit 900" % (args.scenes, cache_mb,
                                                      "HBM-resident" if cache_mb > 256 else "LLC-resident",
                                                      E),
                       "envs_per_gpu": E, "scenes": args.scenes, "frame": list(scenes[0].frame_shape),
                       "parallelism": "dp%d (independent env shards, replicated scene cache)" % world},
            "roofline": {"bound": "hbm", "kernel": "vn_step (env_kernel<MODE_STEP,16>)",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_detail": traffic_info, "bytes_per_env_step": bpe,
                         "bytes_per_launch": bpe * E, "kernel_ms": kern_ms,
                         # torch's device copy of the same frame bytes (read + write), same process
                         "device_copy_gbs": copy_gbs, "frac_of_device_copy": achieved / copy_gbs},
            "cpu_baseline": cpu,
            **{LEG_KEYS[k]: legs.get(k) for k in ("84", "ff", "174", "ref4")},
            **{LEG_KEYS[k]: legs[k] for k in LEG_ORDER[4:] if legs.get(k)},
            **({"dist": dist_info} if dist_info else {}),
            "error_flags": flags,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
        # a multi-GPU line is only valid when every rank joined, each on its own GPU under RCCL
        bad = dist_info["ranks_seen"] != world or (dist_info["backend"] == "nccl" and
                                                   dist_info["distinct_devices"] != world)
        if bad:
            print("bench.py: invalid distributed run: %d of %d ranks seen, %d distinct devices (backend %s)"
                  % (dist_info["ranks_seen"], world, dist_info["distinct_devices"], dist_info["backend"]),
                  file=sys.stderr)
            sys.exit(3)


if __name__ == "__main__":
    main()
