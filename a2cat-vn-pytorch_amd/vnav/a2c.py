"""A2C rollout/update loop on one GPU per process (RCCL all-reduce across processes).

Mirrors the deep_rl Trainer surface the reference drives (train.py:24-25,
experiments/thor_cached_auxiliary.py:26-56): hyper-parameters as attributes with the
reference's values (num_steps 20, gamma .99, RMSprop alpha .99 / eps 1e-5, grad-norm
clip 0.5, lr 7e-4 -> 0 linearly over max_time_steps), ``step()`` = one rollout of
num_steps on every local env + one update, ``run()`` loops to max_time_steps,
``create_env`` / ``create_model`` hooks. The loss is the standard A2C stated in
DESIGN.md ("A2C contract"; value/entropy coefficients are not visible in the
reference — deep-rl 0.2.9 is absent — so parity is unpinned at this level).

Everything per step is a device launch: policy forward on frames gathered zero-copy
from the scene cache by row index, categorical sampling, env step (index-only), then
returns, loss gradient, backward, one flat-buffer all-reduce, norm, clip + RMSprop. No
host synchronisation inside ``step(sync=False)``. The per-update values (sampling counter,
learning rate) come from a device-side schedule (``vn_a2c_rollout_begin``), so one update has no
per-call host arguments: with ``cuda_graph=True`` it is captured once in a hipGraph and
replayed (single process), which removes the per-launch host cost that dominates small
batches (the reference's own run is 4 envs x 20 steps, ~400 launches per update).

With a recurrent net (``recurrent=True``) each step also runs the LSTM core: the input is
[conv_merge features | one-hot last action | last reward] and the carried (h, c), both
zeroed where an episode starts (mask m_t = 1 - done_{t-1}); the update back-propagates
through the T steps of the rollout (truncated BPTT) and (h, c) carry on to the next.

With ``aux_weight > 0`` (AuxiliaryTrainer, experiments/ai2_auxiliary/trainer.py:21-55; its
default auxiliary_weight is 0.05, the logged thor-cached-auxiliary experiment sets 0.1 at
experiments/thor_cached_auxiliary.py:42) the update adds the deconv loss of AuxiliaryBigGoalHouseModel's
depth / segmentation / goal-segmentation heads against avg-pooled targets gathered from
the env's aux arena by row. The reference computes it on a sequence sampled from
UnrealTrainer's replay buffer (deep_rl, absent); here it uses the on-policy rollout batch
(documented deviation, parity unpinned at the trainer level).

With ``unreal=True`` (BigGoalHouseModel's pixel-control and reward-prediction heads,
models/goal.py:94-137; UnrealTrainer's losses with the weights pc 0.05, rp 1.0, vr 1.0 of
experiments/thor_cached_auxiliary.py:39-41) each update also runs, on the rollout sequences
of the first ``unreal_envs`` envs: pixel control (n-step Q-learning on the pixel change of
the image frames, gamma_pc 0.9, on the LSTM features, bootstrap from the last observation),
reward prediction (the sign class of the reward after three consecutive frames of one
episode, from their conv_base maps) and value replay (the critic against the n-step
returns). deep_rl draws these sequences from its replay buffer (absent): here they are the
on-policy sequences, and the loss formulas are the published algorithm's (parity unpinned,
csrc/vn_unreal_loss.hip, oracle/unreal.py).
"""
import ctypes
import os
import time
import warnings

import numpy as np
import torch

from . import _lib
from . import dist as vdist
from .policy import OUT_LD, PolicyNet, frames_from_rows


# rows at or below which vn_policy_heads takes its skinny path (kSkinnyRows, csrc/vn_skinny.h):
# there the env-step launch computes the heads with the same sums (vn_a2c_step.head_weight)
_FUSED_HEADS_MAX_ENVS = 16


class A2CTrainer:
    def __init__(self, env, net=None, params=None, num_steps=20, gamma=0.99, learning_rate=7e-4,
                 max_time_steps=2e6, rms_alpha=0.99, rms_epsilon=1e-5, max_gradient_norm=0.5,
                 value_coefficient=0.5, entropy_coefficient=0.01, seed=0, process_group=None, recurrent=False,
                 aux_weight=0.0, arch="goal", cuda_graph=False, aux_source="rollout", replay_size=8,
                 capture_collectives=False, allreduce_buckets=1, time_collectives=False, dedup_goals=None,
                 unreal=False, pc_weight=0.05, rp_weight=1.0, vr_weight=1.0, pc_gamma=0.9, unreal_envs=16,
                 unreal_source="rollout"):
        self.env = env
        self.lib = _lib.load()
        # check before every replayed UNREAL pass that the side stream's buffers and gradient
        # block are disjoint from the main stream's (_check_side_stream_disjoint)
        self.debug_streams = bool(os.environ.get("VN_DEBUG_STREAMS"))
        self.device = env.device
        self.num_steps = int(num_steps)
        self.gamma = float(gamma)
        self.learning_rate = float(learning_rate)
        self.max_time_steps = float(max_time_steps)
        self.rms_alpha = float(rms_alpha)
        self.rms_epsilon = float(rms_epsilon)
        self.max_gradient_norm = float(max_gradient_norm)
        self.value_coefficient = float(value_coefficient)
        self.entropy_coefficient = float(entropy_coefficient)
        self.seed = int(seed)
        self.group = process_group
        self.world, self.rank = vdist.world_of(process_group)
        if allreduce_buckets not in (1, 2):
            raise ValueError("allreduce_buckets must be 1 or 2")
        self.allreduce_buckets = int(allreduce_buckets)
        self.time_collectives = bool(time_collectives)
        if self.time_collectives and cuda_graph:
            raise ValueError("time_collectives records HIP events per update, which a captured hipGraph would replay "
                             "as fixed events: use one or the other")
        # exposed all-reduce time: the pending update's event pair and a running (sum, count)
        self._coll_pending = []
        self._coll_sum_ms, self._coll_count = 0.0, 0
        self._head_work = None
        self.aux_weight = float(aux_weight)
        self.net = net if net is not None else PolicyNet(env.frame_shape[:2], env.num_actions, self.device,
                                                         recurrent=recurrent, aux=self.aux_weight > 0, arch=arch,
                                                         unreal=unreal)
        self.recurrent = self.net.recurrent
        if self.aux_weight > 0 and (not self.net.aux or getattr(env, "aux_arena", None) is None):
            raise ValueError("aux_weight > 0 needs an aux policy (aux=True) and scenes with depth + segmentation")
        self.A = self.net.num_actions
        self.params = params if params is not None else self.net.init_params(self.seed)
        vdist.broadcast_params_(self.params, group=self.group)
        P = self.net.n_params
        E, T = env.num_envs, self.num_steps
        N = T * E
        kw = dict(device=self.device)
        self.grads = torch.zeros(P, dtype=torch.float32, **kw)
        self.square_avg = torch.zeros(P, dtype=torch.float32, **kw)
        self.acts = self.net.new_acts(N)
        self.boot_acts = self.net.new_acts(E)
        self.out = torch.zeros((N, OUT_LD), dtype=torch.float32, **kw)
        self.boot_out = torch.zeros((E, OUT_LD), dtype=torch.float32, **kw)
        self.rows_img = torch.zeros(N, dtype=torch.int32, **kw)
        self.rows_goal = torch.zeros(N, dtype=torch.int32, **kw)
        self.actions = torch.zeros(N, dtype=torch.int32, **kw)
        self.rewards = torch.zeros((T, E), dtype=torch.float32, **kw)
        self.dones = torch.zeros((T, E), dtype=torch.bool, **kw)
        self.states = torch.zeros(E, dtype=torch.int32, **kw)
        self.returns = torch.zeros(N, dtype=torch.float32, **kw)
        self.dout = torch.zeros((N, OUT_LD), dtype=torch.float32, **kw)
        self.stats = torch.zeros(4, dtype=torch.float32, **kw)
        self.norm_partial = torch.zeros(512, dtype=torch.float64, **kw)
        self.scalars = torch.zeros(2, dtype=torch.float32, **kw)
        self.episode_stats = torch.zeros(3, dtype=torch.float32, **kw)  # count, return sum, length sum
        # device schedule: [next sampling-counter base (updates * T), env-steps so far, this
        # update's counter base] and the learning rate of the update (vn_a2c_schedule)
        self.sched = torch.zeros(3, dtype=torch.int64, **kw)
        self.lr_dev = torch.zeros(1, dtype=torch.float32, **kw)
        self.workspace = torch.empty(self.net.workspace_floats(N), dtype=torch.float32, **kw)
        if self.recurrent:
            X = self.net.lstm["xcat"]
            A1 = self.A + 1
            f32 = dict(dtype=torch.float32, **kw)
            self.xcat = torch.zeros((N, X), **f32)
            self.lstm_acts = torch.zeros((N, 2048), **f32)
            # h and c of every step in one [2][T*E][512] buffer, and the carry into the next
            # rollout in one [2][E][512] buffer: the carry is one strided copy per update
            self._hc_all = torch.zeros((2, N, 512), **f32)
            self.h_all, self.c_all = self._hc_all[0], self._hc_all[1]
            self.gates = torch.zeros((E, 2048), **f32)
            self.masks = torch.ones((T, E), **f32)
            self.lra = torch.zeros((T, E, A1), **f32)
            self._hc0 = torch.zeros((2, E, 512), **f32)  # state entering the rollout
            self.h0, self.c0 = self._hc0[0], self._hc0[1]
            self.prev_action = torch.zeros(E, dtype=torch.int64, **kw)
            self.prev_reward = torch.zeros(E, **f32)
            self.prev_mask = torch.zeros(E, **f32)    # 0: the first step starts every episode
            self.boot_xcat = torch.zeros((E, X), **f32)
            self.boot_la = torch.zeros((E, 2048), **f32)
            self.boot_c = torch.zeros((E, 512), **f32)
            self.boot_h = torch.zeros((E, 512), **f32)
            self.boot_mask = torch.zeros(E, **f32)
            self.boot_lra = torch.zeros((E, A1), **f32)
            self.dz5 = torch.zeros((N, 512), **f32)
            self.lstm_ws = torch.empty(self.net.lstm_workspace_floats(T, E), **f32)
        if self.aux_weight > 0:
            self.a1, self.pred = self.net.aux_buffers(N)
            self.dpred = torch.empty_like(self.pred)
            self.dx4 = torch.zeros((N, self.net.fc_in), dtype=torch.float32, **kw)
            self.aux_stats = torch.zeros(4, dtype=torch.float32, **kw)
            self.aux_ws = torch.empty(self.net.aux_workspace_floats(), dtype=torch.float32, **kw)
            from .policy import AuxTargets
            self.aux_table = self.net.aux_target_table(*env.aux_arena)  # once per scene cache
            self._aux_targets = AuxTargets(self.aux_table.data_ptr(), self.rows_img.data_ptr(),
                                           self.rows_goal.data_ptr())
            ph, pw = self.net.aux_layout["p_hw"]
            self._aux_numel = torch.tensor([1.0, 3.0, 3.0], device=self.device) * (N * ph * pw)
        # aux batch source: "rollout" = the on-policy batch (its trunk activations are reused),
        # "replay" = a sequence from the last replay_size rollouts (AuxiliaryTrainer's
        # self.replay.sample_sequence(), experiments/ai2_auxiliary/trainer.py:29): its own
        # trunk forward + backward, gradients added to the on-policy ones
        if aux_source not in ("rollout", "replay"):
            raise ValueError("aux_source must be 'rollout' or 'replay'")
        if unreal_source not in ("rollout", "replay"):
            raise ValueError("unreal_source must be 'rollout' or 'replay'")
        self.aux_source = aux_source
        self.unreal_source = unreal_source if unreal else "rollout"
        # the replay ring of the last replay_size rollouts (deep_rl's replay buffer, absent: its
        # capacity and sequence shape are parity unpinned); one stored rollout is drawn per update.
        # Push and draw run on the device (vn_replay_push_draw: meta = [next slot, filled, draw
        # counter, drawn slot]), so an update with replay sources is captured by cuda_graph=True.
        self.replay = aux_source == "replay" or self.unreal_source == "replay"
        if self.replay:
            self.replay_rows = torch.zeros((int(replay_size), 2, N), dtype=torch.int32, **kw)
            self.replay_meta = torch.zeros(4, dtype=torch.int64, **kw)
            self._replay_seed = vdist.rank_seed(self.seed + 17, self.rank) & ((1 << 64) - 1)
        if aux_source == "replay":
            if self.aux_weight <= 0:
                raise ValueError("aux_source='replay' needs aux_weight > 0")
            self.aux_rows = torch.zeros((2, N), dtype=torch.int32, **kw)
            self.aux_acts = self.net.new_acts(N)
            self.aux_out = torch.zeros((N, OUT_LD), dtype=torch.float32, **kw)
            self.aux_dz5 = torch.zeros((N, 512), dtype=torch.float32, **kw)
            self.aux_grads = torch.zeros(P, dtype=torch.float32, **kw)
            from .policy import AuxTargets
            self._aux_targets_replay = AuxTargets(self.aux_table.data_ptr(), self.aux_rows[0].data_ptr(),
                                                  self.aux_rows[1].data_ptr())
        # compute_auxiliary_loss overridden by a subclass: called every update (autograd on a
        # GoalNavPolicy view of the flat parameters), its gradient added before the all-reduce
        self._setup_unreal(unreal, pc_weight, rp_weight, vr_weight, pc_gamma, unreal_envs)
        # opt-in (VN_REPLAY_MERGED=1), both batches replayed and the UNREAL record holding every
        # env (S == E, the logged run's 4 envs): the replayed UNREAL pass's trunk forward covers
        # the aux batch's samples (rows t*S + e = t*E + e), so the aux heads can run on it inside
        # the side pass, their dX4 joining its trunk backward — one trunk forward + backward of
        # the replayed rollout instead of two. Measured slower (2.51 vs 2.40 ms per 4-env update,
        # tools/ab/replay_ab.sh): the side stream becomes the critical path while the main
        # stream idles, so the two passes stay the default.
        self._merged_replay = (self.aux_source == "replay" and self.unreal_source == "replay"
                               and self.unreal_S == E and bool(os.environ.get("VN_REPLAY_MERGED")))
        # VN_UNREAL_INLINE=1: the replayed UNREAL pass runs on the main stream before the A2C
        # backward instead of beside it (the race check: both forms must give the same update)
        self._unreal_inline = bool(os.environ.get("VN_UNREAL_INLINE"))
        if self.replay:
            self._replay_segs = self._replay_segments()
        self._custom_aux = type(self).compute_auxiliary_loss is not A2CTrainer.compute_auxiliary_loss
        if self._custom_aux and cuda_graph:
            raise ValueError("a compute_auxiliary_loss override runs torch autograd per update: use cuda_graph=False")
        self.aux_losses = {}
        self._model_view = None
        arena, fb, _, _ = env.frame_arena()
        self._arena, self._fb = arena, fb
        # goal-frame deduplication (vn_goal_runs): an env's goal frame is constant within an
        # episode, so shared_base runs on it once per goal run — at the rollout's first step and
        # after each done — and the backward sums a run's goal-map gradients before conv2 /
        # conv1 (same outputs, gradients up to summation order). Runs where the policy's
        # kernels take frame lists (84x84 / 174x174, more than 16 envs).
        # dedup_goals None = on where supported. Not with companion frames (OrientedGraphEnv's
        # third-person view, vn_env.hip goal_row = companion row + state): that second frame
        # changes at every step, so a run start's maps are not the later steps' maps.
        companion = any(getattr(s, "companion", None) is not None for s in getattr(env, "scenes", ()))
        if dedup_goals and companion:
            raise ValueError("dedup_goals=True needs a goal frame that is constant within an episode; these scenes "
                             "emit companion frames (a per-step third-person view) as the second frame")
        self.dedup_goals = (dedup_goals is None or bool(dedup_goals)) and not companion and \
            self.net.arch == "goal" and self.net.goal_runs_supported(E)
        if self.dedup_goals:
            i32 = dict(dtype=torch.int32, **kw)
            self.goal_delta = torch.zeros((T, E), **i32)
            self.goal_list_step = torch.zeros((T, E), **i32)
            self.goal_count = torch.zeros(T + 1, **i32)  # per step, then the update's
            self.goal_list = torch.zeros(N, **i32)
            self.goal_run_length = torch.zeros(N, **i32)
            self._goal_runs_step = []
            for t in range(T):
                g = _lib.GoalRuns()
                g.goal_list = self.goal_list_step[t].data_ptr()
                g.goal_count = self.goal_count[t:t + 1].data_ptr()
                g.goal_delta = self.goal_delta[t].data_ptr()
                g.num_envs = E
                self._goal_runs_step.append(g)
            g = _lib.GoalRuns()
            g.goal_list = self.goal_list.data_ptr()
            g.goal_count = self.goal_count[T:T + 1].data_ptr()
            g.goal_delta = self.goal_delta.data_ptr()
            g.run_length = self.goal_run_length.data_ptr()
            g.num_envs = E
            self._goal_runs_update = g
        # the rollout's fused env steps (vn_step_a2c): sampling + step + bookkeeping, one launch
        # per step; per-env episode statistics reduced once per rollout (vn_a2c_episode_stats)
        self.stats_env = torch.zeros((3, E), dtype=torch.float32, **kw)
        # a few envs, recurrent: the heads of each rollout step run inside its env-step launch
        # (vn_a2c_step.head_weight: vn_policy_heads' skinny sums, bit-identical), one launch
        # fewer per step
        self._fused_heads = self.recurrent and E <= _FUSED_HEADS_MAX_ENVS
        self._a2c_steps = [self._a2c_step_args(t) for t in range(T)]
        env.observe(gather=False)  # refresh the obs row buffers for the first forward
        self.num_updates = 0
        self.total_steps = 0
        self.cuda_graph = bool(cuda_graph)
        if self.cuda_graph and self.world > 1:
            if not vdist.capturable(process_group):
                raise ValueError("cuda_graph=True at world > 1 needs the nccl (RCCL) backend: a gloo all-reduce "
                                 "cannot be captured in a hipGraph")
            if not capture_collectives:
                # the captured RCCL all-reduce has not run against eager updates on a multi-GPU
                # node (DESIGN.md "Multi-GPU"): opt in explicitly
                raise ValueError("cuda_graph=True at world > 1 captures the RCCL all-reduces in the hipGraph, which "
                                 "is not yet validated against eager updates: pass capture_collectives=True to opt in")
        self._graph = None
        self._graph_out = None
        self._graph_gen = None

    def _setup_unreal(self, unreal, pc_weight, rp_weight, vr_weight, pc_gamma, unreal_envs):
        """Buffers of the UNREAL losses: the first S envs' T + 1 LSTM features (the last row
        the bootstrap's) through the pixel-control heads, their T - 2 three-frame conv_base
        samples through reward prediction. unreal_source 'replay': the same losses on the first
        S envs' sequences of a stored rollout (their own trunk, LSTM and heads pass)."""
        self.unreal = bool(unreal)
        if not self.unreal:
            self.unreal_source = "rollout"
            return
        net, E, T = self.net, self.env.num_envs, self.num_steps
        if not (net.unreal and net.recurrent):
            raise ValueError("unreal=True needs a recurrent policy with the UNREAL heads")
        H, W = self.env.frame_shape[:2]
        C = self.pc_cells = net.pc_side  # 42 (goal.py:72, 112) or 20 (BigHouseModel, bignet.py:77-91)
        if H < 4 * C or W < 4 * C:
            raise ValueError("pixel control crops %d cells of 4 px: frames need >= %d px" % (C, 4 * C))
        if T < 3:
            raise ValueError("reward prediction needs num_steps >= 3")
        self.pc_weight, self.rp_weight, self.vr_weight = float(pc_weight), float(rp_weight), float(vr_weight)
        self.pc_gamma = float(pc_gamma)
        S = self.unreal_S = max(1, min(int(unreal_envs), E))
        kw = dict(dtype=torch.float32, device=self.device)
        n_pc = (T + 1) * S
        self.h_pc = torch.zeros((n_pc, 512), **kw)
        self.pcb, self.pc_a1, self.pc_p2, _ = net.pc_buffers(n_pc, with_q=False)
        self.dh_pc = torch.zeros((n_pc, 512), **kw)
        self.pc_ws = torch.empty(net.pc_workspace_floats(), **kw)
        F = net.fc_in
        n_rp = (T - 2) * S
        self.rp_x = torch.zeros((n_rp, 3 * F), **kw)
        self.rp_dx = torch.zeros((n_rp, 3 * F), **kw)
        self.rp_out = torch.zeros((n_rp, 4), **kw)
        self.rp_dout = torch.zeros((n_rp, 4), **kw)
        # rp's gradient w.r.t. conv_base's map: into the aux heads' dX4 when those run on the
        # rollout, else into its own buffer (rows of envs >= S stay zero)
        self.rp_into_aux = self.aux_weight > 0 and self.aux_source == "rollout"
        self.unreal_dx4 = None if self.rp_into_aux else torch.zeros((T * E, F), **kw)
        self.unreal_stats = torch.zeros(4, **kw)  # pc sum sq, rp mean CE, rp samples, vr sum sq
        self._unreal_norm = torch.tensor([1.0 / (T * S * C * C), 1.0, 1.0 / (T * S)], **kw)
        if self.unreal_source == "replay":
            self._setup_unreal_replay()

    def _setup_unreal_replay(self):
        """The replay ring's per-rollout record of the first S envs (rows t*S + e, the
        bootstrap observation at t = T) and the buffers of their forward / backward pass."""
        net, E, T, S = self.net, self.env.num_envs, self.num_steps, self.unreal_S
        R = self.replay_rows.shape[0]
        A1 = self.A + 1
        n = (T + 1) * S
        f32 = dict(dtype=torch.float32, device=self.device)
        i32 = dict(dtype=torch.int32, device=self.device)
        self.ur = dict(rows=torch.zeros((R, 2, n), **i32), actions=torch.zeros((R, T * S), **i32),
                       rewards=torch.zeros((R, T, S), **f32),
                       dones=torch.zeros((R, T, S), dtype=torch.bool, device=self.device),
                       masks=torch.zeros((R, T + 1, S), **f32), lra=torch.zeros((R, T + 1, S, A1), **f32),
                       hc0=torch.zeros((R, 2, S, 512), **f32))
        # the slot drawn this update, copied out of the ring by vn_replay_push_draw (fixed
        # addresses: the replayed pass's launches do not depend on which slot was drawn)
        self.ur_cur = {key: torch.zeros_like(v[0]) for key, v in self.ur.items()}
        X = net.lstm["xcat"]
        # Side-stream-owned (update(): the replayed pass runs on self._side_u beside the A2C
        # backward): ur_* and ur_cur, h_pc / pcb / pc_a1 / pc_p2 / dh_pc / pc_ws, rp_x / rp_dx /
        # rp_out / rp_dout, unreal_stats, and the pc / rp blocks of self.grads
        # (_side_grad_ranges()). Nothing on the main stream may touch them between the fork and
        # the join — checked by _check_side_stream_disjoint (VN_DEBUG_STREAMS=1 or
        # A2CTrainer.debug_streams) and tests/test_unreal_gpu.py.
        self.ur_acts = net.new_acts(n)
        self.ur_xcat = torch.zeros((n, X), **f32)
        self.ur_lacts = torch.zeros((n, 2048), **f32)
        self.ur_hc = torch.zeros((2, n, 512), **f32)
        self.ur_gates = torch.zeros((S, 2048), **f32)
        self.ur_out = torch.zeros((n, OUT_LD), **f32)
        self.ur_returns = torch.zeros(T * S, **f32)
        self.ur_dout = torch.zeros((n, OUT_LD), **f32)
        self.ur_dz5 = torch.zeros((n, 512), **f32)
        self.ur_dx4 = torch.zeros((n, net.fc_in), **f32)  # the bootstrap rows stay zero
        self.ur_grads = torch.zeros(net.n_params, **f32)
        self.ur_ws = torch.empty(net.workspace_floats(n), **f32)
        self.ur_lstm_ws = torch.empty(net.lstm_workspace_floats(T + 1, S), **f32)
        # the grads of the trunk, heads and LSTM (everything before the aux / UNREAL blocks)
        self._ur_add_end = net.lstm["bhh"] + 2048
        # the replayed pass runs on a side stream beside the A2C backward (update()): its own
        # policy handle, so its small-batch split-K products have their own scratch
        self._net_u = PolicyNet(net.frame_hw, net.num_actions, self.device, recurrent=net.recurrent, aux=net.aux,
                                arch=net.arch, unreal=net.unreal)
        self._side_u = torch.cuda.Stream(device=self.device)
        self._ev_u0, self._ev_u1 = torch.cuda.Event(), torch.cuda.Event()

    def _unreal_forward_losses(self):
        """UNREAL losses of this rollout: vr into dout, pc and rp head gradients into grads;
        returns (dh_extra [T, S, 512], dX4 target). Runs after vn_a2c_loss_grad."""
        lib, net = self.lib, self.net
        E, T, A, S = self.env.num_envs, self.num_steps, self.A, self.unreal_S
        N = T * E
        P, st = _lib.ptr, self._stream()
        self.unreal_stats.zero_()
        if self.vr_weight > 0:
            _lib.check(lib.vn_unreal_vr_grad(P(self.out), P(self.returns), T, E, S, A, ctypes.c_float(self.vr_weight),
                                             P(self.dout), P(self.unreal_stats[3:]), st), "vn_unreal_vr_grad")
        # pixel control on h of the first S envs (+ the bootstrap's), reward prediction on three
        # consecutive conv_base maps of the same envs: both inputs gathered in one launch
        F = net.fc_in
        x4 = net.x4(self.acts, N)
        _lib.check(lib.vn_unreal_gather(P(self.h_all), P(self.boot_h), P(x4), T, E, S, F, P(self.h_pc), P(self.rp_x),
                                        st), "vn_unreal_gather")
        n_pc = (T + 1) * S
        net.pc_forward(self.params, self.h_pc, n_pc, self.pcb, self.pc_a1, self.pc_p2, None, self.pc_ws)
        H, W = self.env.frame_shape[:2]
        info = self.env._info
        # q formed from p2 in the loss kernel, which leaves dL/dp2 in p2 for the backward
        _lib.check(lib.vn_unreal_pc_loss_grad_ex(P(self.pc_p2), self.pc_cells, P(self.actions), P(self.dones),
                                                 ctypes.c_void_p(self._arena), ctypes.c_int64(self._fb), H, W,
                                                 P(self.rows_img), P(info["img_row"]), T, E, S, A,
                                                 ctypes.c_float(self.pc_gamma), ctypes.c_float(self.pc_weight),
                                                 P(self.unreal_stats), st), "vn_unreal_pc_loss_grad")
        net.pc_backward(self.params, self.h_pc, n_pc, self.pcb, self.pc_a1, self.pc_p2, None, self.grads, self.dh_pc,
                        self.pc_ws)
        n_rp = (T - 2) * S
        net.rp_forward(self.params, self.rp_x, n_rp, self.rp_out)
        _lib.check(lib.vn_unreal_rp_loss_grad(P(self.rp_out), P(self.rewards), P(self.dones), T, E, S,
                                              ctypes.c_float(self.rp_weight), P(self.rp_dout),
                                              P(self.unreal_stats[1:3]), st), "vn_unreal_rp_loss_grad")
        net.rp_backward(self.params, self.rp_x, n_rp, self.rp_dout, self.grads, self.rp_dx, self.pc_ws)
        dx4 = self.dx4 if self.rp_into_aux else self.unreal_dx4
        _lib.check(lib.vn_unreal_rp_scatter(P(self.rp_dx), T, E, S, F, P(dx4), int(self.rp_into_aux), st),
                   "vn_unreal_rp_scatter")
        return self.dh_pc[:T * S], dx4

    # deep_rl hook names (experiments/thor_cached_auxiliary.py:50-56)
    def create_env(self, kwargs):
        return self.env

    def create_model(self):
        return self.net

    def sample_training_batch(self):
        """deep_rl's UnrealTrainer.sample_training_batch (AuxiliaryTrainer adds the
        'auxiliary_batch', experiments/ai2_auxiliary/trainer.py:27-31): one rollout of
        num_steps on every local env. Returns (batch, report): the batch references the
        trainer's device buffers (valid until the next rollout), the report holds the
        finished-episode statistics [count, return sum, length sum] as a device tensor."""
        self.rollout()
        batch = RolloutBatch(self, self.rows_img, self.rows_goal)
        if self.replay:
            aux = self._replay_push_and_sample()
            if aux is not None:
                batch["auxiliary_batch"] = aux
        return batch, {"episode_stats": self.episode_stats}

    def compute_auxiliary_loss(self, model, batch, device):
        """deep_rl hook (experiments/ai2_auxiliary/trainer.py:33-43): extra loss terms on a
        batch -> (loss tensor or None, {name: float}). The default adds nothing here: the
        deconv loss of aux_weight > 0 is computed by the fused kernels inside update().
        An override receives a GoalNavPolicy view of the flat parameters (``model``) and the
        RolloutBatch; its loss's parameter gradient is added to the update's gradient
        before the all-reduce, clip and RMSprop."""
        return None, {}

    def model_view(self):
        """GoalNavPolicy (BigHousePolicy) over this trainer's PolicyNet whose parameter aliases
        the flat device buffer the kernels update."""
        if self._model_view is None:
            from .policy import GoalNavPolicy
            self._model_view = GoalNavPolicy.wrap(self.net, self.params)
        return self._model_view

    def _replay_segments(self):
        """The vn_replay_push_draw segments (include/vnav.h vn_replay_seg) of this trainer's
        ring: the frame rows of every sample (drawn into aux_rows for a replayed aux batch) and,
        with unreal_source='replay', the first S envs' record (frame rows of steps 0..T - 1 and
        of the bootstrap observation, actions, rewards, dones, the LSTM inputs of steps 0..T and
        the (h, c) the rollout started from), drawn into ur_cur."""
        E, T, N = self.env.num_envs, self.num_steps, self.num_steps * self.env.num_envs
        segs = []

        def seg(src, ld, rows, cols, ring, slot_elems, cur):
            eb = src.element_size()
            assert ring.element_size() == eb and (cur is None or cur.element_size() == eb)
            assert src.is_contiguous() and ring.is_contiguous() and (cur is None or cur.is_contiguous())
            segs.append(_lib.ReplaySeg(src.data_ptr(), ld, ring.data_ptr(), None if cur is None else cur.data_ptr(),
                                       slot_elems, rows, cols, eb, 0))

        aux = self.aux_source == "replay"
        for j, rows in enumerate((self.rows_img, self.rows_goal)):
            seg(rows, N, 1, N, self.replay_rows[0, j], 2 * N, self.aux_rows[j] if aux else None)
        if self.unreal_source == "replay":
            S, A1 = self.unreal_S, self.A + 1
            n = (T + 1) * S
            u, c, info = self.ur, self.ur_cur, self.env._info
            for j, (rows, last) in enumerate(((self.rows_img, info["img_row"]), (self.rows_goal, info["goal_row"]))):
                seg(rows, E, T, S, u["rows"][0, j], 2 * n, c["rows"][j])
                seg(last, S, 1, S, u["rows"][0, j, T * S:], 2 * n, c["rows"][j, T * S:])
            seg(self.actions, E, T, S, u["actions"][0], T * S, c["actions"])
            seg(self.rewards, E, T, S, u["rewards"][0], T * S, c["rewards"])
            seg(self.dones, E, T, S, u["dones"][0], T * S, c["dones"])
            seg(self.masks, E, T, S, u["masks"][0], (T + 1) * S, c["masks"])
            seg(self.boot_mask, S, 1, S, u["masks"][0, T], (T + 1) * S, c["masks"][T])
            seg(self.lra, E * A1, T, S * A1, u["lra"][0], (T + 1) * S * A1, c["lra"])
            seg(self.boot_lra, S * A1, 1, S * A1, u["lra"][0, T], (T + 1) * S * A1, c["lra"][T])
            seg(self._hc0, E * 512, 2, S * 512, u["hc0"][0], 2 * S * 512, c["hc0"])
        return (_lib.ReplaySeg * len(segs))(*segs)

    @property
    def replay_filled(self):
        """Filled slots of the replay ring (reads the device meta: synchronises)."""
        return int(self.replay_meta[1])

    @property
    def replay_pos(self):
        return int(self.replay_meta[0])

    def _replay_push_and_sample(self):
        """Store this rollout's frame rows (and, for the UNREAL losses, the first S envs'
        sequences) in the replay ring and draw one stored rollout (uniform over the filled
        slots) for this update's replayed batches, on the device in one call
        (vn_replay_push_draw: no host value, capturable). Returns the aux batch (None without
        aux replay)."""
        R = self.replay_rows.shape[0]
        _lib.check(self.lib.vn_replay_push_draw(self._replay_segs, len(self._replay_segs), _lib.ptr(self.replay_meta),
                                                R, self._replay_seed, self._stream()), "vn_replay_push_draw")
        if self.aux_source != "replay":
            return None
        return RolloutBatch(self, self.aux_rows[0], self.aux_rows[1])

    def _unreal_replay_losses(self, add=True):
        """UnrealTrainer's losses on the first S envs of the stored rollout drawn this update
        (deep_rl samples its sequences from a replay buffer, experiments/ai2_auxiliary/trainer.py
        :21-31; its sequence shape and initial state are absent, parity unpinned): trunk forward
        of their T + 1 observations, the LSTM over T + 1 steps from the (h, c) the rollout started
        from, the heads; value replay against their n-step returns (bootstrapped from step T),
        pixel control on their h, reward prediction on their conv_base maps; then the LSTM and
        trunk backward of those losses. Adds the trunk / heads / LSTM gradients to grads (the
        pixel-control and reward-prediction blocks are written there directly); add=False leaves
        that sum to the caller (update(): after the side stream's join). Runs on the second
        policy handle (its own split-K scratch)."""
        lib, net = self.lib, self._net_u
        T, S, A = self.num_steps, self.unreal_S, self.A
        n = (T + 1) * S
        P, st = _lib.ptr, self._stream()
        u = self.ur_cur  # the slot vn_replay_push_draw drew this update
        rows = u["rows"]
        frames = self._frames(rows[0], rows[1])
        net.forward(self.params, frames, n, self.ur_acts, n, 0, None)
        if self._merged_replay:  # the aux heads on the replayed rows t*E + e < T*E (aux_rows' frames)
            N = T * S
            self.aux_stats.zero_()
            net.aux_forward_loss_grad(self.params, self.ur_acts, n, N, self.a1, self.pred, self._aux_targets_replay,
                                      self.aux_weight, self.dpred, self.aux_stats, self.aux_ws)
            net.aux_backward(self.params, self.ur_acts, n, N, self.a1, self.dpred, self.grads, self.ur_dx4, self.aux_ws)
        x5 = net.x5(self.ur_acts, n)
        h_r, c_r = self.ur_hc[0], self.ur_hc[1]
        h0, c0 = u["hc0"][0], u["hc0"][1]
        for t in range(T + 1):
            sl = slice(t * S, (t + 1) * S)
            hp = h0 if t == 0 else h_r[(t - 1) * S:t * S]
            cp = c0 if t == 0 else c_r[(t - 1) * S:t * S]
            net.lstm_step(self.params, S, x5[sl], u["lra"][t], u["masks"][t], hp, cp, self.ur_xcat[sl],
                          self.ur_gates, self.ur_lacts[sl], c_r[sl], h_r[sl])
        net.heads(self.params, h_r, n, self.ur_out)
        self.unreal_stats.zero_()
        self.ur_dout.zero_()
        rew, don = u["rewards"], u["dones"]
        _lib.check(lib.vn_a2c_returns(P(rew), P(don), P(self.ur_out[T * S:]), T, S, A, ctypes.c_float(self.gamma),
                                      P(self.ur_returns), st), "vn_a2c_returns")
        if self.vr_weight > 0:
            _lib.check(lib.vn_unreal_vr_grad(P(self.ur_out), P(self.ur_returns), T, S, S, A,
                                             ctypes.c_float(self.vr_weight), P(self.ur_dout), P(self.unreal_stats[3:]),
                                             st), "vn_unreal_vr_grad")
        # pixel control on the replayed h (rows t*S + e, the bootstrap at t = T)
        net.pc_forward(self.params, h_r, n, self.pcb, self.pc_a1, self.pc_p2, None, self.pc_ws)
        H, W = self.env.frame_shape[:2]
        _lib.check(lib.vn_unreal_pc_loss_grad_ex(P(self.pc_p2), self.pc_cells, P(u["actions"]), P(don),
                                                 ctypes.c_void_p(self._arena), ctypes.c_int64(self._fb), H, W, P(rows[0]),
                                                 P(rows[0][T * S:]), T, S, S, A, ctypes.c_float(self.pc_gamma),
                                                 ctypes.c_float(self.pc_weight), P(self.unreal_stats), st),
                   "vn_unreal_pc_loss_grad")
        net.pc_backward(self.params, h_r, n, self.pcb, self.pc_a1, self.pc_p2, None, self.grads, self.dh_pc, self.pc_ws)
        # reward prediction on three consecutive conv_base maps of the replayed envs
        F = net.fc_in
        _lib.check(lib.vn_unreal_gather(None, None, P(net.x4(self.ur_acts, n)), T, S, S, F, None, P(self.rp_x), st),
                   "vn_unreal_gather")
        n_rp = (T - 2) * S
        net.rp_forward(self.params, self.rp_x, n_rp, self.rp_out)
        _lib.check(lib.vn_unreal_rp_loss_grad(P(self.rp_out), P(rew), P(don), T, S, S, ctypes.c_float(self.rp_weight),
                                              P(self.rp_dout), P(self.unreal_stats[1:3]), st), "vn_unreal_rp_loss_grad")
        net.rp_backward(self.params, self.rp_x, n_rp, self.rp_dout, self.grads, self.rp_dx, self.pc_ws)
        _lib.check(lib.vn_unreal_rp_scatter(P(self.rp_dx), T, S, S, F, P(self.ur_dx4), 1 if self._merged_replay else 0,
                                            st), "vn_unreal_rp_scatter")
        # BPTT over the T + 1 replayed steps (value replay's dout + pixel control's dh), the trunk
        net.lstm_backward(self.params, T + 1, S, self.ur_dout, h_r, self.ur_xcat, self.ur_lacts, c_r, c0,
                          u["masks"], x5, self.ur_dz5, self.ur_grads, self.ur_lstm_ws, dh_extra=self.dh_pc,
                          extra_envs=S)
        net.backward_ex(self.params, frames, n, self.ur_acts, n, None, self.ur_dz5, self.ur_dx4, self.ur_grads,
                        self.ur_ws)
        if add:
            self.grads[:self._ur_add_end].add_(self.ur_grads[:self._ur_add_end])

    def _side_grad_range(self):
        """[lo, hi) of the flat gradient the replayed UNREAL pass writes on the side stream: the
        pixel-control and reward-prediction blocks (include/vnav.h VN_POLICY_UNREAL layout),
        from the aux heads' block on when those run in the same pass (_merged_replay)."""
        lo = min(self.net.unreal_layout.values())
        if self._merged_replay:
            lo = min(lo, self.net.aux_layout["w1"])
        return lo, self.net.n_params

    def _side_owned(self):
        """(name, tensor) the side stream writes between the fork and the join."""
        lo, hi = self._side_grad_range()
        out = [(k, getattr(self, k)) for k in ("ur_acts", "ur_xcat", "ur_lacts", "ur_hc", "ur_gates", "ur_out",
                                               "ur_returns", "ur_dout", "ur_dz5", "ur_dx4", "ur_grads", "ur_ws",
                                               "ur_lstm_ws", "h_pc", "pcb", "pc_a1", "pc_p2", "dh_pc", "pc_ws",
                                               "rp_x", "rp_dx", "rp_out", "rp_dout", "unreal_stats")]
        out += [("ur_cur." + k, v) for k, v in self.ur_cur.items()]
        if self._merged_replay:
            out += [(k, getattr(self, k)) for k in ("a1", "pred", "dpred", "aux_ws", "aux_stats")]
        return out + [("grads[pc/rp]", self.grads[lo:hi])]

    def _main_owned(self):
        """(name, tensor) the main stream writes while the side stream runs."""
        lo, _ = self._side_grad_range()
        names = ("acts", "workspace", "dout", "returns", "stats", "out", "dz5", "dx4", "lstm_ws", "xcat", "lstm_acts",
                 "aux_acts", "aux_out", "aux_dz5", "aux_grads", "unreal_dx4", "norm_partial", "scalars", "_hc0", "h_all",
                 "c_all", "goal_list", "goal_run_length", "goal_count")
        if not self._merged_replay:
            names += ("a1", "pred", "dpred", "aux_ws", "aux_stats")
        out = [(k, getattr(self, k)) for k in names if isinstance(getattr(self, k, None), torch.Tensor)]
        return out + [("grads[trunk/heads/lstm/aux]", self.grads[:lo])]

    def _check_side_stream_disjoint(self):
        """The replayed UNREAL pass runs on a side stream beside the A2C backward (update()); it
        is race-free only while (1) its gradient block [pc_w, P) lies past every block the main
        stream writes and past the range the join adds ([0, _ur_add_end)), and (2) no buffer it
        writes shares memory with a buffer the main stream writes. Raises RuntimeError naming
        the first overlap (debug check: VN_DEBUG_STREAMS=1 or trainer.debug_streams = True)."""
        lo, hi = self._side_grad_range()
        net = self.net
        main_end = max(b + net.shapes[k][0] for k, (_, b) in net.offsets.items() if net.shapes[k][0])
        if net.lstm:
            main_end = max(main_end, net.lstm["bhh"] + 2048)
        if net.aux_layout and not self._merged_replay:
            main_end = max(main_end, net.aux_layout["b2"] + 8)
        if main_end > lo or self._ur_add_end > lo:
            raise RuntimeError("side-stream gradient block [%d, %d) overlaps the main stream's blocks (end %d) or the "
                               "join range [0, %d)" % (lo, hi, main_end, self._ur_add_end))

        def span(t):
            a = t.data_ptr()
            return a, a + t.numel() * t.element_size()

        main = [(k, span(t)) for k, t in self._main_owned() if t.numel()]
        for ks, ts in self._side_owned():
            if not ts.numel():
                continue
            a0, a1 = span(ts)
            for km, (b0, b1) in main:
                if a0 < b1 and b0 < a1:
                    raise RuntimeError("side-stream buffer %s overlaps main-stream buffer %s" % (ks, km))

    def _stream(self):
        return _lib.stream_ptr(self.device)

    def _a2c_step_args(self, t):
        """vn_a2c_step of rollout step t: sample from out[t], write actions[t], the next step's
        (last action, last reward) * mask and mask (the bootstrap slots after the last step),
        the recurrent carries and the per-env episode statistics."""
        E, T = self.env.num_envs, self.num_steps
        sl = slice(t * E, (t + 1) * E)
        s = _lib.A2CStep()
        s.policy_out = self.out[sl].data_ptr()
        s.num_actions = self.A
        s.seed = vdist.rank_seed(self.seed, self.rank)
        s.counter_base_dev = self.sched.data_ptr() + 2 * self.sched.element_size()
        s.counter = t
        s.actions = self.actions[sl].data_ptr()
        if self.recurrent:
            s.prev_action = self.prev_action.data_ptr()
            s.prev_reward = self.prev_reward.data_ptr()
            s.prev_mask = self.prev_mask.data_ptr()
            s.lra_next = (self.lra[t + 1] if t + 1 < T else self.boot_lra).data_ptr()
            s.mask_next = (self.masks[t + 1] if t + 1 < T else self.boot_mask).data_ptr()
        s.episode_stats_env = self.stats_env.data_ptr()
        if self._fused_heads:  # the heads of h_t in the same launch (out[t] written there)
            w_off, b_off = self.net.offsets["head"]
            s.head_weight = self.params.data_ptr() + 4 * w_off
            s.head_bias = self.params.data_ptr() + 4 * b_off
            s.head_input = self.h_all[sl].data_ptr()
            s.head_out = self.out[sl].data_ptr()
        return s

    def _frames(self, img_rows, goal_rows):
        return frames_from_rows(self._arena, self._fb, img_rows, goal_rows)

    def current_lr(self):
        """LinearSchedule(7e-4, 0, max_time_steps) (experiments/thor_cached_auxiliary.py:37)."""
        frac = min(self.total_steps / self.max_time_steps, 1.0) if self.max_time_steps > 0 else 0.0
        return self.learning_rate * (1.0 - frac)

    def _policy_step(self, t, frames):
        """Forward of step t of the rollout into self.out[t*E:(t+1)*E]."""
        net, E, N = self.net, self.env.num_envs, self.num_steps * self.env.num_envs
        sl = slice(t * E, (t + 1) * E)
        goals = None
        if self.dedup_goals:  # step t's new goals: all at t = 0, else the envs done at t - 1
            P = _lib.ptr
            _lib.check(self.lib.vn_goal_runs_step(P(self.dones[t - 1]) if t else None,
                                                  P(self.goal_delta[t - 1]) if t else None, E,
                                                  P(self.goal_delta[t]), P(self.goal_list_step[t]),
                                                  P(self.goal_count[t:t + 1]), self._stream()), "vn_goal_runs_step")
            goals = self._goal_runs_step[t]
        if not self.recurrent:
            net.forward(self.params, frames, E, self.acts, N, t * E, self.out[sl], goals=goals)
            return
        # step 0's mask / last action-reward come from vn_a2c_rollout_begin, later steps' from
        # the env step before them
        net.forward(self.params, frames, E, self.acts, N, t * E, None, goals=goals)
        hp = self.h0 if t == 0 else self.h_all[(t - 1) * E:t * E]
        cp = self.c0 if t == 0 else self.c_all[(t - 1) * E:t * E]
        net.lstm_step(self.params, E, net.x5(self.acts, N)[sl], self.lra[t], self.masks[t], hp, cp, self.xcat[sl],
                      self.gates, self.lstm_acts[sl], self.c_all[sl], self.h_all[sl])
        if not self._fused_heads:
            net.heads(self.params, self.h_all[sl], E, self.out[sl])

    def _bootstrap(self, frames):
        net, E = self.net, self.env.num_envs
        if not self.recurrent:
            net.forward(self.params, frames, E, self.boot_acts, E, 0, self.boot_out)
            return
        T = self.num_steps
        net.forward(self.params, frames, E, self.boot_acts, E, 0, None)
        last = slice((T - 1) * E, T * E)
        net.lstm_step(self.params, E, net.x5(self.boot_acts, E), self.boot_lra, self.boot_mask, self.h_all[last],
                      self.c_all[last], self.boot_xcat, self.gates, self.boot_la, self.boot_c, self.boot_h)
        net.heads(self.params, self.boot_h, E, self.boot_out)

    def rollout(self):
        env, net, lib = self.env, self.net, self.lib
        E, T, A = env.num_envs, self.num_steps, self.A
        N = T * E
        info = env._info
        # one launch: the device schedule, step 0's frame rows (later steps' rows are written
        # into their slots by the env step before them) and, recurrent, step 0's mask and
        # [one_hot(a) | r] * m from the carried last action / reward / mask
        rec = self.recurrent
        _lib.check(lib.vn_a2c_rollout_begin(
            _lib.ptr(self.sched), _lib.ptr(self.lr_dev), ctypes.c_double(self.learning_rate),
            ctypes.c_double(self.max_time_steps), ctypes.c_int64(N * self.world), T, _lib.ptr(info["img_row"]),
            _lib.ptr(info["goal_row"]), _lib.ptr(self.rows_img), _lib.ptr(self.rows_goal), E,
            _lib.ptr(self.prev_action) if rec else None, _lib.ptr(self.prev_reward) if rec else None,
            _lib.ptr(self.prev_mask) if rec else None, A, _lib.ptr(self.masks) if rec else None,
            _lib.ptr(self.lra) if rec else None, self._stream()), "vn_a2c_rollout_begin")
        for t in range(T):
            sl = slice(t * E, (t + 1) * E)
            self._policy_step(t, self._frames(self.rows_img[sl], self.rows_goal[sl]))
            # the emitted frames' arena rows go straight into step t + 1's slots (the last step's
            # into the env's own info rows: the bootstrap and the next rollout read them there)
            nxt = slice((t + 1) * E, (t + 2) * E)
            if t + 1 < T:
                env.set_row_outputs(self.rows_img[nxt], self.rows_goal[nxt])
            else:
                env.set_row_outputs(None, None)
            # one launch: the categorical draw from out[t] (Philox counter = updates * T + t from
            # the device schedule), the index-only env step, and the next step's recurrent
            # inputs, carries and episode statistics
            env.step_a2c(self._a2c_steps[t], self.rewards[t], self.dones[t], self.states)
        _lib.check(lib.vn_a2c_episode_stats(_lib.ptr(self.stats_env), E, _lib.ptr(self.episode_stats), self._stream()),
                   "vn_a2c_episode_stats")
        # bootstrap value of the final observation
        self._bootstrap(self._frames(info["img_row"], info["goal_row"]))

    def update(self, batch=None):
        """One A2C update on the rollout just sampled (``batch`` from sample_training_batch;
        None = the trainer's own rollout buffers with the on-policy aux batch; with
        unreal_source='replay' the rollout is then pushed into the ring and a sequence drawn)."""
        lib, net = self.lib, self.net
        E, T, A = self.env.num_envs, self.num_steps, self.A
        N = T * E
        st = self._stream()
        aux_batch = batch.get("auxiliary_batch") if batch is not None else None
        if batch is None and self.replay:
            # a bare rollout(): store it and draw this update's sequence now (the replayed aux
            # batch included, as sample_training_batch() would have)
            aux_batch = self._replay_push_and_sample()
        u_side = self.unreal and self.unreal_source == "replay"
        if u_side:
            # the replayed UNREAL pass reads the parameters and its own ring slot and writes its
            # own buffers and the pc / rp gradient blocks, which the A2C backward never touches:
            # it runs on a side stream from here; its trunk / heads / LSTM gradients are added
            # after the join below, in the unforked order
            if self.debug_streams:
                self._check_side_stream_disjoint()
            if self._unreal_inline:
                self._unreal_replay_losses(add=False)
            else:
                main = torch.cuda.current_stream(self.device)
                self._ev_u0.record(main)
                self._side_u.wait_event(self._ev_u0)
                with torch.cuda.stream(self._side_u):
                    self._unreal_replay_losses(add=False)
                    self._ev_u1.record(self._side_u)
        _lib.check(lib.vn_a2c_returns(_lib.ptr(self.rewards), _lib.ptr(self.dones), _lib.ptr(self.boot_out), T, E, A,
                                      ctypes.c_float(self.gamma), _lib.ptr(self.returns), st), "vn_a2c_returns")
        _lib.check(lib.vn_a2c_loss_grad(_lib.ptr(self.out), _lib.ptr(self.actions), _lib.ptr(self.returns), N, A,
                                        ctypes.c_float(self.value_coefficient),
                                        ctypes.c_float(self.entropy_coefficient), _lib.ptr(self.dout),
                                        _lib.ptr(self.stats), st), "vn_a2c_loss_grad")
        dx4 = None
        unreal_dh = None
        if self._merged_replay:
            pass  # the aux heads run inside the replayed UNREAL pass (side stream)
        elif self.aux_weight > 0 and aux_batch is not None:
            # replayed sequence: its own trunk forward, the heads' loss and backward, and the
            # trunk backward of dL/dX4 alone into aux_grads (added after the main backward)
            self.aux_stats.zero_()
            af = self._frames(aux_batch.rows_img, aux_batch.rows_goal)
            net.forward(self.params, af, N, self.aux_acts, N, 0, None if self.recurrent else self.aux_out)
            net.aux_forward_loss_grad(self.params, self.aux_acts, N, N, self.a1, self.pred, self._aux_targets_replay,
                                      self.aux_weight, self.dpred, self.aux_stats, self.aux_ws)
            net.aux_backward(self.params, self.aux_acts, N, N, self.a1, self.dpred, self.grads, self.dx4, self.aux_ws)
            net.backward_ex(self.params, af, N, self.aux_acts, N, None, self.aux_dz5, self.dx4, self.aux_grads,
                            self.workspace)
        elif self.aux_weight > 0:  # deconv heads: forward, loss gradient, backward -> dL/dX4
            # (in line: a side stream measured slower — their persistent kernels size their grids
            # to the whole chip, so nothing runs beside them; DESIGN "Two streams in the update")
            self.aux_stats.zero_()
            net.aux_forward_loss_grad(self.params, self.acts, N, N, self.a1, self.pred, self._aux_targets,
                                      self.aux_weight, self.dpred, self.aux_stats, self.aux_ws)
            net.aux_backward(self.params, self.acts, N, N, self.a1, self.dpred, self.grads, self.dx4, self.aux_ws)
            dx4 = self.dx4
        if self.unreal and self.unreal_source == "rollout":  # after the aux heads: rp adds to their dX4
            unreal_dh, dx4 = self._unreal_forward_losses()
        frames = self._frames(self.rows_img, self.rows_goal)
        goals = None
        if self.dedup_goals:  # the rollout's goal runs: starts ascending, run lengths
            P = _lib.ptr
            _lib.check(lib.vn_goal_runs_rollout(P(self.dones), T, E, P(self.goal_list), P(self.goal_run_length),
                                                P(self.goal_count[T:T + 1]), st), "vn_goal_runs_rollout")
            goals = self._goal_runs_update
        if self.recurrent:
            net.lstm_backward(self.params, T, E, self.dout, self.h_all, self.xcat, self.lstm_acts, self.c_all, self.c0,
                              self.masks, net.x5(self.acts, N), self.dz5, self.grads, self.lstm_ws,
                              dh_extra=unreal_dh, extra_envs=self.unreal_S if self.unreal else 0)
            # the heads + LSTM (+ aux heads) gradients are final here: their all-reduce runs on
            # RCCL's stream while the trunk backward runs on this one
            self._allreduce_head_bucket()
            net.backward_ex(self.params, frames, N, self.acts, N, None, self.dz5, dx4, self.grads, self.workspace,
                            goals=goals)
            # (h, c) after the last step carry into the next rollout (one copy launch)
            self._carry_states()
        else:
            net.backward_ex(self.params, frames, N, self.acts, N, self.dout, None, dx4, self.grads, self.workspace,
                            goals=goals)
        # the side passes' gradient sums: in the norm's first pass (vn_grad_norm_join) on one
        # rank with no override; before the all-reduce / the override's autograd otherwise
        joins = []
        if aux_batch is not None and not self._merged_replay:
            w, _ = self.net.offsets["conv1"]
            _, b = self.net.offsets["fc"]
            joins.append((self.aux_grads, w, b + self.net.shapes["fc"][0]))
        if u_side:
            if not self._unreal_inline:
                torch.cuda.current_stream(self.device).wait_event(self._ev_u1)
            joins.append((self.ur_grads, 0, self._ur_add_end))
        fuse_join = self.world == 1 and not self._custom_aux
        if not fuse_join:
            for g, lo, hi in joins:
                self.grads[lo:hi].add_(g[lo:hi])
            joins = []
        if self._custom_aux:
            loss, self.aux_losses = self.compute_auxiliary_loss(self.model_view(), batch, self.device)
            if loss is not None:
                g, = torch.autograd.grad(loss, self.model_view().params, allow_unused=True)
                if g is not None:
                    self.grads.add_(g)
        scale = self._allreduce_tail()
        P = net.n_params
        if joins:
            (a0, lo0, hi0), (a1, lo1, hi1) = (joins + [(None, 0, 0)])[:2]
            _lib.check(lib.vn_grad_norm_join(_lib.ptr(self.grads), P, _lib.ptr(a0), lo0, hi0, _lib.ptr(a1), lo1, hi1,
                                             ctypes.c_float(scale), ctypes.c_float(self.max_gradient_norm),
                                             _lib.ptr(self.norm_partial), _lib.ptr(self.scalars), st),
                       "vn_grad_norm_join")
        else:
            _lib.check(lib.vn_grad_norm(_lib.ptr(self.grads), P, ctypes.c_float(scale),
                                        ctypes.c_float(self.max_gradient_norm), _lib.ptr(self.norm_partial),
                                        _lib.ptr(self.scalars), st), "vn_grad_norm")
        # lr of this update from the device schedule (== current_lr() of the host counters)
        _lib.check(lib.vn_rmsprop_step_dev(_lib.ptr(self.params), _lib.ptr(self.grads), _lib.ptr(self.square_avg), P,
                                           ctypes.c_float(scale), _lib.ptr(self.scalars), _lib.ptr(self.lr_dev),
                                           ctypes.c_float(self.rms_alpha), ctypes.c_float(self.rms_epsilon), st),
                   "vn_rmsprop_step_dev")

    def _buckets_split(self):
        """Two gradient buckets when the head bucket is final before the trunk backward:
        [head.w, P) = heads + LSTM + aux heads (flat layout, include/vnav.h), [0, head.w) =
        the conv / conv_merge trunk. One bucket otherwise (feed-forward nets compute heads and
        trunk in one call; a compute_auxiliary_loss override may touch every parameter)."""
        return (self.world > 1 and self.allreduce_buckets == 2 and self.recurrent and not self._custom_aux
                and self.unreal_source != "replay")  # the replayed UNREAL pass adds to head / LSTM grads later

    def _allreduce_head_bucket(self):
        self._head_work = None
        if not self._buckets_split():
            return
        hw, _ = self.net.offsets["head"]
        self._head_work = vdist.allreduce_async_(self.grads[hw:], self.group)

    def _allreduce_tail(self):
        """The remaining all-reduce (the trunk bucket, or the whole flat gradient) and the
        wait for the head bucket; returns the 1/world scale. With time_collectives the
        compute-stream time from here to the all-reduced gradient (the exposed, not
        overlapped, collective time) is recorded per update."""
        if self.world == 1:
            return 1.0
        ev = None
        if self.time_collectives:
            self._collect_pending()
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        if getattr(self, "_head_work", None) is not None:
            hw, _ = self.net.offsets["head"]
            scale = vdist.allreduce_gradients_(self.grads[:hw], self.group)
            self._head_work.wait()
            self._head_work = None
        else:
            scale = vdist.allreduce_gradients_(self.grads, self.group)  # RCCL, one flat bucket
        if ev is not None:
            ev[1].record()
            self._coll_pending.append(ev)
        return scale

    def _collect_pending(self, wait=False):
        """Fold the completed event pairs into the running (sum, count): non-blocking unless
        ``wait`` or more than 8 pairs are pending, so the record stays bounded however long
        the run and the host does not stall behind the device."""
        keep = []
        for k, ev in enumerate(self._coll_pending):
            if wait or len(self._coll_pending) - k > 8 or ev[1].query():
                ev[1].synchronize()
                self._coll_sum_ms += ev[0].elapsed_time(ev[1])
                self._coll_count += 1
            else:
                keep.append(ev)
        self._coll_pending = keep

    def collective_ms(self):
        """Mean exposed all-reduce time per update (ms) over the updates since the last call
        (syncs on the last update's events); None when nothing was recorded."""
        self._collect_pending(wait=True)
        if not self._coll_count:
            return None
        ms = self._coll_sum_ms / self._coll_count
        self._coll_sum_ms, self._coll_count = 0.0, 0
        return ms

    def _carry_states(self):
        """(h0, c0) = (h, c) of the rollout's last step, both in one strided copy."""
        E, T = self.env.num_envs, self.num_steps
        self._hc0.copy_(self._hc_all.view(2, T, E, 512)[:, T - 1])

    def _add_trunk_grads(self, g):
        """grads[trunk] += g[trunk]: the conv / conv_merge layers (the only ones backward_ex
        writes when it is given dZ5 instead of the heads' output gradient)."""
        w, _ = self.net.offsets["conv1"]
        _, b = self.net.offsets["fc"]
        end = b + self.net.shapes["fc"][0]
        self.grads[w:end].add_(g[w:end])

    def _update_metrics(self):
        """rollout + update; returns the device metric vector [value_loss, action_loss,
        entropy, return mean, grad norm, aux loss, episodes, return sum, length sum]."""
        batch, _ = self.sample_training_batch()
        self.update(batch)
        N = self.num_steps * self.env.num_envs
        # [stats / N, grad norm, aux loss (sum of the per-head MSEs, trainer.py:51-54),
        # episode stats] in one launch; / N is torch's tensor / scalar (times the f32 reciprocal)
        # with the UNREAL losses + [pc loss, rp loss, vr loss] (means: averaged over ranks too)
        m = torch.empty(12 if self.unreal else 9, dtype=torch.float32, device=self.device)
        aux = self.aux_weight > 0
        P = _lib.ptr
        _lib.check(self.lib.vn_a2c_metrics_ex(P(self.stats), ctypes.c_float(np.float32(1.0) / np.float32(N)),
                                              P(self.scalars), P(self.aux_stats) if aux else None,
                                              P(self._aux_numel) if aux else None, P(self.episode_stats),
                                              P(self.unreal_stats) if self.unreal else None,
                                              P(self._unreal_norm) if self.unreal else None, P(m), self._stream()),
                   "vn_a2c_metrics_ex")
        vdist.reduce_metrics_(m, 6, self.group)
        if self.unreal and self.world > 1:
            m[9:] /= self.world
        return m

    def _graph_update(self):
        """The update through a captured hipGraph: the first update runs eagerly (kernel
        attributes and occupancy caches are set up), the second is captured — capture
        records the launches without running them — and every update replays it."""
        gen = getattr(self.env, "config_generation", 0)
        if self._graph is not None and gen != self._graph_gen:
            # the env was reconfigured after capture (tables, schedule, curriculum, limits):
            # the graph's launches point at the old buffers and arguments — capture again
            self._graph, self._graph_out = None, None
        if self._graph is None:
            if self.num_updates == 0:
                return self._update_metrics()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._graph_out = self._update_metrics()
            self._graph, self._graph_gen = g, gen
        self._graph.replay()
        return self._graph_out

    def step(self, sync=True):
        """One rollout (num_steps x num_envs) + one update. Returns the metric dict
        (deep_rl log keys) as floats when sync, else as device tensors."""
        t0 = time.perf_counter()
        m = self._graph_update() if self.cuda_graph else self._update_metrics()
        N = self.num_steps * self.env.num_envs
        self.total_steps += N * self.world
        self.num_updates += 1
        if not sync:
            # a graph replay writes the same static tensor every update: hand out a copy
            return {"raw": m.clone() if self.cuda_graph else m}
        vals = m.tolist()
        vl, al, ent, ret_mean, gnorm, aux_loss, eps, rsum, lsum = vals[:9]
        unreal = {}
        if self.unreal:
            unreal = {"pc_loss": vals[9], "rp_loss": vals[10], "vr_loss": vals[11]}
        dt = time.perf_counter() - t0
        return {
            "step": self.total_steps, "updates": self.num_updates,
            "value_loss": vl, "action_loss": al, "entropy": ent,
            "loss": self.value_coefficient * vl + al - self.entropy_coefficient * ent + (
                self.pc_weight * unreal["pc_loss"] + self.rp_weight * unreal["rp_loss"] +
                self.vr_weight * unreal["vr_loss"] if unreal else 0.0),
            "episodes": eps, "reward": rsum / eps if eps else float("nan"),
            "episode_length": lsum / eps if eps else float("nan"),
            "grad_norm": gnorm, "return_mean": ret_mean, "fps": N * self.world / dt,
            **({"aux_loss": aux_loss} if self.aux_weight > 0 else {}),
            **unreal,
        }

    def run(self, log_every=10, logger=print):
        while self.total_steps < self.max_time_steps:
            metrics = self.step(sync=(self.num_updates % log_every == 0))
            if "raw" not in metrics and self.rank == 0 and logger:
                logger(metrics)
        return self

    def evaluate(self, episodes=10, max_rollouts=10000):
        """deep_rl's Trainer.test() on this trainer's envs: the current policy (sampled
        actions), no update, until ``episodes`` episodes have finished on all ranks together
        (or ``max_rollouts`` rollouts). The recurrent state carries across rollouts as in
        training; the learning-rate step count is left as it was. Returns the episode count
        and the mean reward and length of the finished episodes."""
        saved_sched = self.sched.clone()  # sampling counter and step count: evaluation leaves both
        E, T = self.env.num_envs, self.num_steps
        tot = torch.zeros(3, dtype=torch.float64)
        for _ in range(int(max_rollouts)):
            self.rollout()
            if self.recurrent:  # (h, c) after the last step carry on, as update() does
                self._carry_states()
            st = self.episode_stats.to(torch.float64)
            vdist.reduce_metrics_(st, 0, self.group)
            tot += st.cpu()
            if tot[0] >= episodes:
                break
        self.sched.copy_(saved_sched)
        n, rsum, lsum = tot.tolist()
        return {"episodes": n, "reward": rsum / n if n else float("nan"),
                "episode_length": lsum / n if n else float("nan")}

    _RECURRENT_STATE = ("h0", "c0", "prev_action", "prev_reward", "prev_mask")

    def state_dict(self):
        sd = {"params": self.params.detach().cpu(), "square_avg": self.square_avg.cpu(),
              "env_state": self.env.get_state().cpu(), "env_ep_return": self.env.get_episode_returns().cpu(),
              "num_updates": self.num_updates, "sched": self.sched.cpu(),
              "total_steps": self.total_steps, "seed": self.seed, "rank": self.rank, "world": self.world}
        if self.recurrent:
            for k in self._RECURRENT_STATE:
                sd[k] = getattr(self, k).cpu()
        if self.replay:  # the replay ring and its draw stream resume exactly
            sd["replay_rows"] = self.replay_rows.cpu()
            sd["replay_meta"] = self.replay_meta.cpu()  # next slot, filled, draw counter, drawn slot
            if self.unreal_source == "replay":
                for key, v in self.ur.items():
                    sd["ur_" + key] = v.cpu()
        return sd

    def params_state_dict(self):
        """The world-agnostic part of the state: parameters, RMSprop state and the update /
        step counters (what a single-process ``test()`` needs after distributed training)."""
        return {"params": self.params.detach().cpu(), "square_avg": self.square_avg.cpu(),
                "num_updates": self.num_updates, "total_steps": self.total_steps, "sched": self.sched.cpu(),
                "seed": self.seed, "world": self.world, "params_only": True}

    def load_params_state_dict(self, sd):
        """Parameters (and RMSprop state, counters when present) of any world's checkpoint;
        the env state and recurrent carry of this trainer are left as they are."""
        if tuple(sd["params"].shape) != tuple(self.params.shape):
            raise ValueError("checkpoint holds %d parameters, this policy has %d"
                             % (sd["params"].numel(), self.params.numel()))
        self.params.copy_(sd["params"].to(self.device))
        if "square_avg" in sd:
            self.square_avg.copy_(sd["square_avg"].to(self.device))
        self.num_updates = int(sd.get("num_updates", self.num_updates))
        self.total_steps = int(sd.get("total_steps", self.total_steps))
        if "sched" in sd:
            self.sched.copy_(sd["sched"].to(self.device))

    def load_state_dict(self, sd):
        """Restore a state_dict() of this rank (env shard, running returns, recurrent carry
        are per rank; the env count must match)."""
        E = self.env.num_envs
        if tuple(sd["env_ep_return"].shape) != (E,):
            raise ValueError("checkpoint holds %d envs, this trainer has %d" % (sd["env_ep_return"].shape[0], E))
        if "world" in sd and (int(sd["world"]), int(sd["rank"])) != (self.world, self.rank):
            raise ValueError("checkpoint of rank %d/%d loaded on rank %d/%d"
                             % (int(sd["rank"]), int(sd["world"]), self.rank, self.world))
        self.params.copy_(sd["params"].to(self.device))
        self.square_avg.copy_(sd["square_avg"].to(self.device))
        self.env.set_state(sd["env_state"])
        self.env.set_episode_returns(sd["env_ep_return"])
        self.num_updates = int(sd["num_updates"])
        self.total_steps = int(sd["total_steps"])
        if "sched" in sd:
            self.sched.copy_(sd["sched"].to(self.device))
        else:  # checkpoints from before the schedule was saved
            self.sched.copy_(torch.tensor([self.num_updates * self.num_steps, self.total_steps, 0], dtype=torch.int64))
        if self.recurrent:
            for k in self._RECURRENT_STATE:
                getattr(self, k).copy_(sd[k].to(self.device))
        if self.replay:
            self._load_replay_state(sd)
        self.env.observe(gather=False)

    def _load_replay_state(self, sd):
        """The replay ring of a checkpoint. The ring restarts empty (with a warning) when the
        checkpoint has no ring, a ring of another capacity, or no UNREAL record while this
        trainer replays the UNREAL losses (a checkpoint of aux-only replay or of
        unreal_source='rollout'): restoring the frame rows alone would draw slots whose UNREAL
        record is empty. Checkpoints from before the device-side ring (host draw stream,
        'replay_fill_pos') keep their slots; the draw stream restarts at counter 0."""
        ring = sd.get("replay_rows")
        need_ur = self.unreal_source == "replay"
        why = None
        if ring is None:
            why = "the checkpoint holds no replay ring"
        elif tuple(ring.shape) != tuple(self.replay_rows.shape):
            why = "the checkpoint's ring is %s, this trainer's %s" % (tuple(ring.shape), tuple(self.replay_rows.shape))
        elif need_ur and any("ur_" + key not in sd for key in self.ur):
            why = "the checkpoint has no UNREAL record in its ring (saved without unreal_source='replay')"
        if why is not None:
            warnings.warn("replay ring restarts empty: " + why)
            self.replay_rows.zero_()
            self.replay_meta.zero_()
            if need_ur:
                for v in self.ur.values():
                    v.zero_()
            return
        self.replay_rows.copy_(ring.to(self.device))
        if "replay_meta" in sd:
            self.replay_meta.copy_(sd["replay_meta"].to(self.device))
        else:
            pos_filled = [int(x) for x in sd["replay_fill_pos"]]
            self.replay_meta.copy_(torch.tensor([pos_filled[1], pos_filled[0], 0, 0], dtype=torch.int64))
        if need_ur:
            for key, v in self.ur.items():
                v.copy_(sd["ur_" + key].to(self.device))


class RolloutBatch(dict):
    """A sampled batch (deep_rl's batch dict): the frame rows of every sample in the scene
    cache (time-major, row t*E + e) plus the trainer's rollout buffers; ``observations()``
    gathers the uint8 frames batch-first [E, T, H, W, 3] as the reference's wrappers
    deliver them (a device copy: only hooks that need pixels call it)."""

    def __init__(self, trainer, rows_img, rows_goal):
        super().__init__()
        self.trainer, self.rows_img, self.rows_goal = trainer, rows_img, rows_goal
        T, E = trainer.num_steps, trainer.env.num_envs
        self["actions"] = trainer.actions.view(T, E)
        self["rewards"] = trainer.rewards
        self["dones"] = trainer.dones

    def observations(self):
        tr = self.trainer
        T, E = tr.num_steps, tr.env.num_envs
        shape = tuple(tr.env.frame_shape)
        out = []
        for rows in (self.rows_img, self.rows_goal):
            dst = torch.empty((T * E,) + shape, dtype=torch.uint8, device=tr.device)
            _lib.check(tr.lib.vn_gather_rows(ctypes.c_void_p(tr._arena), int(tr._fb), _lib.ptr(rows), T * E,
                                             _lib.ptr(dst), tr._stream()), "vn_gather_rows")
            out.append(dst.view((T, E) + shape).transpose(0, 1))
        return tuple(out)
