/*
 * vnav.h — C ABI of libvnav.so, the MI355X-native batched cached-scene
 * visual-navigation engine (env.step hot path + A2C policy kernels).
 *
 * Every entry point returns 0 on success or a negative VN_E* code; the text of
 * the last error of the calling thread is available from vn_last_error().
 * Device buffers are caller-owned (e.g. torch tensors) and passed as raw
 * pointers; the library owns only the scene cache, per-env state and RNG keys.
 * All launches are stream-ordered and asynchronous; nothing here synchronises
 * the device except the explicitly named *_sync getters. A context is bound to
 * one GPU and is not thread-safe.
 *
 * Reference interfaces each group replaces (paths inside the reference repo
 * felipefelixarias/a2cat-vn-pytorch):
 *   vn_create/vn_destroy  <- THORDiscreteCachedEnv.__init__ loading the h5
 *                            datasets (environments/gym_ai2thor/envs/cached.py:19-36)
 *                            and THORCachedEnv.ensure_scene_loaded
 *                            (environments/gym_thor_cached.py:25-35)
 *   vn_reset              <- THORDiscreteCachedEnv.reset / _get_random_start_goal_tuple
 *                            (cached.py:38-57), THORCachedEnv.reset (gym_thor_cached.py:45-50)
 *   vn_observe            <- _render_observation / observe (cached.py:59-60,
 *                            gym_thor_cached.py:52-53)
 *   vn_step               <- THORDiscreteCachedEnv.step (cached.py:74-99) batched as the
 *                            deep_rl SubprocVecEnv.step with auto-reset
 *                            (experiments/thor_cached_auxiliary.py:66-67) and gym's
 *                            TimeLimit(max_episode_steps=900)
 *                            (environments/gym_ai2thor/__init__.py:45-49)
 *   vn_policy_*           <- BigGoalHouseModel trunk + heads (models/goal.py:36-59,77-92)
 *   vn_a2c_*              <- the deep_rl A2C update used by the Trainer
 *                            (experiments/thor_cached_auxiliary.py:26-42)
 */
#ifndef VNAV_H
#define VNAV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vn_ctx vn_ctx;
typedef void* vn_stream_t; /* a hipStream_t; NULL = the null stream */

enum {
  VN_OK = 0,
  VN_EINVAL = -1,   /* bad argument */
  VN_EHIP = -2,     /* HIP runtime error */
  VN_ENOMEM = -3,   /* device allocation failed */
  VN_ESTATE = -4,   /* call not valid in the context's current state */
};

/* Device-side error flags (sticky; read with vn_error_flags_sync). */
enum {
  VN_FLAG_BAD_ACTION = 1u << 0,     /* an action outside [0,4) was treated as a blocked move */
  VN_FLAG_RESET_EXHAUSTED = 1u << 1,/* no start with spd[s][g] > 0 found within the bounded search */
  VN_FLAG_BAD_SCHEDULE = 1u << 2,   /* a schedule entry was out of range */
};

/* One cached scene (the h5 layout written by graph/util.py:202-247):
 *   graph        [N][4] int64, -1 = blocked (row convention util.py:212-218,231-232)
 *   spd          [N][N] int64 shortest_path_distance (used by reset, cached.py:43)
 *   observations [N][H][W][C] uint8, or NULL to synthesise frames on the device
 *                from the counter hash (scene_id, state, word) documented in DESIGN.md
 * Rewards follow reward_configuration (cached.py:70-72, 84-88): a plain move
 * returns reward_step (cached.py uses -0.0), reaching the goal reward_goal, a
 * blocked move reward_collision. terminal_obs = 0 re-emits the previous
 * observation on a terminal step (cached.py:90-96); 1 emits the goal-state frame
 * (graph/env.py:130-133). */
typedef struct vn_scene_desc {
  int32_t n_states;
  int32_t height, width, channels;
  const int64_t* graph;
  const int64_t* spd;
  const uint8_t* observations;
  float reward_goal;
  float reward_step;
  float reward_collision;
  int32_t terminal_obs;
  uint32_t synth_id; /* scene id fed to the frame hash when observations == NULL */
  /* [n_states][H][W][C] or NULL. When set, the second output of every observation is the
   * companion frame of the emitted state instead of the goal frame: OrientedGraphEnv's
   * observation (rgb, third-person rgb) of ThorGridWorld.render (graph/thor_graph.py:15-33,
   * environments/gym_graph/graph.py:56-58). */
  const uint8_t* companion;
} vn_scene_desc;

/* ---- environment ------------------------------------------------------- */

int vn_create(const vn_scene_desc* scenes, int n_scenes, int n_envs, uint64_t seed,
              int device, vn_ctx** out);
int vn_destroy(vn_ctx* ctx);

/* Re-sample (scene, start, goal) for every env whose env_mask_dev[e] != 0
 * (NULL = all envs). */
int vn_reset(vn_ctx* ctx, const int32_t* env_mask_dev, vn_stream_t stream);

/* Write the current (image, goal) frames, [n_envs][H][W][C] uint8 each, and the
 * current state index per env; any output may be NULL. Also refreshes the img_row /
 * goal_row info buffers (vn_set_info_buffers). */
int vn_observe(vn_ctx* ctx, uint8_t* obs_dev, uint8_t* goal_dev, int32_t* state_dev,
               vn_stream_t stream);

/* One batched env.step. actions_dev: [n_envs] int32. Outputs per env: the
 * (image, goal) frames (NULL skips the gather: index-only step), reward f32,
 * done u8, state int32 (after any auto-reset). */
int vn_step(vn_ctx* ctx, const int32_t* actions_dev, uint8_t* obs_dev, uint8_t* goal_dev,
            float* reward_dev, uint8_t* done_dev, int32_t* state_dev, vn_stream_t stream);

/* The A2C rollout's env step (the trainer's fast path; vn_step stays the gym/VecEnv
 * boundary): the action of env e is sampled in the step from the policy's output row e
 * (categorical over logits 0..A-1 of policy_out [E][8], Philox stream 3 with counter
 * (e, *counter_base_dev + counter), key seed — the draw of vn_policy_sample_dev), the
 * index-only step runs on it, and the per-step bookkeeping of vn_a2c_step_post follows
 * in the same launch: the next step's recurrent inputs (last action one-hot and reward,
 * times the episode mask m = 1 - done) and the finished-episode statistics accumulated per
 * env into episode_stats_env [3][E] (count, return sum, length sum; reduced and cleared by
 * vn_a2c_episode_stats). Optional outputs may be NULL. */
typedef struct vn_a2c_step {
  const float* policy_out;          /* [E][8] */
  int num_actions;                  /* 1..7 */
  uint64_t seed;
  const int64_t* counter_base_dev;  /* may be NULL (base 0) */
  uint64_t counter;
  int32_t* actions;                 /* [E] sampled actions (out) */
  int64_t* prev_action;             /* [E] */
  float* prev_reward;               /* [E] */
  float* prev_mask;                 /* [E] */
  float* lra_next;                  /* [E][A+1] */
  float* mask_next;                 /* [E] */
  float* episode_stats_env;         /* [3][E], accumulated */
  /* Optional (a few envs): the policy heads computed in the same launch. With head_weight
   * non-NULL the logits and value of env e are head_bias + head_weight . head_input[e]
   * (head_weight [A+1][512], head_input [E][512], the same sums in the same order as
   * vn_policy_heads), written to head_out [E][8] — the buffer policy_out points at — and
   * sampled from; otherwise they are read from policy_out. */
  const float* head_weight;
  const float* head_bias;
  const float* head_input;
  float* head_out;
} vn_a2c_step;
int vn_step_a2c(vn_ctx* ctx, const vn_a2c_step* a2c, float* reward_dev, uint8_t* done_dev,
                int32_t* state_dev, vn_stream_t stream);

/* Optional persistent per-env info outputs written by every vn_step (any may be NULL):
 *   ep_return/ep_length: the finished episode's sum of rewards / length where done
 *     (RewardCollector statistics, experiments/thor_cached_auxiliary.py:60);
 *   terminal_state: the state index the single env returned as its terminal state;
 *   truncated: 1 where done came from the TimeLimit only;
 *   img_row/goal_row: global frame rows (arena rows, see vn_frame_arena) of the
 *     emitted frames — the zero-copy handle the fused policy input gather uses. */
int vn_set_info_buffers(vn_ctx* ctx, float* ep_return, int32_t* ep_length,
                        int32_t* terminal_state, uint8_t* truncated, int32_t* img_row,
                        int32_t* goal_row);

/* Test-mode exact replay: schedule_dev [n_envs][len][2] = (start, goal) consumed in
 * order by each env's subsequent resets (then back to the RNG). len = 0 clears. */
int vn_set_schedule(vn_ctx* ctx, const int32_t* start_goal_dev, int len);

/* Multi-scene tasks (gym_thor_cached.py:45-50): tasks_host [n][2] = (scene, goal);
 * goal = -1 draws a uniform goal. n = 0 restores fixed env->scene assignment. */
int vn_set_tasks(vn_ctx* ctx, const int32_t* tasks_host, int n_tasks);
/* Fixed env -> scene assignment (default e mod n_scenes). */
int vn_set_env_scenes(vn_ctx* ctx, const int32_t* env_scene_host);
int vn_set_max_episode_steps(vn_ctx* ctx, int max_steps); /* <= 0: no limit */

/* Curriculum start sampling (set_complexity / set_hardness: graph/util.py:88-143,
 * environments/gym_graph/graph.py:43-52, graph/env.py:101-106,
 * experiments/thor_cached_auxiliary.py:68-70). opt = complexity*(maxd + offset) + 1 with
 * maxd the scene's largest spd; starts with 0 < spd[s][g] <= opt are drawn uniformly
 * (mode 1, OrientedGraphEnv/sample_initial_state) or with probability 0.9 among them and
 * 0.1 among the farther ones (mode 2, SimpleGraphEnv/sample_initial_position); mode 0 =
 * off (uniform rejection sampling of cached.py). One O(1) draw from per-goal sorted tables
 * built on the first call. complexity and offset are fp64 (the reference computes opt in
 * Python floats, so floor(opt) matches it bit for bit). */
int vn_set_curriculum(vn_ctx* ctx, double complexity, int mode, double offset);
/* Per-scene (mode, offset) arrays of n_scenes entries (host memory). */
int vn_set_curriculum_scenes(vn_ctx* ctx, double complexity, const int32_t* modes_host,
                             const double* offsets_host);
int vn_set_autoreset(vn_ctx* ctx, int on);                /* default on */

/* Synthetic uniform actions in [0,4) from Philox(seed, env, step). */
int vn_random_actions(vn_ctx* ctx, int32_t* actions_dev, uint64_t step, vn_stream_t stream);
/* dst[i] = src[rows[i]] (rows of row_bytes, device memory): gathers the auxiliary frames
 * (depth, segmentation) of AuxiliaryGraph's 5-tuple observation (environments/gym_graph/
 * graph.py:96-120) by the env's img_row/goal_row indices. */
int vn_gather_rows(const uint8_t* src_dev, int64_t row_bytes, const int32_t* rows_dev, int n, uint8_t* dst_dev,
                   vn_stream_t stream);

/* Per-env state tensors (device, [n_envs] int32 each): for checkpoint/resume and tests.
 * Order: scene, state, goal, obs_state, elapsed, episode(reset count), sched_pos. */
int vn_get_state(vn_ctx* ctx, int32_t* dst_dev_7xE, vn_stream_t stream);
int vn_set_state(vn_ctx* ctx, const int32_t* src_dev_7xE, vn_stream_t stream);
/* Running (unfinished) episode return per env, [n_envs] f32 on the device: the rest of the
 * per-env state a checkpoint needs (the finished-episode return RewardCollector reports,
 * A18, is this sum at done). Tasks, scene assignment and curriculum are configuration and
 * are re-applied by the caller. */
int vn_get_episode_returns(vn_ctx* ctx, float* dst_dev_E, vn_stream_t stream);
int vn_set_episode_returns(vn_ctx* ctx, const float* src_dev_E, vn_stream_t stream);

/* Scene-cache arena: all scenes' frames back to back, row = frame. */
int vn_frame_arena(vn_ctx* ctx, const uint8_t** arena_dev, int64_t* frame_bytes,
                   int64_t* n_rows);
int vn_scene_row_base(vn_ctx* ctx, int scene, int64_t* row_base);

int vn_error_flags_sync(vn_ctx* ctx, uint32_t* flags, int clear);
int vn_num_envs(vn_ctx* ctx);


/* ---- policy: BigGoalHouseModel trunk + heads (models/goal.py:36-59,77-92) ---- */

typedef struct vn_policy vn_policy;

/* Frames for a batch of n samples (uint8 HWC, as the env emits them): sample i uses
 * image + image_rows[i]*frame_bytes and goal + goal_rows[i]*frame_bytes (rows NULL =
 * i). Passing the scene-cache arena (vn_frame_arena) with the env's img_row/goal_row
 * info makes the policy input a zero-copy gather. image_f32/goal_f32, when set, are
 * dense float [n][3][H][W] frames (the reference's TransposeImage + ScaledFloatFrame
 * output) used instead. */
typedef struct vn_frames {
  const uint8_t* image;
  const uint8_t* goal;
  const int32_t* image_rows;
  const int32_t* goal_rows;
  int64_t frame_bytes;
  const float* image_f32;
  const float* goal_f32;
} vn_frames;

/* frame 84x84 or 174x174; num_actions 1..7. Parameters live in one flat fp32 buffer:
 * per layer (conv1, conv2, conv3, conv4, conv_merge, head) W [Cout][ky][kx][Cin] (K padded
 * to a multiple of 4) then b [Cout]; the head stacks policy_logits (rows 0..A-1) and critic
 * (row A). layout12 = (w, b) float offsets per layer. */
int vn_policy_create(int frame_h, int frame_w, int num_actions, vn_policy** out);
int vn_policy_destroy(vn_policy* p);
int vn_policy_info(vn_policy* p, int64_t* n_params, int64_t* act_floats_per_sample, int64_t* layout12);
int vn_policy_workspace_floats(vn_policy* p, int64_t n_samples, int64_t* floats);
/* out [n][8]: logits in 0..A-1, value at A (out may be NULL for a VN_POLICY_LSTM policy:
 * trunk only, features kept in the activation store). Activations of the n samples are kept at
 * sample offset act_offset of an activation store holding act_capacity samples. */
int vn_policy_forward(vn_policy* p, const float* params, const vn_frames* frames, int n, float* acts,
                      int64_t act_capacity, int64_t act_offset, float* out, vn_stream_t stream);
/* Gradients of the n samples stored from offset 0 given dL/d(out) [n][8]; overwrites grads
 * (flat, same layout as params). Consumes the stored activations (conv1's are overwritten). */
int vn_policy_backward(vn_policy* p, const float* params, const vn_frames* frames, int n, float* acts,
                       int64_t act_capacity, const float* dout, float* grads, float* workspace,
                       vn_stream_t stream);

/* ---- recurrent core: MaskedRNN(nn.LSTM(512 + A + 1, 512)) (models/goal.py:61-67, 91-92) ----
 * A policy created with VN_POLICY_LSTM appends W_cat [2048][xcat] = [W_ih | 0 pad | W_hh]
 * (torch gate order i, f, g, o), b_ih [2048], b_hh [2048] to the flat parameters; its heads
 * read h_t instead of the conv_merge features. info8 = (W_cat, b_ih, b_hh offsets, xcat,
 * xoff = column of h in W_cat, lin = 512 + A + 1, hidden 512, 0).
 * Step t of a batch of E: x5 [E][512] conv_merge features (the trunk activations stored
 * by vn_policy_forward with out == NULL), lra [E][A+1] (one-hot last action, last reward;
 * NULL = zeros), mask [E] (0 resets the carried state: m * h_prev, m * c_prev; NULL = 1),
 * h_prev/c_prev [E][512] (NULL = zeros). Writes xcat [E][xcat], gates scratch [E][2048],
 * acts [E][2048] (i, f, g, o), c_out, h_out [E][512] — keep xcat/acts/c/h of every step of a
 * rollout (rows t*E + e) for vn_lstm_backward. */
#define VN_POLICY_LSTM 1
int vn_policy_create_ex(int frame_h, int frame_w, int num_actions, int flags, vn_policy** out);
int vn_policy_lstm_info(vn_policy* p, int64_t* info8);
int vn_lstm_forward_step(vn_policy* p, const float* params, int E, const float* x5, const float* lra,
                         const float* mask, const float* h_prev, const float* c_prev, float* xcat, float* gates,
                         float* acts, float* c_out, float* h_out, vn_stream_t stream);
/* Heads on n feature rows [n][512] -> out [n][8]. */
int vn_policy_heads(vn_policy* p, const float* params, const float* feat, int n, float* out, vn_stream_t stream);
int vn_lstm_workspace_floats(vn_policy* p, int T, int E, int64_t* floats);
/* BPTT within one rollout (the state entering it is a constant): writes the head and LSTM
 * gradients into grads and dL/d(conv_merge pre-activation) [T*E][512] into dz5_all. */
int vn_lstm_backward(vn_policy* p, const float* params, int T, int E, const float* dout, const float* h_all,
                     const float* xcat_all, const float* acts_all, const float* c_all, const float* c_init,
                     const float* mask_all, const float* x5_all, float* dz5_all, float* grads, float* workspace,
                     vn_stream_t stream);
/* vn_lstm_backward plus dh_extra [T][extra_envs][512]: another head's gradient w.r.t. h_t of
 * envs 0..extra_envs-1 (pixel control, vn_pc_backward), added to the policy heads'. */
int vn_lstm_backward_ex(vn_policy* p, const float* params, int T, int E, const float* dout, const float* h_all,
                        const float* xcat_all, const float* acts_all, const float* c_all, const float* c_init,
                        const float* mask_all, const float* x5_all, const float* dh_extra, int extra_envs,
                        float* dz5_all, float* grads, float* workspace, vn_stream_t stream);
/* Trunk gradients (conv1..conv_merge) of the n stored samples from dz5 [n][512]. */
int vn_policy_backward_trunk(vn_policy* p, const float* params, const vn_frames* frames, int n, float* acts,
                             int64_t act_capacity, const float* dz5, float* grads, float* workspace,
                             vn_stream_t stream);

/* ---- aux deconv heads: AuxiliaryBigGoalHouseModel (models/goal.py:144-189) and the
 * auxiliary deconv loss (experiments/ai2_auxiliary/trainer.py:9-55) ----
 * A policy created with VN_POLICY_AUX appends W1 [32][4][4][48], b1 [48] (the three heads'
 * ConvTranspose2d(32,16,4,2) side by side: depth 0-15, mask 16-31, goal mask 32-47) and
 * W2 [48][4][4][8], b2 [8] (ConvTranspose2d(16,C,4,2) per head, block diagonal: depth ->
 * channel 0, mask -> 1-3, goal mask -> 4-6, 7 padding). info8 = (W1, b1, W2, b2 offsets,
 * AH, AW = first deconv map, PH, PW = prediction map). Heads read conv_base's output (X4)
 * from the activation store of vn_policy_forward; a1 [n][AH][AW][48], pred [n][PH][PW][8]. */
#define VN_POLICY_AUX 2
/* BigHouseModel (models/bignet.py:26-75) instead of BigGoalHouseModel: image only (the goal
 * frames are ignored), Conv(3,32,k8,s4) ReLU, Conv(32,64,k4,s2) ReLU, Conv(64,32,k3) ReLU,
 * Linear(7*7*32, 512) ReLU (84x84 frames only, as the reference's Linear fixes), then the same
 * heads / recurrent core. Layer slots: conv1 [32][8][8][3], conv2 [64][4][4][32],
 * conv3 [32][3][3][64], (conv4 slot empty), conv_merge, head. */
#define VN_POLICY_BIGHOUSE 4
typedef struct vn_aux_targets {
  const float* table;           /* [rows][PH][PW][4] from vn_aux_target_table */
  const int32_t* image_rows;    /* [n] row of each sample's state (vn_frames.image_rows) */
  const int32_t* goal_rows;     /* [n] row of each sample's goal */
} vn_aux_targets;
int vn_policy_aux_info(vn_policy* p, int64_t* info8);
int vn_aux_workspace_floats(vn_policy* p, int64_t* floats);
int vn_aux_forward(vn_policy* p, const float* params, float* acts, int64_t act_capacity, int n, float* a1,
                   float* pred, float* workspace, vn_stream_t stream);
/* Per-state targets, built once per scene cache: table [n_rows][PH][PW][4] = (depth, seg0-2)
 * of avg_pool(centre crop(obs/255), 4) (compute_auxiliary_target, trainer.py:9-15) from the
 * depth [rows][H][W][1] and segmentation [rows][H][W][3] arenas (row-indexed like the frame
 * arena). */
int vn_aux_target_table(vn_policy* p, const uint8_t* depth, const uint8_t* segmentation, int height, int width,
                        int64_t n_rows, float* table, vn_stream_t stream);
/* dpred = weight * d(sum of per-head MSE)/dpred against the image row's (depth, seg) and the
 * goal row's seg targets; stats4[0..2] += per-head sums of squared errors. */
int vn_aux_loss_grad(vn_policy* p, const float* pred, int n, const vn_aux_targets* targets, float weight,
                     float* dpred, float* stats4, vn_stream_t stream);
/* vn_aux_forward + vn_aux_loss_grad in one pass: the second head layer computes each
 * prediction pixel and its loss gradient together (the trainer's path: the prediction is
 * never stored; pred is scratch, written only for maps too large for the fused kernel). */
int vn_aux_forward_loss_grad(vn_policy* p, const float* params, float* acts, int64_t act_capacity, int n,
                             float* a1, float* pred, const vn_aux_targets* targets, float weight,
                             float* dpred, float* stats4, float* workspace, vn_stream_t stream);
/* Head gradients into grads and dL/dX4 [n][h3][w3][32] (before conv_base's ReLU mask) into
 * dx4; consumes a1. */
int vn_aux_backward(vn_policy* p, const float* params, float* acts, int64_t act_capacity, int n, float* a1,
                    const float* dpred, float* grads, float* dx4, float* workspace, vn_stream_t stream);
/* ---- UNREAL heads: pixel control and reward prediction (models/goal.py:94-133,
 * models/bignet.py:77-111) ----
 * A policy created with VN_POLICY_UNREAL appends, 16-byte aligned (BigGoalHouseModel):
 *   pc_base W [2592][512] (rows in (y, x, c) order of the reference's (32, 9, 9) view), b [2592];
 *   pc W1 [32][4][4][64], b1 [64]: pc_value's ConvTranspose2d(32,32,4,2) -> channels 0-31,
 *     pc_action's -> 32-63;
 *   pc W2 [64][4][4][8], b2 [8]: block diagonal, pc_value's ConvTranspose2d(32,A,4,2) ->
 *     channels 0..A-1 from rows 0-31, pc_action's ConvTranspose2d(32,1,4,2) -> channel A from
 *     rows 32-63, the rest padding;
 *   rp W [3][3 * FCIN] (FCIN = h3 * w3 * 32; the three frames' conv_base maps, NHWC each:
 *     the reference's Linear(9*9*32*3, 3) at 174x174), b [4] (3 + pad).
 * With VN_POLICY_BIGHOUSE (BigHouseModel: one ConvTranspose2d(32, C, 4, 2) + ReLU per branch):
 *   pc_base W, b as above; pc W1 [32][4][4][8], b1 [8]: pc_value's ConvTranspose2d(32,A,4,2)
 *     -> channels 0..A-1, pc_action's ConvTranspose2d(32,1,4,2) -> channel A, the rest padding;
 *   no second layer (W2, b2 empty: their offsets equal rp W's); rp W [3][3 * 1568] (the
 *     reference's Linear(9*9*32*3, 3) fits 100x100 frames only: in_features derived), b [4].
 *   The pixel-control map is 20x20 (p2 [n][20][20][8], q [n][20][20][A]); a1 is unused (NULL ok);
 *   conv_base's output is X3, whose gradient vn_policy_backward_ex takes as dx4_extra.
 * info8 = (pc_base W, pc_base b, W1, b1, W2, b2, rp W, rp b offsets). */
#define VN_POLICY_UNREAL 8
int vn_policy_unreal_info(vn_policy* p, int64_t* info8);
int vn_pc_workspace_floats(vn_policy* p, int64_t* floats);
/* pixel_control (goal.py:131-137; bignet.py:105-111 with VN_POLICY_BIGHOUSE: a1 unused, p2
 * [n][20][20][8], q [n][20][20][A]) on feature rows h [n][512] (the LSTM outputs): writes
 * pcb [n][9][9][32], a1 [n][20][20][64], p2 [n][42][42][8] (kept for the backward) and
 * q [n][42][42][A] = (pc_value + pc_action) - mean_c(pc_action) (q may be NULL: not formed). */
int vn_pc_forward(vn_policy* p, const float* params, const float* h, int n, float* pcb, float* a1, float* p2,
                  float* q, float* workspace, vn_stream_t stream);
/* From dL/dq [n][42][42][A] (or dq == NULL: p2 already holds dL/dp2, as
 * vn_unreal_pc_loss_grad leaves it): the pixel-control parameter gradients into grads
 * (overwritten) and dL/dh [n][512] into dh (stored, or added to dh when accumulate != 0).
 * Consumes pcb, a1 and p2 (overwritten by their gradients). */
int vn_pc_backward(vn_policy* p, const float* params, const float* h, int n, float* pcb, float* a1, float* p2,
                   const float* dq, float* grads, float* dh, int accumulate, float* workspace, vn_stream_t stream);
/* reward_prediction (goal.py:121-129): out [n][4] = logits of x [n][3 * FCIN] (column 3 unused). */
int vn_rp_forward(vn_policy* p, const float* params, const float* x, int n, float* out, vn_stream_t stream);
/* rp gradients into grads (overwritten) from dL/dout [n][4] (column 3 ignored); dx [n][3 * FCIN]
 * (may be NULL) = dout x W. workspace: vn_pc_workspace_floats. */
int vn_rp_backward(vn_policy* p, const float* params, const float* x, int n, const float* dout, float* grads,
                   float* dx, float* workspace, vn_stream_t stream);
/* ---- UNREAL losses of the trainer (deep_rl's UnrealTrainer, absent: parity unpinned; the
 * published algorithm, csrc/vn_unreal_loss.hip, weights experiments/thor_cached_auxiliary.py:39-41) ----
 * Sequences are the first S envs of a rollout of T steps x E envs (rows t*E + e).
 * Pixel control: p2 [(T+1)*S][42][42][8] from vn_pc_forward on rows t*S + e (row T*S + e: the
 * bootstrap observation), q = (v + a) - a formed from it; pseudo-reward r_t = mean over each
 * 4x4 cell and 3 channels of |obs_{t+1} - obs_t| / 255 on the centre 168x168 crop of the u8
 * image frames (arena rows rows_img[t*E + e], rows_last[e] for obs_T); R_T = max_a q_T,
 * R_t = r_t + gamma (1 - done_t) R_{t+1} with r_t = 0 on a done step (the next frame is the
 * auto-reset frame of the next episode: recorded deviation); p2 is overwritten by dL/dp2 of weight *
 * mean((q_t[a_t] - R_t)^2) (under the value ReLU; 0 on the bootstrap rows), ready for
 * vn_pc_backward with dq == NULL; stats[0] += sum of squared errors. */
int vn_unreal_pc_loss_grad(float* p2, const int32_t* actions, const uint8_t* dones, const uint8_t* arena,
                           int64_t frame_bytes, int height, int width, const int32_t* rows_img,
                           const int32_t* rows_last, int T, int E, int S, int num_actions, float gamma, float weight,
                           float* stats, vn_stream_t stream);
/* The same on a cells x cells map: 42 (above) or 20 (BigHouseModel's p2 [(T+1)*S][20][20][8],
 * the centre 80x80 crop of 84x84 frames). */
int vn_unreal_pc_loss_grad_ex(float* p2, int cells, const int32_t* actions, const uint8_t* dones,
                              const uint8_t* arena, int64_t frame_bytes, int height, int width,
                              const int32_t* rows_img, const int32_t* rows_last, int T, int E, int S, int num_actions,
                              float gamma, float weight, float* stats, vn_stream_t stream);
/* Reward prediction: logits [(T-2)*S][4] of samples j = (ts-2)*S + e (frames ts-2..ts of env
 * e); class of rewards[ts][e]: 0 (r = 0), 1 (r > 0), 2 (r < 0); samples with a done at ts-2
 * or ts-1 are skipped. dlogits = weight * d mean CE / dlogits; stats2 = (mean CE, count). */
int vn_unreal_rp_loss_grad(const float* logits, const float* rewards, const uint8_t* dones, int T, int E, int S,
                           float weight, float* dlogits, float* stats2, vn_stream_t stream);
/* dx [(T-2)*S][3][fcin] (vn_rp_backward's input gradient) onto dx4 rows t*E + e, e < S
 * (stored, or added when accumulate != 0; other rows untouched). */
int vn_unreal_rp_scatter(const float* dx, int T, int E, int S, int fcin, float* dx4, int accumulate,
                         vn_stream_t stream);
/* The losses' inputs in one launch: h_pc [(T+1)*S][512] = h_all rows t*E + e (t < T, e < S)
 * then boot_h rows e < S; rp_x [(T-2)*S][3][fcin] (may be NULL) slot k of sample t*S + e =
 * x4 row (t+k)*E + e (conv_base maps of frames t..t+2). h_pc == NULL (h_all / boot_h unused) gathers
 * only rp_x. */
int vn_unreal_gather(const float* h_all, const float* boot_h, const float* x4, int T, int E, int S, int fcin,
                     float* h_pc, float* rp_x, vn_stream_t stream);
/* Value replay on rows t*E + e, e < S: dout[.][A] += weight * d mean((V - R)^2) / dV;
 * stats[0] += sum of squared errors. */
int vn_unreal_vr_grad(const float* out, const float* returns, int T, int E, int S, int num_actions, float weight,
                      float* dout, float* stats, vn_stream_t stream);

/* General backward: from dL/d(out) [n][8] (dz5 == NULL) or from dz5 [n][512] (recurrent
 * policies, heads and LSTM done by vn_lstm_backward); dx4_extra [n][h3][w3][32] (aux heads,
 * may be NULL) is added to conv_base's output gradient under its ReLU mask. */
int vn_policy_backward_ex(vn_policy* p, const float* params, const vn_frames* frames, int n, float* acts,
                          int64_t act_capacity, const float* dout, const float* dz5, const float* dx4_extra,
                          float* grads, float* workspace, vn_stream_t stream);

/* ---- goal-frame deduplication: shared_base on the goal frame once per episode ----
 * BigGoalHouseModel runs shared_base on the goal frame at every step (models/goal.py:88), but
 * an env's goal frame does not change within an episode. A goal run is a sample whose goal is
 * new — the first step of a rollout, or the step after a done (the env auto-reset) — followed
 * by the same env's later steps up to its next done. With goal runs the policy computes conv1 /
 * conv2 of a goal frame only at the run's first sample, conv_base reads every sample's goal
 * map from its run start, and the backward sums a run's goal-map gradients before conv2's
 * weight / input gradient and conv1's weight gradient: the same outputs (bitwise: the
 * kernels are batch-independent) and the same gradients up to summation order. Samples are
 * time-major (t*E + e). */
typedef struct vn_goal_runs {
  const int32_t* goal_list;   /* samples (of the call) that start a goal run, ascending */
  const int32_t* goal_count;  /* device scalar: entries of goal_list */
  const int32_t* goal_delta;  /* [n] offset (<= 0, in samples) to the sample holding this sample's goal maps */
  const int32_t* run_length;  /* backward: [n] steps of the run starting at each listed sample */
  int num_envs;               /* backward: E, the sample stride between an env's steps */
} vn_goal_runs;
/* *supported = 1 when the policy takes goal runs for calls of n samples (84x84 / 174x174
 * uint8 frames, n > 16, no VN_*_GENERIC override set); else 0. */
int vn_policy_goal_runs_supported(vn_policy* p, int n, int* supported);
/* vn_policy_forward with the goal runs of this call's n samples (goals != NULL; an unsupported
 * configuration is an error, not a silent fallback). */
int vn_policy_forward_goals(vn_policy* p, const float* params, const vn_frames* frames, int n, float* acts,
                            int64_t act_capacity, int64_t act_offset, float* out, const vn_goal_runs* goals,
                            vn_stream_t stream);
/* vn_policy_backward_ex over samples whose forward ran with these goal runs (the goal maps
 * of non-start samples were never computed: a backward without the runs would read them). */
int vn_policy_backward_goals(vn_policy* p, const float* params, const vn_frames* frames, int n, float* acts,
                             int64_t act_capacity, const float* dout, const float* dz5, const float* dx4_extra,
                             float* grads, float* workspace, const vn_goal_runs* goals, vn_stream_t stream);
/* Rollout step t's goal runs (before its forward): new[e] = done_prev == NULL || done_prev[e]
 * (done_prev = step t - 1's dones; NULL at t = 0); delta[e] = new ? 0 : delta_prev[e] - E;
 * list = the envs with new goals, ascending; *count = their number. One workgroup. */
int vn_goal_runs_step(const uint8_t* done_prev, const int32_t* delta_prev, int E, int32_t* delta, int32_t* list,
                      int32_t* count, vn_stream_t stream);
/* The update's goal runs over the rollout's T*E samples (dones [T][E]): list = the run starts
 * ascending, run_length [T*E] at each start, *count. One workgroup. */
int vn_goal_runs_rollout(const uint8_t* dones, int T, int E, int32_t* list, int32_t* run_length, int32_t* count,
                         vn_stream_t stream);

/* ---- A2C (the deep_rl trainer contract; DESIGN.md "A2C contract") ---- */
int vn_policy_sample(const float* out, int n, int num_actions, uint64_t seed, uint64_t counter,
                     int32_t* actions, float* logp, float* entropy, float* value, vn_stream_t stream);
int vn_policy_greedy(const float* out, int n, int num_actions, int32_t* actions, vn_stream_t stream);
int vn_a2c_returns(const float* rewards, const uint8_t* dones, const float* bootstrap_out, int T, int E,
                   int num_actions, float gamma, float* returns, vn_stream_t stream);
int vn_a2c_loss_grad(const float* out, const int32_t* actions, const float* returns, int n,
                     int num_actions, float value_coef, float entropy_coef, float* dout,
                     float* stats4, vn_stream_t stream);
/* Rollout bookkeeping after env step t (one launch): the next step's recurrent inputs —
 * last action one-hot and last reward times the episode mask m = 1 - done, and m itself
 * (UnrealEnvBaseWrapper's extra input, models/goal.py:63-64; mask rule of MaskedRNN,
 * unpinned) into lra_next [E][A+1] / mask_next [E] — prev_* carries, and the finished
 * episodes' (count, return sum, length sum) added to episode_stats3 in a fixed order
 * (deep_rl RewardCollector, experiments/thor_cached_auxiliary.py:59-64). Pointers other
 * than the inputs and episode_stats3 may be NULL. */
int vn_a2c_step_post(const int32_t* actions, const float* rewards, const uint8_t* dones,
                     const float* ep_return, const int32_t* ep_length, int E, int num_actions,
                     int64_t* prev_action, float* prev_reward, float* prev_mask, float* lra_next,
                     float* mask_next, float* episode_stats3, vn_stream_t stream);
/* stats3 = the fixed-order sums over envs of episode_stats_env [3][E] (vn_step_a2c's
 * accumulators: finished-episode count, return sum, length sum), which are then zeroed. */
int vn_a2c_episode_stats(float* episode_stats_env, int E, float* stats3, vn_stream_t stream);
/* scalars2 = (total norm of scale*grads, clip coefficient) computed on the device. */
int vn_grad_norm(const float* grads, int64_t n, float scale, float max_norm, double* partial_512,
                 float* scalars2, vn_stream_t stream);
int vn_rmsprop_step(float* params, const float* grads, float* square_avg, int64_t n, float scale,
                    const float* scalars2, float lr, float alpha, float eps, vn_stream_t stream);
/* vn_grad_norm with up to two gradient addends joined first: grads[i] += add_j[i] for i in
 * [lo_j, hi_j) (add_j NULL = none), written back to grads, then the norm of scale*grads —
 * the side passes' sums (a replayed aux batch's trunk gradient, the replayed UNREAL pass's
 * trunk / heads / LSTM gradient) without a launch of their own; bitwise equal to the adds
 * followed by vn_grad_norm. */
int vn_grad_norm_join(float* grads, int64_t n, const float* add0, int64_t lo0, int64_t hi0, const float* add1,
                      int64_t lo1, int64_t hi1, float scale, float max_norm, double* partial_512,
                      float* scalars2, vn_stream_t stream);

/* The replay ring on the device (deep_rl's replay buffer behind AuxiliaryTrainer's
 * self.replay.sample_sequence(), experiments/ai2_auxiliary/trainer.py:27-31; deep_rl is
 * absent, so capacity and sequence shape are parity unpinned). One call pushes a rollout's
 * record into slot meta4[0] and draws this update's slot among the filled ones — no host
 * value, so an update with replay sources is captured in a hipGraph (A2CTrainer(cuda_graph=True)).
 * meta4 = int64 [next slot, filled slots, draw counter, last drawn slot]. Segment j copies
 * rows x cols elements of elem_bytes (1 or 4) from src (row r at src + r*src_ld elements) to
 * ring + slot*slot_elems (packed rows) and, when cur != NULL, the drawn slot's elements to cur
 * (packed). The draw: k = uniform_below(Philox4x32-10(ctr_lo, ctr_hi, 0, STREAM_REPLAY = 4)
 * under key seed, min(filled + 1, capacity)); then meta4 = [(slot + 1) % capacity,
 * min(filled + 1, capacity), ctr + 1, k]. At most 16 segments. */
typedef struct vn_replay_seg {
  const void* src;
  int64_t src_ld;
  void* ring;
  void* cur;
  int64_t slot_elems;
  int32_t rows, cols, elem_bytes, pad_;
} vn_replay_seg;
int vn_replay_push_draw(const vn_replay_seg* segs, int nseg, int64_t* meta4, int capacity, uint64_t seed,
                        vn_stream_t stream);

/* Device-side schedule, so that one update has no per-call host arguments and can be
 * captured once in a hipGraph and replayed (A2CTrainer(cuda_graph=True)):
 *   vn_a2c_schedule: state3 = int64 [next counter base, env-steps so far, this update's
 *     counter base]; this update's base = state3[0] (then += T), lr_out = lr0 * (1 -
 *     min(state3[1] / max_time_steps, 1)) computed in double (LinearSchedule,
 *     experiments/thor_cached_auxiliary.py:37), then state3[1] += steps_per_update;
 *   vn_policy_sample_dev: vn_policy_sample with counter = *counter_base_dev + offset;
 *   vn_rmsprop_step_dev: vn_rmsprop_step with lr read from lr_dev.
 * Bit-identical to the host-argument forms fed the same values. */
int vn_a2c_schedule(int64_t* state3, float* lr_out, double lr0, double max_time_steps,
                    int64_t steps_per_update, int T, vn_stream_t stream);
/* First launch of a rollout (replaces vn_a2c_schedule + the step-0 input copies):
 * vn_a2c_schedule's update of state3 / lr_out, img/goal_row_dst[e] = *_src[e] (step 0's
 * frame rows) and, when mask0 != NULL, mask0[e] = prev_mask[e] and lra0 [E][A+1] =
 * [one_hot(prev_action[e]) | prev_reward[e]] * prev_mask[e] (vn_a2c_step_post's form). */
int vn_a2c_rollout_begin(int64_t* state3, float* lr_out, double lr0, double max_time_steps,
                         int64_t steps_per_update, int T, const int32_t* img_row_src,
                         const int32_t* goal_row_src, int32_t* img_row_dst, int32_t* goal_row_dst, int E,
                         const int64_t* prev_action, const float* prev_reward, const float* prev_mask,
                         int num_actions, float* mask0, float* lra0, vn_stream_t stream);
/* An update's metric vector out9 = [stats4 * inv_n, scalars2[0] (grad norm), aux loss =
 * sum over the three heads of aux3[h] / aux_numel3[h] (0 when aux3 == NULL), episode_stats3]
 * in one launch. */
int vn_a2c_metrics(const float* stats4, float inv_n, const float* scalars2, const float* aux3,
                   const float* aux_numel3, const float* episode_stats3, float* out9, vn_stream_t stream);
/* vn_a2c_metrics + the UNREAL loss means: out[9..11] = [unreal4[0] * norm3[0] (pc),
 * unreal4[1] * norm3[1] (rp), unreal4[3] * norm3[2] (vr)] when unreal4 != NULL (out holds 12). */
int vn_a2c_metrics_ex(const float* stats4, float inv_n, const float* scalars2, const float* aux3,
                      const float* aux_numel3, const float* episode_stats3, const float* unreal4,
                      const float* unreal_norm3, float* out, vn_stream_t stream);
int vn_policy_sample_dev(const float* out, int n, int num_actions, uint64_t seed,
                         const int64_t* counter_base_dev, uint64_t counter_offset, int32_t* actions,
                         float* logp, float* entropy, float* value, vn_stream_t stream);
int vn_rmsprop_step_dev(float* params, const float* grads, float* square_avg, int64_t n, float scale,
                        const float* scalars2, const float* lr_dev, float alpha, float eps,
                        vn_stream_t stream);

/* Copy the message of the calling thread's last error (NUL-terminated). */
int vn_last_error(char* buf, size_t len);
const char* vn_version(void);

/* Diagnostics: launch an empty kernel of `tag` (1..65535) workgroups of 64 lanes on the
 * stream. A kernel trace records its grid size, which marks where a test (or any phase of
 * a program) begins in a trace (tests/conftest.py, tools/test_kernel_map.py). */
int vn_trace_marker(int tag, vn_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* VNAV_H */
