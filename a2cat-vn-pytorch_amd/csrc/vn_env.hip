// vn_env.hip — batched cached-scene env.step for gfx950 (CDNA4).
//
// Semantics restate THORDiscreteCachedEnv (environments/gym_ai2thor/envs/cached.py):
//   transition  nxt = graph[s][a]; -1 = blocked                     (cached.py:74-79)
//   terminal    goal == state                                        (cached.py:83)
//   reward      -reward_configuration[1], goal -> [0], blocked -> [2] (cached.py:84-88)
//   obs         (frame[s], frame[g]), or the previous obs on terminal (cached.py:90-98)
//   reset       goal ~ U[0,N), start ~ U[0,N) until spd[start][goal] > 0 (cached.py:38-45)
// batched the way deep_rl's SubprocVecEnv drives it (auto-reset on done, the reset
// observation replaces the terminal one) under gym's TimeLimit(900).
//
// Design (DESIGN.md "vn_step"): one wave64 per env, 4 envs per 256-thread workgroup.
// The per-env state is wave-uniform (scalar loads); a reset runs 64 Philox start
// candidates in parallel, one per lane, and a wave ballot picks the first valid one —
// the same result as the sequential rejection loop over the same counter stream.
// The two frames are then streamed with 16-B lanes, 8 loads in flight per lane.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "vn_common.h"

namespace vn {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}
int hip_fail(hipError_t e, const char* what) {
  set_error(std::string(what) + ": " + hipGetErrorString(e));
  return VN_EHIP;
}
const std::string& last_error() { return g_last_error; }

struct SceneDev {
  int64_t row_base;  // first arena row (frame) of the scene
  int64_t spd_off;   // element offset of the scene's [N][N] spd block (and curriculum order block)
  int64_t cnt_off;   // element offset of the scene's [N][maxd+2] curriculum count block
  int64_t comp_base; // first arena row of the scene's companion frames, -1 = second output is the goal frame
  int32_t graph_off; // first row of the scene's [N][4] adjacency block
  int32_t n;         // states
  int32_t maxd;      // largest spd value of the scene
  int32_t cur_oi;    // curriculum threshold floor(c*(maxd+offset)+1) clamped to [0, maxd] (host, fp64)
  int32_t cur_mode;  // 0 off, 1 uniform over 0 < spd <= opt, 2 0.9 / 0.1 split (graph/util.py:88-117)
  float r_goal, r_step, r_coll;
  int32_t terminal_obs;
};

enum { ST_SCENE = 0, ST_STATE, ST_GOAL, ST_OBS, ST_ELAPSED, ST_EPISODE, ST_SCHED, ST_COUNT };

struct EnvArgs {
  const SceneDev* scenes;
  const int32_t* graph;
  const int32_t* spd;
  const uint8_t* arena;
  int64_t frame_bytes;
  int32_t* st;  // [ST_COUNT][n_envs]
  float* ep_ret;
  const int32_t* env_scene;
  const int32_t* tasks;
  const int32_t* sched;
  const int32_t* cur_order;  // per scene, per goal: states sorted by spd[s][g] (stable)
  const int32_t* cur_count;  // per scene, per goal: #states with clamp(spd,-1,maxd)+1 <= b
  uint32_t* flags;
  int n_tasks, sched_len, max_steps, autoreset, n_envs;
  int cur_mode;  // any scene with a curriculum (the per-scene mode is SceneDev::cur_mode)
  uint32_t k0, k1;
  // per call
  const int32_t* actions;
  const int32_t* mask;
  uint8_t* obs;
  uint8_t* goal_out;
  float* reward;
  uint8_t* done;
  int32_t* state_out;
  float* info_ret;
  int32_t* info_len;
  int32_t* info_term;
  uint8_t* info_trunc;
  int32_t* info_img_row;
  int32_t* info_goal_row;
  // vn_step_a2c: action sampled in the step, then the rollout's per-step bookkeeping
  const float* pol_out;
  int pol_A;
  uint32_t pk0, pk1;
  const int64_t* pctr_dev;
  uint64_t pctr;
  int32_t* act_out;
  int64_t* prev_action;
  float* prev_reward;
  float* prev_mask;
  float* lra_next;
  float* mask_next;
  float* stats_env;
  const float* head_w;  // optional: heads computed here (vn_a2c_step.head_weight)
  const float* head_b;
  const float* head_x;
  float* head_out;
};

// MODE_STEP_HEADS: a step of vn_step_a2c that also computes the policy heads (its own
// instantiation, so the plain step keeps its register budget)
enum { MODE_STEP = 0, MODE_RESET = 1, MODE_OBSERVE = 2, MODE_STEP_HEADS = 3 };
constexpr int kEnvsPerBlock = 4;
constexpr int kStartRounds = 16;  // 1024 rejection attempts before flagging

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Wave-cooperative reset of env e (all 64 lanes call with uniform arguments).
__device__ void reset_env(const EnvArgs& a, int e, int lane, int& sc, int& s, int& g) {
  const int n_envs = a.n_envs;
  const int k = a.st[ST_EPISODE * n_envs + e];
  const int sp = a.st[ST_SCHED * n_envs + e];
  if (a.sched_len > 0 && sp < a.sched_len) {
    sc = a.env_scene[e];
    const int n = a.scenes[sc].n;
    s = a.sched[((int64_t)e * a.sched_len + sp) * 2 + 0];
    g = a.sched[((int64_t)e * a.sched_len + sp) * 2 + 1];
    if ((unsigned)s >= (unsigned)n || (unsigned)g >= (unsigned)n) {
      if (lane == 0) atomicOr(a.flags, (uint32_t)VN_FLAG_BAD_SCHEDULE);
      s = min(max(s, 0), n - 1);
      g = min(max(g, 0), n - 1);
    }
    if (lane == 0) a.st[ST_SCHED * n_envs + e] = sp + 1;
    return;
  }
  const u32x4 rg = philox4x32_10(u32x4{(uint32_t)e, (uint32_t)k, 0u, STREAM_GOAL}, a.k0, a.k1);
  if (a.n_tasks > 0) {
    const int t = (int)uniform_below(rg.x, (uint32_t)a.n_tasks);
    sc = a.tasks[2 * t];
    g = a.tasks[2 * t + 1];
    if (g < 0) g = (int)uniform_below(rg.y, (uint32_t)a.scenes[sc].n);
  } else {
    sc = a.env_scene[e];
    g = (int)uniform_below(rg.x, (uint32_t)a.scenes[sc].n);
  }
  const SceneDev S = a.scenes[sc];
  const int32_t* spd = a.spd + S.spd_off;
  s = -1;
  if (a.cur_mode > 0 && S.cur_mode > 0) {
    // curriculum (graph/util.py:88-143, environments/gym_graph/graph.py:43-52):
    // opt = c * (maxd + offset) + 1 (S.cur_oi = its floor); candidates 0 < spd <= opt, uniform (mode 1) or
    // 0.9 over them / 0.1 over the farther ones (mode 2); one O(1) draw from the sorted table
    const int oi = S.cur_oi;
    const int32_t* cnt = a.cur_count + S.cnt_off + (int64_t)g * (S.maxd + 2);
    const int lo = cnt[1], hi = cnt[oi + 1], n = S.n;
    const u32x4 r = philox4x32_10(u32x4{(uint32_t)e, (uint32_t)k, 0u, STREAM_START}, a.k0, a.k1);
    // far set when the 0.1 coin says so (and it is not empty) or when the near set is empty
    const bool use_far = (S.cur_mode == 2 && r.y >= 3865470566u && hi < n) || hi <= lo;  // 0.9 * 2^32
    const int b0 = use_far ? hi : lo, b1 = use_far ? n : hi;
    if (b1 > b0) s = a.cur_order[S.spd_off + (int64_t)g * n + b0 + (int)uniform_below(r.x, (uint32_t)(b1 - b0))];
  }
  for (int round = 0; round < kStartRounds && s < 0; ++round) {
    const uint32_t att = (uint32_t)(round * 64 + lane);
    const u32x4 r = philox4x32_10(u32x4{(uint32_t)e, (uint32_t)k, att, STREAM_START}, a.k0, a.k1);
    const int cand = (int)uniform_below(r.x, (uint32_t)S.n);
    const bool ok = spd[(int64_t)cand * S.n + g] > 0;
    const unsigned long long m = __ballot(ok);
    if (m) {
      s = __shfl(cand, __ffsll((long long)m) - 1);
      break;
    }
  }
  if (s < 0) {  // bounded search exhausted: flag and take attempt 0
    if (lane == 0) atomicOr(a.flags, (uint32_t)VN_FLAG_RESET_EXHAUSTED);
    const u32x4 r = philox4x32_10(u32x4{(uint32_t)e, (uint32_t)k, 0u, STREAM_START}, a.k0, a.k1);
    s = (int)uniform_below(r.x, (uint32_t)S.n);
  }
  s = uni(s);
}

// Copy the image frame and goal frame of one env: 16-B lanes, 4 x 2 loads in flight. The
// output rows are written with nontemporal (`nt`) stores; loads keep the default policy.
// Measured (tools/copybench.hip cache-policy sweep over the 16 load/store combinations, and
// the bench, tools/ab/copy_variants.sh): at 4096 envs default stores 57-60 us, any single nt
// stream 54-56 us; at 32768 envs per GPU nt on both stores 446 us (6.2 TB/s) vs 551 us
// default and 545-563 us with nt loads; nt on all four streams is the slowest everywhere.
__device__ __forceinline__ void st16_nt(uint4* p, const uint4 v) {
  __builtin_nontemporal_store(v.x, &p->x);
  __builtin_nontemporal_store(v.y, &p->y);
  __builtin_nontemporal_store(v.z, &p->z);
  __builtin_nontemporal_store(v.w, &p->w);
}

template <int VEC>
__device__ __forceinline__ void copy_two_frames(uint8_t* __restrict__ d1, const uint8_t* __restrict__ s1,
                                                uint8_t* __restrict__ d2, const uint8_t* __restrict__ s2,
                                                int64_t bytes, int lane) {
  if constexpr (VEC == 16) {
    constexpr int U = 4;
    const int n = (int)(bytes >> 4);
    const uint4* a = reinterpret_cast<const uint4*>(s1);
    const uint4* b = reinterpret_cast<const uint4*>(s2);
    uint4* x = reinterpret_cast<uint4*>(d1);
    uint4* y = reinterpret_cast<uint4*>(d2);
    int i = lane;
    for (; i + 64 * (U - 1) < n; i += 64 * U) {
      uint4 va[U], vb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) va[u] = a[i + 64 * u];
#pragma unroll
      for (int u = 0; u < U; ++u) vb[u] = b[i + 64 * u];
#pragma unroll
      for (int u = 0; u < U; ++u) st16_nt(x + i + 64 * u, va[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) st16_nt(y + i + 64 * u, vb[u]);
    }
    for (; i < n; i += 64) {
      const uint4 a0 = a[i], b0 = b[i];
      st16_nt(x + i, a0);
      st16_nt(y + i, b0);
    }
  } else if constexpr (VEC == 4) {
    const int n = (int)(bytes >> 2);
    const uint32_t* a = reinterpret_cast<const uint32_t*>(s1);
    const uint32_t* b = reinterpret_cast<const uint32_t*>(s2);
    uint32_t* x = reinterpret_cast<uint32_t*>(d1);
    uint32_t* y = reinterpret_cast<uint32_t*>(d2);
    for (int i = lane; i < n; i += 64) {
      const uint32_t a0 = a[i], b0 = b[i];
      x[i] = a0;
      y[i] = b0;
    }
  } else {
    for (int64_t i = lane; i < bytes; i += 64) {
      d1[i] = s1[i];
      d2[i] = s2[i];
    }
  }
}

template <int MODE, int VEC>
__global__ __launch_bounds__(256) void env_kernel(EnvArgs a) {
  const int lane = threadIdx.x & 63;
  const int e = uni(blockIdx.x * kEnvsPerBlock + (threadIdx.x >> 6));
  if (e >= a.n_envs) return;
  const int n_envs = a.n_envs;
  int32_t* st = a.st;

  int sc = st[ST_SCENE * n_envs + e];
  int s = st[ST_STATE * n_envs + e];
  int g = st[ST_GOAL * n_envs + e];
  int os = st[ST_OBS * n_envs + e];

  if constexpr (MODE == MODE_STEP || MODE == MODE_STEP_HEADS) {
    int t = st[ST_ELAPSED * n_envs + e];
    const SceneDev S = a.scenes[sc];
    int act;
    if (a.pol_out) {  // the policy's categorical draw for this env (vn_policy_sample_dev's)
      float lg[7], p[7], lp[7], H;
      if constexpr (MODE == MODE_STEP_HEADS) {
        // the heads of this env (logits, value): vn_policy_heads' skinny product for one row —
        // 32 lanes, 4 consecutive k at 4 kl + 128 i, fma chains, a 32-lane xor tree, + bias:
        // the same sums in the same order (both 32-lane halves compute them)
        const int kl = lane & 31;
        const float* x = a.head_x + (int64_t)e * 512;
        float4 xv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) xv[i] = *reinterpret_cast<const float4*>(x + 4 * kl + 128 * i);
        float sj[8], bj[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) bj[j] = a.head_b[min(j, a.pol_A)];
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // all rows' loads in flight together (A + 1 <= 8)
          const float* w = a.head_w + (int64_t)min(j, a.pol_A) * 512;
          float s = 0.0f;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float4 wv = *reinterpret_cast<const float4*>(w + 4 * kl + 128 * i);
            s = fmaf(xv[i].x, wv.x, s);
            s = fmaf(xv[i].y, wv.y, s);
            s = fmaf(xv[i].z, wv.z, s);
            s = fmaf(xv[i].w, wv.w, s);
          }
          sj[j] = s;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
          for (int o = 16; o > 0; o >>= 1) sj[j] += __shfl_xor(sj[j], o, 32);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (j <= a.pol_A) {
            const float v = sj[j] + bj[j];
            if (j < a.pol_A) lg[j] = v;
            if (lane == 0) a.head_out[(int64_t)e * 8 + j] = v;
          }
        }
      } else {
        for (int j = 0; j < a.pol_A; ++j) lg[j] = a.pol_out[(int64_t)e * 8 + j];
      }
      const uint64_t ctr = a.pctr + (a.pctr_dev ? (uint64_t)*a.pctr_dev : 0ull);
      act = uni(sample_action(lg, a.pol_A, a.pk0, a.pk1, ctr, (uint32_t)e, p, lp, H));
    } else {
      act = a.actions[e];
    }
    const bool bad = (unsigned)act > 3u;
    int nxt = -1;
    if (!bad) nxt = a.graph[((int64_t)S.graph_off + s) * 4 + act];
    const bool collided = nxt == -1;
    if (!collided) s = nxt;
    const bool terminal = (s == g);
    float r = S.r_step;
    if (terminal) r = S.r_goal;
    if (collided) r = S.r_coll;
    if (!terminal || S.terminal_obs) os = s;
    t += 1;
    const bool limit = a.max_steps > 0 && t >= a.max_steps;
    const bool done = terminal || limit;
    const float ret = a.ep_ret[e] + r;
    const int term_state = os;
    const int ep_len = t;
    float new_ret = ret;
    if (done && a.autoreset) {
      reset_env(a, e, lane, sc, s, g);
      os = s;
      t = 0;
      new_ret = 0.0f;
    }
    if (lane == 0) {
      st[ST_SCENE * n_envs + e] = sc;
      st[ST_STATE * n_envs + e] = s;
      st[ST_GOAL * n_envs + e] = g;
      st[ST_OBS * n_envs + e] = os;
      st[ST_ELAPSED * n_envs + e] = t;
      if (done && a.autoreset) st[ST_EPISODE * n_envs + e] += 1;
      a.ep_ret[e] = new_ret;
      if (bad) atomicOr(a.flags, (uint32_t)VN_FLAG_BAD_ACTION);
      if (a.reward) a.reward[e] = r;
      if (a.done) a.done[e] = done ? 1 : 0;
      if (a.state_out) a.state_out[e] = s;
      if (a.info_ret) a.info_ret[e] = ret;
      if (a.info_len) a.info_len[e] = ep_len;
      if (a.info_term) a.info_term[e] = term_state;
      if (a.info_trunc) a.info_trunc[e] = (limit && !terminal) ? 1 : 0;
      if (a.pol_out) {  // vn_a2c_step_post's bookkeeping for this env
        const float m = done ? 0.0f : 1.0f;
        a.act_out[e] = act;
        if (a.prev_action) a.prev_action[e] = act;
        if (a.prev_reward) a.prev_reward[e] = r;
        if (a.prev_mask) a.prev_mask[e] = m;
        if (a.mask_next) a.mask_next[e] = m;
        if (a.lra_next) {
          for (int j = 0; j < a.pol_A; ++j) a.lra_next[(int64_t)e * (a.pol_A + 1) + j] = j == act ? m : 0.0f;
          a.lra_next[(int64_t)e * (a.pol_A + 1) + a.pol_A] = r * m;
        }
        if (a.stats_env && done) {
          a.stats_env[e] += 1.0f;
          a.stats_env[n_envs + e] += ret;
          a.stats_env[2 * (int64_t)n_envs + e] += (float)ep_len;
        }
      }
    }
  } else if constexpr (MODE == MODE_RESET) {
    if (a.mask == nullptr || a.mask[e] != 0) {
      reset_env(a, e, lane, sc, s, g);
      os = s;
      if (lane == 0) {
        st[ST_SCENE * n_envs + e] = sc;
        st[ST_STATE * n_envs + e] = s;
        st[ST_GOAL * n_envs + e] = g;
        st[ST_OBS * n_envs + e] = os;
        st[ST_ELAPSED * n_envs + e] = 0;
        st[ST_EPISODE * n_envs + e] += 1;
        a.ep_ret[e] = 0.0f;
      }
    }
    return;
  } else {
    if (lane == 0 && a.state_out) a.state_out[e] = s;
  }

  const int64_t base = a.scenes[sc].row_base, comp = a.scenes[sc].comp_base;
  const int64_t img_row = base + os, goal_row = comp >= 0 ? comp + os : base + g;
  if (lane == 0) {
    if (a.info_img_row) a.info_img_row[e] = (int32_t)img_row;
    if (a.info_goal_row) a.info_goal_row[e] = (int32_t)goal_row;
  }
  if (a.obs != nullptr && a.goal_out != nullptr) {
    const int64_t F = a.frame_bytes;
    copy_two_frames<VEC>(a.obs + (int64_t)e * F, a.arena + img_row * F, a.goal_out + (int64_t)e * F,
                         a.arena + goal_row * F, F, lane);
  } else if (a.obs != nullptr || a.goal_out != nullptr) {
    const int64_t F = a.frame_bytes;
    uint8_t* d = a.obs ? a.obs + (int64_t)e * F : a.goal_out + (int64_t)e * F;
    const uint8_t* src = a.arena + (a.obs ? img_row : goal_row) * F;
    for (int64_t i = lane; i < F; i += 64) d[i] = src[i];
  }
}

__global__ void synth_frames_kernel(uint8_t* arena, int64_t row_base, int n_rows, int64_t frame_bytes,
                                    uint32_t scene_id) {
  const int64_t words = frame_bytes >> 2;
  const int64_t total = words * n_rows;
  uint32_t* dst = reinterpret_cast<uint32_t*>(arena + row_base * frame_bytes);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / words, w = i - row * words;
    dst[i] = frame_hash(scene_id, (uint32_t)row, (uint32_t)w);
  }
}

// dst[i] = src[rows[i]] for rows of row_bytes (one wave per row, 16-B lanes when aligned).
__global__ __launch_bounds__(256) void gather_rows_kernel(const uint8_t* __restrict__ src, int64_t row_bytes,
                                                          const int32_t* __restrict__ rows, int n,
                                                          uint8_t* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  const int i = uni(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (i >= n) return;
  const uint8_t* s = src + (int64_t)rows[i] * row_bytes;
  uint8_t* d = dst + (int64_t)i * row_bytes;
  if ((row_bytes & 15) == 0) {
    const uint4* a = reinterpret_cast<const uint4*>(s);
    uint4* b = reinterpret_cast<uint4*>(d);
    for (int64_t j = lane; j < (row_bytes >> 4); j += 64) b[j] = a[j];
  } else {
    for (int64_t j = lane; j < row_bytes; j += 64) d[j] = s[j];
  }
}

__global__ void random_actions_kernel(int32_t* actions, int n, uint32_t k0, uint32_t k1, uint64_t step) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const u32x4 r = philox4x32_10(u32x4{(uint32_t)e, (uint32_t)step, (uint32_t)(step >> 32), STREAM_ACTION}, k0, k1);
  actions[e] = (int32_t)(r.x >> 30);
}

}  // namespace vn

using namespace vn;

struct vn_ctx {
  int device = 0;
  int n_envs = 0, n_scenes = 0;
  uint64_t seed = 0;
  int64_t frame_bytes = 0, n_rows = 0;
  uint8_t* arena = nullptr;
  int32_t* graph = nullptr;
  int32_t* spd = nullptr;
  SceneDev* scenes = nullptr;
  std::vector<SceneDev> scenes_host;
  int32_t* st = nullptr;
  float* ep_ret = nullptr;
  int32_t* env_scene = nullptr;
  int32_t* tasks = nullptr;
  int n_tasks = 0;
  int32_t* sched = nullptr;
  int sched_len = 0;
  std::vector<int32_t> spd_host;  // kept for building curriculum tables on demand
  int32_t* cur_order = nullptr;
  int32_t* cur_count = nullptr;
  int cur_mode = 0;
  double cur_c = 0.0;
  uint32_t* flags = nullptr;
  int max_steps = 900, autoreset = 1;
  float* info_ret = nullptr;
  int32_t* info_len = nullptr;
  int32_t* info_term = nullptr;
  uint8_t* info_trunc = nullptr;
  int32_t* info_img_row = nullptr;
  int32_t* info_goal_row = nullptr;
};

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(d);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

EnvArgs make_args(vn_ctx* c) {
  EnvArgs a;
  std::memset(&a, 0, sizeof(a));
  a.scenes = c->scenes;
  a.graph = c->graph;
  a.spd = c->spd;
  a.arena = c->arena;
  a.frame_bytes = c->frame_bytes;
  a.st = c->st;
  a.ep_ret = c->ep_ret;
  a.env_scene = c->env_scene;
  a.tasks = c->tasks;
  a.sched = c->sched;
  a.cur_order = c->cur_order;
  a.cur_count = c->cur_count;
  a.cur_mode = c->cur_mode;
  a.flags = c->flags;
  a.n_tasks = c->n_tasks;
  a.sched_len = c->sched_len;
  a.max_steps = c->max_steps;
  a.autoreset = c->autoreset;
  a.n_envs = c->n_envs;
  a.k0 = (uint32_t)c->seed;
  a.k1 = (uint32_t)(c->seed >> 32);
  a.info_ret = c->info_ret;
  a.info_len = c->info_len;
  a.info_term = c->info_term;
  a.info_trunc = c->info_trunc;
  a.info_img_row = c->info_img_row;
  a.info_goal_row = c->info_goal_row;
  return a;
}

template <int MODE>
int launch_env(vn_ctx* c, const EnvArgs& a, hipStream_t stream) {
  const dim3 grid((c->n_envs + kEnvsPerBlock - 1) / kEnvsPerBlock), block(64 * kEnvsPerBlock);
  const int64_t F = c->frame_bytes;
  const bool al16 = (F % 16 == 0) && ((uintptr_t)a.obs % 16 == 0) && ((uintptr_t)a.goal_out % 16 == 0);
  const bool al4 = (F % 4 == 0) && ((uintptr_t)a.obs % 4 == 0) && ((uintptr_t)a.goal_out % 4 == 0);
  if (al16)
    hipLaunchKernelGGL((env_kernel<MODE, 16>), grid, block, 0, stream, a);
  else if (al4)
    hipLaunchKernelGGL((env_kernel<MODE, 4>), grid, block, 0, stream, a);
  else
    hipLaunchKernelGGL((env_kernel<MODE, 1>), grid, block, 0, stream, a);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

void free_ctx(vn_ctx* c) {
  if (!c) return;
  void* ptrs[] = {c->arena, c->graph, c->spd, c->scenes, c->st, c->ep_ret, c->env_scene,
                  c->tasks, c->sched, c->flags, c->cur_order, c->cur_count};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  delete c;
}

}  // namespace

extern "C" {

const char* vn_version(void) { return "vnav 0.1.0 gfx950"; }

int vn_last_error(char* buf, size_t len) {
  if (!buf || len == 0) return VN_EINVAL;
  const std::string& m = vn::last_error();
  const size_t n = std::min(len - 1, m.size());
  std::memcpy(buf, m.data(), n);
  buf[n] = 0;
  return VN_OK;
}

int vn_create(const vn_scene_desc* scenes, int n_scenes, int n_envs, uint64_t seed, int device,
              vn_ctx** out) {
  if (!out) return fail(VN_EINVAL, "vn_create: out is NULL");
  *out = nullptr;
  if (!scenes || n_scenes <= 0) return fail(VN_EINVAL, "vn_create: need at least one scene");
  if (n_envs <= 0) return fail(VN_EINVAL, "vn_create: n_envs must be > 0");
  const int H = scenes[0].height, W = scenes[0].width, C = scenes[0].channels;
  if (H <= 0 || W <= 0 || C <= 0) return fail(VN_EINVAL, "vn_create: bad frame shape");
  const int64_t F = (int64_t)H * W * C;
  int64_t rows = 0, graph_rows = 0, spd_elems = 0;
  std::vector<SceneDev> sh(n_scenes);
  for (int k = 0; k < n_scenes; ++k) {
    const vn_scene_desc& d = scenes[k];
    if (d.height != H || d.width != W || d.channels != C)
      return fail(VN_EINVAL, "vn_create: all scenes must share one frame shape");
    if (d.n_states <= 0 || !d.graph || !d.spd) return fail(VN_EINVAL, "vn_create: scene missing graph/spd");
    if (!d.observations && (F % 4) != 0)
      return fail(VN_EINVAL, "vn_create: synthetic frames need frame bytes % 4 == 0");
    sh[k].row_base = rows;
    sh[k].graph_off = (int32_t)graph_rows;
    sh[k].spd_off = spd_elems;
    sh[k].n = d.n_states;
    sh[k].r_goal = d.reward_goal;
    sh[k].r_step = d.reward_step;
    sh[k].r_coll = d.reward_collision;
    sh[k].terminal_obs = d.terminal_obs;
    rows += d.n_states;
    sh[k].comp_base = -1;
    if (d.companion) {
      sh[k].comp_base = rows;
      rows += d.n_states;
    }
    graph_rows += d.n_states;
    spd_elems += (int64_t)d.n_states * d.n_states;
  }
  if (rows >= (1ll << 31)) return fail(VN_EINVAL, "vn_create: more than 2^31 frames");
  // Host-side conversion int64 -> int32 with range checks (the h5 datasets are int64).
  std::vector<int32_t> g32(graph_rows * 4);
  std::vector<int32_t> spd32(spd_elems);
  for (int k = 0; k < n_scenes; ++k) {
    const vn_scene_desc& d = scenes[k];
    const int64_t n = d.n_states;
    for (int64_t i = 0; i < n * 4; ++i) {
      const int64_t v = d.graph[i];
      if (v < -1 || v >= n) return fail(VN_EINVAL, "vn_create: graph entry out of range");
      g32[(int64_t)sh[k].graph_off * 4 + i] = (int32_t)v;
    }
    int32_t mx = 0;
    for (int64_t i = 0; i < n * n; ++i) {
      const int64_t v = d.spd[i];
      spd32[sh[k].spd_off + i] = (int32_t)std::max<int64_t>(std::min<int64_t>(v, INT32_MAX), INT32_MIN);
      mx = std::max(mx, spd32[sh[k].spd_off + i]);
    }
    if (mx > (1 << 20)) return fail(VN_EINVAL, "vn_create: spd values above 2^20");
    sh[k].maxd = mx;
  }
  int64_t cnt_elems = 0;
  for (int k = 0; k < n_scenes; ++k) {
    sh[k].cnt_off = cnt_elems;
    cnt_elems += (int64_t)sh[k].n * (sh[k].maxd + 2);
  }
  DeviceGuard guard(device);
  vn_ctx* c = new (std::nothrow) vn_ctx();
  if (!c) return fail(VN_ENOMEM, "vn_create: host allocation failed");
  c->device = device;
  c->n_envs = n_envs;
  c->n_scenes = n_scenes;
  c->seed = seed;
  c->frame_bytes = F;
  c->n_rows = rows;
  c->scenes_host = sh;
  c->spd_host = spd32;
  auto alloc = [&](void** p, size_t bytes) -> bool {
    return hipMalloc(p, std::max<size_t>(bytes, 16)) == hipSuccess;
  };
  bool ok = alloc((void**)&c->arena, (size_t)(rows * F)) && alloc((void**)&c->graph, g32.size() * 4) &&
            alloc((void**)&c->spd, spd32.size() * 4) && alloc((void**)&c->scenes, sh.size() * sizeof(SceneDev)) &&
            alloc((void**)&c->st, (size_t)ST_COUNT * n_envs * 4) && alloc((void**)&c->ep_ret, (size_t)n_envs * 4) &&
            alloc((void**)&c->env_scene, (size_t)n_envs * 4) && alloc((void**)&c->flags, 4);
  if (!ok) {
    free_ctx(c);
    return fail(VN_ENOMEM, "vn_create: device allocation failed");
  }
  hipError_t e = hipSuccess;
  std::vector<int32_t> es(n_envs);
  for (int i = 0; i < n_envs; ++i) es[i] = i % n_scenes;
  if (e == hipSuccess) e = hipMemcpy(c->graph, g32.data(), g32.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->spd, spd32.data(), spd32.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->scenes, sh.data(), sh.size() * sizeof(SceneDev), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->env_scene, es.data(), es.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(c->st, 0, (size_t)ST_COUNT * n_envs * 4);
  if (e == hipSuccess) e = hipMemset(c->ep_ret, 0, (size_t)n_envs * 4);
  if (e == hipSuccess) e = hipMemset(c->flags, 0, 4);
  for (int k = 0; k < n_scenes && e == hipSuccess; ++k) {
    const vn_scene_desc& d = scenes[k];
    if (d.companion)
      e = hipMemcpy(c->arena + sh[k].comp_base * F, d.companion, (size_t)d.n_states * F, hipMemcpyHostToDevice);
    if (e != hipSuccess) break;
    if (d.observations) {
      e = hipMemcpy(c->arena + sh[k].row_base * F, d.observations, (size_t)d.n_states * F, hipMemcpyHostToDevice);
    } else {
      hipLaunchKernelGGL(synth_frames_kernel, dim3(2048), dim3(256), 0, 0, c->arena, sh[k].row_base, d.n_states, F,
                         d.synth_id);
      e = hipGetLastError();
    }
  }
  if (e != hipSuccess) {
    free_ctx(c);
    return hip_fail(e, "vn_create: upload");
  }
  // The constructor's reset (cached.py:36): every env starts from a sampled (start, goal).
  EnvArgs a = make_args(c);
  int rc = launch_env<MODE_RESET>(c, a, 0);
  if (rc == VN_OK) {
    e = hipDeviceSynchronize();
    if (e != hipSuccess) rc = hip_fail(e, "vn_create: initial reset");
  }
  if (rc != VN_OK) {
    free_ctx(c);
    return rc;
  }
  *out = c;
  return VN_OK;
}

int vn_destroy(vn_ctx* c) {
  if (!c) return VN_OK;
  DeviceGuard guard(c->device);
  (void)hipDeviceSynchronize();
  free_ctx(c);
  return VN_OK;
}

int vn_num_envs(vn_ctx* c) { return c ? c->n_envs : VN_EINVAL; }

int vn_reset(vn_ctx* c, const int32_t* env_mask_dev, vn_stream_t stream) {
  if (!c) return fail(VN_EINVAL, "vn_reset: NULL ctx");
  DeviceGuard guard(c->device);
  EnvArgs a = make_args(c);
  a.mask = env_mask_dev;
  return launch_env<MODE_RESET>(c, a, (hipStream_t)stream);
}

int vn_observe(vn_ctx* c, uint8_t* obs_dev, uint8_t* goal_dev, int32_t* state_dev, vn_stream_t stream) {
  if (!c) return fail(VN_EINVAL, "vn_observe: NULL ctx");
  DeviceGuard guard(c->device);
  EnvArgs a = make_args(c);
  a.obs = obs_dev;
  a.goal_out = goal_dev;
  a.state_out = state_dev;
  return launch_env<MODE_OBSERVE>(c, a, (hipStream_t)stream);
}

int vn_step(vn_ctx* c, const int32_t* actions_dev, uint8_t* obs_dev, uint8_t* goal_dev, float* reward_dev,
            uint8_t* done_dev, int32_t* state_dev, vn_stream_t stream) {
  if (!c) return fail(VN_EINVAL, "vn_step: NULL ctx");
  if (!actions_dev) return fail(VN_EINVAL, "vn_step: actions is NULL");
  DeviceGuard guard(c->device);
  EnvArgs a = make_args(c);
  a.actions = actions_dev;
  a.obs = obs_dev;
  a.goal_out = goal_dev;
  a.reward = reward_dev;
  a.done = done_dev;
  a.state_out = state_dev;
  return launch_env<MODE_STEP>(c, a, (hipStream_t)stream);
}

int vn_step_a2c(vn_ctx* c, const vn_a2c_step* p, float* reward_dev, uint8_t* done_dev, int32_t* state_dev,
                vn_stream_t stream) {
  if (!c) return fail(VN_EINVAL, "vn_step_a2c: NULL ctx");
  if (!p || !p->policy_out || !p->actions || p->num_actions < 1 || p->num_actions > 7)
    return fail(VN_EINVAL, "vn_step_a2c: bad a2c arguments");
  DeviceGuard guard(c->device);
  EnvArgs a = make_args(c);
  a.reward = reward_dev;
  a.done = done_dev;
  a.state_out = state_dev;
  a.pol_out = p->policy_out;
  a.pol_A = p->num_actions;
  a.pk0 = (uint32_t)p->seed;
  a.pk1 = (uint32_t)(p->seed >> 32);
  a.pctr_dev = p->counter_base_dev;
  a.pctr = p->counter;
  a.act_out = p->actions;
  a.prev_action = p->prev_action;
  a.prev_reward = p->prev_reward;
  a.prev_mask = p->prev_mask;
  a.lra_next = p->lra_next;
  a.mask_next = p->mask_next;
  a.stats_env = p->episode_stats_env;
  if (p->head_weight) {
    if (!p->head_bias || !p->head_input || !p->head_out || p->head_out != p->policy_out)
      return fail(VN_EINVAL, "vn_step_a2c: head_weight needs head_bias, head_input and head_out == policy_out");
    if ((reinterpret_cast<uintptr_t>(p->head_weight) | reinterpret_cast<uintptr_t>(p->head_input)) & 15)
      return fail(VN_EINVAL, "vn_step_a2c: head_weight / head_input must be 16-byte aligned");
    a.head_w = p->head_weight;
    a.head_b = p->head_bias;
    a.head_x = p->head_input;
    a.head_out = p->head_out;
    return launch_env<MODE_STEP_HEADS>(c, a, (hipStream_t)stream);
  }
  return launch_env<MODE_STEP>(c, a, (hipStream_t)stream);
}

int vn_set_info_buffers(vn_ctx* c, float* ep_return, int32_t* ep_length, int32_t* terminal_state,
                        uint8_t* truncated, int32_t* img_row, int32_t* goal_row) {
  if (!c) return fail(VN_EINVAL, "vn_set_info_buffers: NULL ctx");
  c->info_ret = ep_return;
  c->info_len = ep_length;
  c->info_term = terminal_state;
  c->info_trunc = truncated;
  c->info_img_row = img_row;
  c->info_goal_row = goal_row;
  return VN_OK;
}

int vn_set_schedule(vn_ctx* c, const int32_t* start_goal_dev, int len) {
  if (!c) return fail(VN_EINVAL, "vn_set_schedule: NULL ctx");
  if (len < 0 || (len > 0 && !start_goal_dev)) return fail(VN_EINVAL, "vn_set_schedule: bad schedule");
  DeviceGuard guard(c->device);
  if (c->sched) {
    VN_HIP(hipDeviceSynchronize());
    VN_HIP(hipFree(c->sched));
    c->sched = nullptr;
  }
  c->sched_len = 0;
  if (len > 0) {
    const size_t bytes = (size_t)c->n_envs * len * 2 * 4;
    if (hipMalloc((void**)&c->sched, bytes) != hipSuccess) return fail(VN_ENOMEM, "vn_set_schedule: alloc");
    VN_HIP(hipMemcpy(c->sched, start_goal_dev, bytes, hipMemcpyDefault));
    c->sched_len = len;
  }
  VN_HIP(hipMemset(c->st + (size_t)ST_SCHED * c->n_envs, 0, (size_t)c->n_envs * 4));
  return VN_OK;
}

int vn_set_tasks(vn_ctx* c, const int32_t* tasks_host, int n_tasks) {
  if (!c) return fail(VN_EINVAL, "vn_set_tasks: NULL ctx");
  if (n_tasks < 0 || (n_tasks > 0 && !tasks_host)) return fail(VN_EINVAL, "vn_set_tasks: bad tasks");
  for (int t = 0; t < n_tasks; ++t) {
    const int sc = tasks_host[2 * t], g = tasks_host[2 * t + 1];
    if (sc < 0 || sc >= c->n_scenes) return fail(VN_EINVAL, "vn_set_tasks: scene out of range");
    if (g < -1 || g >= c->scenes_host[sc].n) return fail(VN_EINVAL, "vn_set_tasks: goal out of range");
  }
  DeviceGuard guard(c->device);
  if (c->tasks) {
    VN_HIP(hipDeviceSynchronize());
    VN_HIP(hipFree(c->tasks));
    c->tasks = nullptr;
  }
  c->n_tasks = 0;
  if (n_tasks > 0) {
    if (hipMalloc((void**)&c->tasks, (size_t)n_tasks * 8) != hipSuccess) return fail(VN_ENOMEM, "vn_set_tasks: alloc");
    VN_HIP(hipMemcpy(c->tasks, tasks_host, (size_t)n_tasks * 8, hipMemcpyHostToDevice));
    c->n_tasks = n_tasks;
  }
  return VN_OK;
}

int vn_set_env_scenes(vn_ctx* c, const int32_t* env_scene_host) {
  if (!c || !env_scene_host) return fail(VN_EINVAL, "vn_set_env_scenes: NULL argument");
  for (int e = 0; e < c->n_envs; ++e)
    if (env_scene_host[e] < 0 || env_scene_host[e] >= c->n_scenes)
      return fail(VN_EINVAL, "vn_set_env_scenes: scene out of range");
  DeviceGuard guard(c->device);
  VN_HIP(hipMemcpy(c->env_scene, env_scene_host, (size_t)c->n_envs * 4, hipMemcpyHostToDevice));
  return VN_OK;
}

int vn_set_curriculum_scenes(vn_ctx* c, double complexity, const int32_t* modes_host, const double* offsets_host) {
  if (!c || !modes_host || !offsets_host) return fail(VN_EINVAL, "vn_set_curriculum_scenes: NULL argument");
  if (!(complexity >= 0.0)) return fail(VN_EINVAL, "vn_set_curriculum: bad complexity");
  int any = 0;
  for (int i = 0; i < c->n_scenes; ++i) {
    if (modes_host[i] < 0 || modes_host[i] > 2) return fail(VN_EINVAL, "vn_set_curriculum: bad mode");
    any |= modes_host[i];
  }
  DeviceGuard guard(c->device);
  if (any && !c->cur_order) {
    // per scene and goal: states sorted by spd[s][g] (stable counting sort) + inclusive counts
    int64_t n_order = 0, n_cnt = 0;
    for (const SceneDev& S : c->scenes_host) {
      n_order += (int64_t)S.n * S.n;
      n_cnt += (int64_t)S.n * (S.maxd + 2);
    }
    std::vector<int32_t> order(n_order), cnt(n_cnt);
    for (const SceneDev& S : c->scenes_host) {
      const int n = S.n, B = S.maxd + 2;
      const int32_t* spd = c->spd_host.data() + S.spd_off;
      std::vector<int32_t> hist(B);
      for (int g = 0; g < n; ++g) {
        std::fill(hist.begin(), hist.end(), 0);
        for (int s = 0; s < n; ++s) hist[std::min(std::max(spd[(int64_t)s * n + g], -1), S.maxd) + 1]++;
        int32_t* cg = cnt.data() + S.cnt_off + (int64_t)g * B;
        int run = 0;
        for (int b = 0; b < B; ++b) {
          const int h = hist[b];
          hist[b] = run;  // start of bucket b
          run += h;
          cg[b] = run;    // inclusive count
        }
        int32_t* og = order.data() + S.spd_off + (int64_t)g * n;
        for (int s = 0; s < n; ++s) og[hist[std::min(std::max(spd[(int64_t)s * n + g], -1), S.maxd) + 1]++] = s;
      }
    }
    if (hipMalloc((void**)&c->cur_order, std::max<size_t>(order.size() * 4, 16)) != hipSuccess ||
        hipMalloc((void**)&c->cur_count, std::max<size_t>(cnt.size() * 4, 16)) != hipSuccess)
      return fail(VN_ENOMEM, "vn_set_curriculum: device allocation failed");
    VN_HIP(hipMemcpy(c->cur_order, order.data(), order.size() * 4, hipMemcpyHostToDevice));
    VN_HIP(hipMemcpy(c->cur_count, cnt.data(), cnt.size() * 4, hipMemcpyHostToDevice));
  }
  for (int i = 0; i < c->n_scenes; ++i) {  // the reference computes opt in Python floats (fp64)
    SceneDev& S = c->scenes_host[i];
    const double opt = complexity * ((double)S.maxd + offsets_host[i]) + 1.0;
    S.cur_oi = (int32_t)std::min<double>(std::max<double>(std::floor(opt), 0.0), (double)S.maxd);
    S.cur_mode = modes_host[i];
  }
  VN_HIP(hipMemcpy(c->scenes, c->scenes_host.data(), c->scenes_host.size() * sizeof(SceneDev), hipMemcpyHostToDevice));
  c->cur_mode = any ? 1 : 0;
  c->cur_c = complexity;
  return VN_OK;
}

int vn_set_curriculum(vn_ctx* c, double complexity, int mode, double offset) {
  if (!c) return fail(VN_EINVAL, "vn_set_curriculum: NULL ctx");
  std::vector<int32_t> modes(c->n_scenes, mode);
  std::vector<double> offsets(c->n_scenes, offset);
  return vn_set_curriculum_scenes(c, complexity, modes.data(), offsets.data());
}


int vn_set_max_episode_steps(vn_ctx* c, int max_steps) {
  if (!c) return fail(VN_EINVAL, "vn_set_max_episode_steps: NULL ctx");
  c->max_steps = max_steps;
  return VN_OK;
}

int vn_set_autoreset(vn_ctx* c, int on) {
  if (!c) return fail(VN_EINVAL, "vn_set_autoreset: NULL ctx");
  c->autoreset = on ? 1 : 0;
  return VN_OK;
}

int vn_random_actions(vn_ctx* c, int32_t* actions_dev, uint64_t step, vn_stream_t stream) {
  if (!c || !actions_dev) return fail(VN_EINVAL, "vn_random_actions: NULL argument");
  DeviceGuard guard(c->device);
  hipLaunchKernelGGL(random_actions_kernel, dim3((c->n_envs + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     actions_dev, c->n_envs, (uint32_t)c->seed ^ 0xA5A5A5A5u, (uint32_t)(c->seed >> 32), step);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_gather_rows(const uint8_t* src_dev, int64_t row_bytes, const int32_t* rows_dev, int n, uint8_t* dst_dev,
                   vn_stream_t stream) {
  if (!src_dev || !rows_dev || !dst_dev || row_bytes <= 0 || n < 0) return fail(VN_EINVAL, "vn_gather_rows: bad args");
  if (n == 0) return VN_OK;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, src_dev, row_bytes,
                     rows_dev, n, dst_dev);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_get_state(vn_ctx* c, int32_t* dst, vn_stream_t stream) {
  if (!c || !dst) return fail(VN_EINVAL, "vn_get_state: NULL argument");
  DeviceGuard guard(c->device);
  VN_HIP(hipMemcpyAsync(dst, c->st, (size_t)ST_COUNT * c->n_envs * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return VN_OK;
}

int vn_set_state(vn_ctx* c, const int32_t* src, vn_stream_t stream) {
  if (!c || !src) return fail(VN_EINVAL, "vn_set_state: NULL argument");
  DeviceGuard guard(c->device);
  VN_HIP(hipMemcpyAsync(c->st, src, (size_t)ST_COUNT * c->n_envs * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return VN_OK;
}

int vn_get_episode_returns(vn_ctx* c, float* dst, vn_stream_t stream) {
  if (!c || !dst) return fail(VN_EINVAL, "vn_get_episode_returns: NULL argument");
  DeviceGuard guard(c->device);
  VN_HIP(hipMemcpyAsync(dst, c->ep_ret, (size_t)c->n_envs * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return VN_OK;
}

int vn_set_episode_returns(vn_ctx* c, const float* src, vn_stream_t stream) {
  if (!c || !src) return fail(VN_EINVAL, "vn_set_episode_returns: NULL argument");
  DeviceGuard guard(c->device);
  VN_HIP(hipMemcpyAsync(c->ep_ret, src, (size_t)c->n_envs * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return VN_OK;
}

int vn_frame_arena(vn_ctx* c, const uint8_t** arena, int64_t* frame_bytes, int64_t* n_rows) {
  if (!c) return fail(VN_EINVAL, "vn_frame_arena: NULL ctx");
  if (arena) *arena = c->arena;
  if (frame_bytes) *frame_bytes = c->frame_bytes;
  if (n_rows) *n_rows = c->n_rows;
  return VN_OK;
}

int vn_scene_row_base(vn_ctx* c, int scene, int64_t* row_base) {
  if (!c || !row_base || scene < 0 || scene >= c->n_scenes) return fail(VN_EINVAL, "vn_scene_row_base: bad args");
  *row_base = c->scenes_host[scene].row_base;
  return VN_OK;
}

int vn_error_flags_sync(vn_ctx* c, uint32_t* flags, int clear) {
  if (!c || !flags) return fail(VN_EINVAL, "vn_error_flags_sync: NULL argument");
  DeviceGuard guard(c->device);
  VN_HIP(hipDeviceSynchronize());
  VN_HIP(hipMemcpy(flags, c->flags, 4, hipMemcpyDeviceToHost));
  if (clear) VN_HIP(hipMemset(c->flags, 0, 4));
  return VN_OK;
}

}  // extern "C"
