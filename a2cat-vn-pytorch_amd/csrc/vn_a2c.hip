// vn_a2c.hip — the A2C pieces around the policy on gfx950: categorical sampling,
// n-step returns, the loss gradient w.r.t. the head outputs, the global gradient norm
// and the fused clip + RMSprop step.
//
// Contract (DESIGN.md "A2C contract"; parity unpinned at this level because the
// reference's trainer is the absent deep-rl==0.2.9, experiments/thor_cached_auxiliary.py:26-42):
//   R_T = V(s_T); R_t = r_t + gamma R_{t+1} (1 - done_t); A_t = R_t - V(s_t)
//   L = vc mean(A^2) - mean(A.detach() log pi(a_t)) - ec mean(H(pi))
//   clip_grad_norm_(max_norm) then RMSprop(lr, alpha, eps) with torch's update rule.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "vn_common.h"

namespace vn {

constexpr int OUT_LD_A2C = 8;

// ctr_dev (optional): the Philox counter is *ctr_dev + ctr (a device-side update counter, so
// a captured hipGraph of the update samples with a fresh counter on every replay).
__global__ void sample_kernel(const float* __restrict__ out, int n, int A, uint32_t k0, uint32_t k1, uint64_t ctr,
                              const int64_t* __restrict__ ctr_dev, int32_t* actions, float* logp_out, float* ent_out,
                              float* value_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (ctr_dev) ctr += (uint64_t)*ctr_dev;
  float lg[7], p[7], lp[7], H;
  for (int j = 0; j < A; ++j) lg[j] = out[(int64_t)i * OUT_LD_A2C + j];
  const int a = sample_action(lg, A, k0, k1, ctr, (uint32_t)i, p, lp, H);
  actions[i] = a;
  if (logp_out) logp_out[i] = lp[a];
  if (ent_out) ent_out[i] = H;
  if (value_out) value_out[i] = out[(int64_t)i * OUT_LD_A2C + A];
}

__global__ void greedy_kernel(const float* __restrict__ out, int n, int A, int32_t* actions) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int a = 0;
  float best = out[(int64_t)i * OUT_LD_A2C];
  for (int j = 1; j < A; ++j) {
    const float v = out[(int64_t)i * OUT_LD_A2C + j];
    if (v > best) {
      best = v;
      a = j;
    }
  }
  actions[i] = a;
}

__global__ void returns_kernel(const float* __restrict__ rewards, const uint8_t* __restrict__ dones,
                               const float* __restrict__ boot_out, int T, int E, int A, float gamma, float* returns) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  float R = boot_out[(int64_t)e * OUT_LD_A2C + A];
  for (int t = T - 1; t >= 0; --t) {
    const int64_t i = (int64_t)t * E + e;
    R = rewards[i] + gamma * R * (1.0f - (float)dones[i]);
    returns[i] = R;
  }
}

// dL/d(head outputs) for L = vc mean(A^2) - mean(A logp_a) - ec mean(H); stats += block sums of
// (A^2, -A logp_a, H, R).
__global__ __launch_bounds__(256) void loss_grad_kernel(const float* __restrict__ out, const int32_t* __restrict__ actions,
                                                        const float* __restrict__ returns, int n, int A, float vc,
                                                        float ec, float inv_n, float* dout, float* stats) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (i < n) {
    float lg[7], p[7], lp[7], H;
    for (int j = 0; j < A; ++j) lg[j] = out[(int64_t)i * OUT_LD_A2C + j];
    softmax_stats(lg, A, p, lp, H);
    const int a = actions[i];
    const float R = returns[i];
    const float V = out[(int64_t)i * OUT_LD_A2C + A];
    const float adv = R - V;
    for (int j = 0; j < A; ++j) {
      const float ind = (j == a) ? 1.0f : 0.0f;
      dout[(int64_t)i * OUT_LD_A2C + j] = (-adv * (ind - p[j]) + ec * p[j] * (lp[j] + H)) * inv_n;
    }
    dout[(int64_t)i * OUT_LD_A2C + A] = vc * (-2.0f * adv) * inv_n;
    for (int j = A + 1; j < OUT_LD_A2C; ++j) dout[(int64_t)i * OUT_LD_A2C + j] = 0.0f;
    s0 = adv * adv;
    s1 = -adv * lp[a];
    s2 = H;
    s3 = R;
  }
  __shared__ float red[4][4];
  for (int off = 32; off > 0; off >>= 1) {
    s0 += __shfl_down(s0, off);
    s1 += __shfl_down(s1, off);
    s2 += __shfl_down(s2, off);
    s3 += __shfl_down(s3, off);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w][0] = s0;
    red[w][1] = s1;
    red[w][2] = s2;
    red[w][3] = s3;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const float v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    atomicAdd(&stats[threadIdx.x], v);
  }
}

constexpr int kNormBlocks = 512;

__global__ __launch_bounds__(256) void sumsq_partial_kernel(const float* __restrict__ g, int64_t n, float scale,
                                                            double* partial) {
  double s = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = g[i] * scale;
    s += (double)v * (double)v;
  }
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// sumsq_partial_kernel with up to two gradient addends joined first: g[i] += add_j[i] for i in
// [lo_j, hi_j) (written back, each addend in its own range, the ranges disjoint or added in
// order j = 0, 1), so the side passes' gradient sums (the replayed aux / UNREAL trunk, heads
// and LSTM) cost no launch of their own. The same grid-stride order as sumsq_partial_kernel:
// the partial sums, hence the norm, are bitwise those of a separate add + norm.
__global__ __launch_bounds__(256) void sumsq_join_partial_kernel(float* __restrict__ g, int64_t n, float scale,
                                                                 const float* __restrict__ a0, int64_t lo0, int64_t hi0,
                                                                 const float* __restrict__ a1, int64_t lo1, int64_t hi1,
                                                                 double* partial) {
  double s = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float x = g[i];
    const bool j0 = a0 && i >= lo0 && i < hi0, j1 = a1 && i >= lo1 && i < hi1;
    if (j0) x = x + a0[i];
    if (j1) x = x + a1[i];
    if (j0 || j1) g[i] = x;
    const float v = x * scale;
    s += (double)v * (double)v;
  }
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// scalars[0] = total norm, scalars[1] = clip coefficient (torch clip_grad_norm_: max_norm / (norm + 1e-6), <= 1)
__global__ void norm_final_kernel(const double* partial, int nb, float max_norm, float* scalars) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256) s += partial[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float norm = (float)sqrt(red[0]);
    scalars[0] = norm;
    scalars[1] = max_norm > 0.0f ? fminf(max_norm / (norm + 1e-6f), 1.0f) : 1.0f;
  }
}

__global__ __launch_bounds__(256) void rmsprop_kernel(float* __restrict__ params, const float* __restrict__ grads,
                                                      float* __restrict__ sq, int64_t n, float scale,
                                                      const float* __restrict__ scalars, float lr,
                                                      const float* __restrict__ lr_dev, float alpha, float eps) {
  const float coef = scalars[1] * scale;
  if (lr_dev) lr = *lr_dev;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float g = grads[i] * coef;
    const float s = sq[i] * alpha + (1.0f - alpha) * g * g;
    sq[i] = s;
    params[i] += -lr * (g / (sqrtf(s) + eps));
  }
}

// Per-env-step bookkeeping of the rollout, one workgroup: the next step's recurrent inputs
// (last action / last reward of UnrealEnvBaseWrapper, models/goal.py:63-64, and the episode
// mask m = 1 - done) and the finished-episode statistics of deep_rl's RewardCollector
// (experiments/thor_cached_auxiliary.py:59-64: count, return sum, length sum) summed in a
// fixed order — replaces ~20 small framework kernels per step.
constexpr int kPostThreads = 1024;
__global__ __launch_bounds__(kPostThreads) void step_post_kernel(const int32_t* __restrict__ actions,
                                                                 const float* __restrict__ rewards,
                                                                 const uint8_t* __restrict__ dones,
                                                                 const float* __restrict__ ep_return,
                                                                 const int32_t* __restrict__ ep_length, int E, int A,
                                                                 int64_t* prev_action, float* prev_reward,
                                                                 float* prev_mask, float* lra, float* mask_out,
                                                                 float* stats3) {
  float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f;
  for (int e = threadIdx.x; e < E; e += kPostThreads) {
    const bool d = dones[e] != 0;
    const int a = actions[e];
    const float r = rewards[e], m = d ? 0.0f : 1.0f;
    if (prev_action) prev_action[e] = a;
    if (prev_reward) prev_reward[e] = r;
    if (prev_mask) prev_mask[e] = m;
    if (mask_out) mask_out[e] = m;
    if (lra) {
      for (int j = 0; j < A; ++j) lra[(int64_t)e * (A + 1) + j] = j == a ? m : 0.0f;
      lra[(int64_t)e * (A + 1) + A] = r * m;
    }
    if (d) {
      s0 += 1.0f;
      s1 += ep_return[e];
      s2 += (float)ep_length[e];
    }
  }
  __shared__ float red[3][kPostThreads / 64];
  for (int o = 32; o > 0; o >>= 1) {
    s0 += __shfl_xor(s0, o);
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = s0;
    red[1][w] = s1;
    red[2][w] = s2;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    float t = 0.0f;
    for (int i = 0; i < kPostThreads / 64; ++i) t += red[threadIdx.x][i];
    stats3[threadIdx.x] += t;
  }
}

// Fixed-order sums of the per-env episode statistics of a rollout (vn_step_a2c), then zeroed.
__global__ __launch_bounds__(kPostThreads) void episode_stats_kernel(float* __restrict__ st_env, int E,
                                                                     float* __restrict__ stats3) {
  float s[3] = {0.0f, 0.0f, 0.0f};
  for (int e = threadIdx.x; e < E; e += kPostThreads)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      s[k] += st_env[(int64_t)k * E + e];
      st_env[(int64_t)k * E + e] = 0.0f;
    }
  __shared__ float red[3][kPostThreads / 64];
#pragma unroll
  for (int k = 0; k < 3; ++k)
    for (int o = 32; o > 0; o >>= 1) s[k] += __shfl_xor(s[k], o);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < 3; ++k) red[k][w] = s[k];
  __syncthreads();
  if (threadIdx.x < 3) {
    float t = 0.0f;
    for (int i = 0; i < kPostThreads / 64; ++i) t += red[threadIdx.x][i];
    stats3[threadIdx.x] = t;
  }
}

// Device-side trainer schedule, one thread, launched first in every update:
//   state[2] (counter of this update) = state[0]; state[0] += T (policy sampling counter base,
//   = updates * T); lr = lr0 * (1 - min(state[1] / max_steps, 1)) in double as the host's
//   LinearSchedule (experiments/thor_cached_auxiliary.py:37) computes it, rounded once to f32;
//   state[1] += steps_per_update (env-steps of all ranks).
__global__ void a2c_schedule_kernel(int64_t* state, float* lr_out, double lr0, double max_steps,
                                    int64_t steps_per_update, int T) {
  const int64_t total = state[1];
  const double frac = max_steps > 0.0 ? fmin((double)total / max_steps, 1.0) : 0.0;
  *lr_out = (float)(lr0 * (1.0 - frac));
  state[2] = state[0];
  state[0] += T;
  state[1] = total + steps_per_update;
}

// First launch of a rollout: the device schedule (thread 0: a2c_schedule_kernel's
// arithmetic), step 0's frame rows copied from the env's current rows, and — recurrent —
// step 0's mask = the carried m and its [one_hot(a) | r] * m (UnrealEnvBaseWrapper,
// models/goal.py:63-64), with step_post_kernel's arithmetic. Replaces eight launches
// (schedule, two row copies, the mask copy and four framework kernels of the one-hot build).
__global__ __launch_bounds__(256) void rollout_begin_kernel(int64_t* state, float* lr_out, double lr0, double max_steps,
                                                            int64_t steps_per_update, int T,
                                                            const int32_t* __restrict__ img_src,
                                                            const int32_t* __restrict__ goal_src,
                                                            int32_t* __restrict__ img_dst,
                                                            int32_t* __restrict__ goal_dst, int E,
                                                            const int64_t* __restrict__ prev_action,
                                                            const float* __restrict__ prev_reward,
                                                            const float* __restrict__ prev_mask, int A,
                                                            float* __restrict__ mask0, float* __restrict__ lra0) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e == 0) {
    const int64_t total = state[1];
    const double frac = max_steps > 0.0 ? fmin((double)total / max_steps, 1.0) : 0.0;
    *lr_out = (float)(lr0 * (1.0 - frac));
    state[2] = state[0];
    state[0] += T;
    state[1] = total + steps_per_update;
  }
  if (e >= E) return;
  img_dst[e] = img_src[e];
  goal_dst[e] = goal_src[e];
  if (mask0) {
    const float m = prev_mask[e];
    const int64_t a = prev_action[e];
    mask0[e] = m;
    for (int j = 0; j < A; ++j) lra0[(int64_t)e * (A + 1) + j] = j == a ? m : 0.0f;
    lra0[(int64_t)e * (A + 1) + A] = prev_reward[e] * m;
  }
}

// The update's metric vector in one thread (replaces four framework kernels): [stats4 *
// inv_n (torch's tensor / scalar: times the f32 reciprocal), grad norm, aux loss = the
// per-head MSEs summed (ai2_auxiliary/trainer.py:51-54), episode stats3].
__global__ void metrics_kernel(const float* __restrict__ stats4, float inv_n, const float* __restrict__ scalars2,
                               const float* __restrict__ aux3, const float* __restrict__ aux_numel3,
                               const float* __restrict__ episode3, const float* __restrict__ unreal4,
                               const float* __restrict__ unreal_norm3, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  for (int i = 0; i < 4; ++i) out[i] = stats4[i] * inv_n;
  out[4] = scalars2[0];
  // (h0 + h2) + h1: torch's sum of three values (two threads along the reduction, thread 0
  // takes elements 0 and 2, then one shuffle step)
  out[5] = aux3 ? (aux3[0] / aux_numel3[0] + aux3[2] / aux_numel3[2]) + aux3[1] / aux_numel3[1] : 0.0f;
  for (int i = 0; i < 3; ++i) out[6 + i] = episode3[i];
  if (unreal4) {  // [pc sum sq, rp mean CE, (rp count), vr sum sq] x [pc, rp, vr] normalisers
    out[9] = unreal4[0] * unreal_norm3[0];
    out[10] = unreal4[1] * unreal_norm3[1];
    out[11] = unreal4[3] * unreal_norm3[2];
  }
}

// ---- goal runs (vn_goal_runs, include/vnav.h) ----------------------------------------
// One workgroup of kGoalThreads: thread i takes a contiguous chunk of the items, counts its
// flagged ones, an inclusive scan over the threads gives each chunk its base, and the chunk
// writes its flagged items in order — the list is ascending (deterministic).
constexpr int kGoalThreads = 1024;

__device__ __forceinline__ int block_scan_incl(int v, int* sh) {
  const int tid = threadIdx.x;
  sh[tid] = v;
  __syncthreads();
  for (int d = 1; d < kGoalThreads; d <<= 1) {
    const int add = tid >= d ? sh[tid - d] : 0;
    __syncthreads();
    sh[tid] += add;
    __syncthreads();
  }
  return sh[tid];
}

__global__ __launch_bounds__(kGoalThreads) void goal_runs_step_kernel(const uint8_t* __restrict__ done_prev,
                                                                      const int32_t* __restrict__ delta_prev, int E,
                                                                      int32_t* __restrict__ delta,
                                                                      int32_t* __restrict__ list,
                                                                      int32_t* __restrict__ count) {
  __shared__ int sh[kGoalThreads];
  const int tid = threadIdx.x, per = (E + kGoalThreads - 1) / kGoalThreads;
  const int e0 = min(tid * per, E), e1 = min(e0 + per, E);
  int c = 0;
  for (int e = e0; e < e1; ++e) {
    const bool nw = !done_prev || done_prev[e];
    delta[e] = nw ? 0 : delta_prev[e] - E;
    c += nw;
  }
  const int incl = block_scan_incl(c, sh);
  int o = incl - c;
  for (int e = e0; e < e1; ++e)
    if (!done_prev || done_prev[e]) list[o++] = e;
  if (tid == kGoalThreads - 1) *count = incl;
}

__global__ __launch_bounds__(kGoalThreads) void goal_runs_rollout_kernel(const uint8_t* __restrict__ dones, int T,
                                                                         int E, int32_t* __restrict__ list,
                                                                         int32_t* __restrict__ run_length,
                                                                         int32_t* __restrict__ count) {
  __shared__ int sh[kGoalThreads];
  const int tid = threadIdx.x;
  // run lengths, per env from the last step back: a run ends at its env's next done (that
  // step still has the run's goal) or at the rollout's last step
  for (int e = tid; e < E; e += kGoalThreads) {
    int end = T - 1;
    for (int t = T - 1; t >= 0; --t) {
      if (dones[(int64_t)t * E + e]) end = t;
      if (t == 0 || dones[(int64_t)(t - 1) * E + e]) run_length[(int64_t)t * E + e] = end - t + 1;
    }
  }
  const int64_t N = (int64_t)T * E, per = (N + kGoalThreads - 1) / kGoalThreads;
  const int64_t s0 = min((int64_t)tid * per, N), s1 = min(s0 + per, N);
  auto start = [&](int64_t s) { return s < E || dones[s - E] != 0; };
  int c = 0;
  for (int64_t s = s0; s < s1; ++s) c += start(s);
  const int incl = block_scan_incl(c, sh);
  int o = incl - c;
  for (int64_t s = s0; s < s1; ++s)
    if (start(s)) list[o++] = (int32_t)s;
  if (tid == kGoalThreads - 1) *count = incl;
}

// Trace marker: an empty kernel whose grid size (tag workgroups of 64 lanes) a kernel
// trace records, so a rocprofv3 trace of a test run can be split per test.
// ---- the replay ring on the device (vn_replay_push_draw) ---------------------------
constexpr int kReplayMaxSegs = 16;
struct ReplaySegs {
  vn_replay_seg s[kReplayMaxSegs];
  int n;
};

// Slot k drawn over the filled slots after this push: Philox4x32-10 (ctr_lo, ctr_hi, 0,
// STREAM_REPLAY) under key (seed_lo, seed_hi), uniform_below(r.x, filled') (DESIGN "RNG streams").
__device__ __forceinline__ void replay_draw(const int64_t* meta, int R, uint32_t k0, uint32_t k1, int& pos, int& filled,
                                            int& k) {
  pos = (int)meta[0];
  filled = min((int)meta[1] + 1, R);
  const uint64_t ctr = (uint64_t)meta[2];
  const u32x4 r = philox4x32_10(u32x4{(uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, STREAM_REPLAY}, k0, k1);
  k = (int)(((uint64_t)r.x * (uint64_t)filled) >> 32);
}

// Every block reads meta (pos, filled, counter), copies its share of each segment's source into
// ring slot pos and, when cur != NULL, the drawn slot k into cur: from the source itself when
// k == pos (the slot this launch writes), else from slot k (which no block writes). meta itself
// is advanced by replay_meta_kernel afterwards (a block here may still be reading it).
__global__ __launch_bounds__(256) void replay_push_draw_kernel(ReplaySegs segs, const int64_t* __restrict__ meta, int R,
                                                               uint32_t k0, uint32_t k1) {
  int pos, filled, k;
  replay_draw(meta, R, k0, k1, pos, filled, k);
  const int64_t g0 = blockIdx.x * 256ll + threadIdx.x, gs = (int64_t)gridDim.x * 256;
  for (int j = 0; j < segs.n; ++j) {
    const vn_replay_seg& sg = segs.s[j];
    const int64_t cnt = (int64_t)sg.rows * sg.cols;
    if (sg.elem_bytes == 4) {
      const uint32_t* src = (const uint32_t*)sg.src;
      uint32_t* ring = (uint32_t*)sg.ring;
      uint32_t* cur = (uint32_t*)sg.cur;
      for (int64_t i = g0; i < cnt; i += gs) {
        const int64_t r = i / sg.cols, c = i - r * sg.cols;
        const uint32_t v = src[r * sg.src_ld + c];
        ring[(int64_t)pos * sg.slot_elems + i] = v;
        if (cur) cur[i] = k == pos ? v : ring[(int64_t)k * sg.slot_elems + i];
      }
    } else {
      const uint8_t* src = (const uint8_t*)sg.src;
      uint8_t* ring = (uint8_t*)sg.ring;
      uint8_t* cur = (uint8_t*)sg.cur;
      for (int64_t i = g0; i < cnt; i += gs) {
        const int64_t r = i / sg.cols, c = i - r * sg.cols;
        const uint8_t v = src[r * sg.src_ld + c];
        ring[(int64_t)pos * sg.slot_elems + i] = v;
        if (cur) cur[i] = k == pos ? v : ring[(int64_t)k * sg.slot_elems + i];
      }
    }
  }
}

__global__ void replay_meta_kernel(int64_t* meta, int R, uint32_t k0, uint32_t k1) {
  int pos, filled, k;
  replay_draw(meta, R, k0, k1, pos, filled, k);
  meta[0] = (pos + 1) % R;
  meta[1] = filled;
  meta[2] += 1;
  meta[3] = k;
}

__global__ void trace_marker_kernel() {}

}  // namespace vn

using namespace vn;

extern "C" {

int vn_a2c_episode_stats(float* episode_stats_env, int E, float* stats3, vn_stream_t stream) {
  if (!episode_stats_env || !stats3 || E <= 0) return fail(VN_EINVAL, "vn_a2c_episode_stats: bad args");
  hipLaunchKernelGGL(episode_stats_kernel, dim3(1), dim3(kPostThreads), 0, (hipStream_t)stream, episode_stats_env, E,
                     stats3);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_replay_push_draw(const vn_replay_seg* segs, int nseg, int64_t* meta4, int capacity, uint64_t seed,
                        vn_stream_t stream) {
  if (!segs || nseg < 1 || nseg > kReplayMaxSegs || !meta4 || capacity < 1)
    return fail(VN_EINVAL, "vn_replay_push_draw: bad args (1..16 segments, capacity >= 1)");
  ReplaySegs a{};
  int64_t most = 0;
  for (int j = 0; j < nseg; ++j) {
    const vn_replay_seg& g = segs[j];
    if (!g.src || !g.ring || g.rows < 1 || g.cols < 1 || (g.elem_bytes != 1 && g.elem_bytes != 4) ||
        g.src_ld < g.cols || g.slot_elems < (int64_t)g.rows * g.cols)
      return fail(VN_EINVAL, "vn_replay_push_draw: bad segment");
    a.s[j] = g;
    most = std::max<int64_t>(most, (int64_t)g.rows * g.cols);
  }
  a.n = nseg;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((most + 255) / 256, 1024));
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(replay_push_draw_kernel, dim3(blocks), dim3(256), 0, st, a, meta4, capacity, k0, k1);
  hipLaunchKernelGGL(replay_meta_kernel, dim3(1), dim3(1), 0, st, meta4, capacity, k0, k1);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_goal_runs_step(const uint8_t* done_prev, const int32_t* delta_prev, int E, int32_t* delta, int32_t* list,
                      int32_t* count, vn_stream_t stream) {
  if (E <= 0 || !delta || !list || !count || (done_prev && !delta_prev))
    return fail(VN_EINVAL, "vn_goal_runs_step: bad args");
  hipLaunchKernelGGL(goal_runs_step_kernel, dim3(1), dim3(kGoalThreads), 0, (hipStream_t)stream, done_prev, delta_prev,
                     E, delta, list, count);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_goal_runs_rollout(const uint8_t* dones, int T, int E, int32_t* list, int32_t* run_length, int32_t* count,
                         vn_stream_t stream) {
  if (!dones || T <= 0 || E <= 0 || !list || !run_length || !count || (int64_t)T * E > INT32_MAX)
    return fail(VN_EINVAL, "vn_goal_runs_rollout: bad args");
  hipLaunchKernelGGL(goal_runs_rollout_kernel, dim3(1), dim3(kGoalThreads), 0, (hipStream_t)stream, dones, T, E, list,
                     run_length, count);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_trace_marker(int tag, vn_stream_t stream) {
  if (tag < 1 || tag > 65535) return fail(VN_EINVAL, "vn_trace_marker: tag must be 1..65535");
  hipLaunchKernelGGL(trace_marker_kernel, dim3(tag), dim3(64), 0, (hipStream_t)stream);
  return VN_OK;
}

int vn_policy_sample(const float* out, int n, int num_actions, uint64_t seed, uint64_t counter, int32_t* actions,
                     float* logp, float* entropy, float* value, vn_stream_t stream) {
  if (!out || !actions || n <= 0 || num_actions < 1 || num_actions > 7)
    return fail(VN_EINVAL, "vn_policy_sample: bad args");
  hipLaunchKernelGGL(sample_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, out, n, num_actions,
                     (uint32_t)seed, (uint32_t)(seed >> 32), counter, (const int64_t*)nullptr, actions, logp, entropy,
                     value);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_policy_sample_dev(const float* out, int n, int num_actions, uint64_t seed, const int64_t* counter_base_dev,
                         uint64_t counter_offset, int32_t* actions, float* logp, float* entropy, float* value,
                         vn_stream_t stream) {
  if (!out || !actions || !counter_base_dev || n <= 0 || num_actions < 1 || num_actions > 7)
    return fail(VN_EINVAL, "vn_policy_sample_dev: bad args");
  hipLaunchKernelGGL(sample_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, out, n, num_actions,
                     (uint32_t)seed, (uint32_t)(seed >> 32), counter_offset, counter_base_dev, actions, logp, entropy,
                     value);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_a2c_schedule(int64_t* state3, float* lr_out, double lr0, double max_time_steps, int64_t steps_per_update,
                    int T, vn_stream_t stream) {
  if (!state3 || !lr_out || T <= 0 || steps_per_update < 0) return fail(VN_EINVAL, "vn_a2c_schedule: bad args");
  hipLaunchKernelGGL(a2c_schedule_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, state3, lr_out, lr0,
                     max_time_steps, steps_per_update, T);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_a2c_rollout_begin(int64_t* state3, float* lr_out, double lr0, double max_time_steps, int64_t steps_per_update,
                         int T, const int32_t* img_row_src, const int32_t* goal_row_src, int32_t* img_row_dst,
                         int32_t* goal_row_dst, int E, const int64_t* prev_action, const float* prev_reward,
                         const float* prev_mask, int num_actions, float* mask0, float* lra0, vn_stream_t stream) {
  if (!state3 || !lr_out || T <= 0 || steps_per_update < 0 || E <= 0 || !img_row_src || !goal_row_src ||
      !img_row_dst || !goal_row_dst)
    return fail(VN_EINVAL, "vn_a2c_rollout_begin: bad args");
  if (mask0 && (!lra0 || !prev_action || !prev_reward || !prev_mask || num_actions <= 0))
    return fail(VN_EINVAL, "vn_a2c_rollout_begin: mask0 needs lra0, prev_action, prev_reward, prev_mask");
  hipLaunchKernelGGL(rollout_begin_kernel, dim3((E + 255) / 256), dim3(256), 0, (hipStream_t)stream, state3, lr_out,
                     lr0, max_time_steps, steps_per_update, T, img_row_src, goal_row_src, img_row_dst, goal_row_dst,
                     E, prev_action, prev_reward, prev_mask, num_actions, mask0, lra0);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_a2c_metrics_ex(const float* stats4, float inv_n, const float* scalars2, const float* aux3,
                      const float* aux_numel3, const float* episode_stats3, const float* unreal4,
                      const float* unreal_norm3, float* out, vn_stream_t stream) {
  if (!stats4 || !scalars2 || !episode_stats3 || !out || (aux3 && !aux_numel3) || (unreal4 && !unreal_norm3))
    return fail(VN_EINVAL, "vn_a2c_metrics: bad args");
  hipLaunchKernelGGL(metrics_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, stats4, inv_n, scalars2, aux3,
                     aux_numel3, episode_stats3, unreal4, unreal_norm3, out);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_a2c_metrics(const float* stats4, float inv_n, const float* scalars2, const float* aux3,
                   const float* aux_numel3, const float* episode_stats3, float* out9, vn_stream_t stream) {
  return vn_a2c_metrics_ex(stats4, inv_n, scalars2, aux3, aux_numel3, episode_stats3, nullptr, nullptr, out9, stream);
}

int vn_policy_greedy(const float* out, int n, int num_actions, int32_t* actions, vn_stream_t stream) {
  if (!out || !actions || n <= 0 || num_actions < 1 || num_actions > 7)
    return fail(VN_EINVAL, "vn_policy_greedy: bad args");
  hipLaunchKernelGGL(greedy_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, out, n, num_actions,
                     actions);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_a2c_returns(const float* rewards, const uint8_t* dones, const float* bootstrap_out, int T, int E,
                   int num_actions, float gamma, float* returns, vn_stream_t stream) {
  if (!rewards || !dones || !bootstrap_out || !returns || T <= 0 || E <= 0)
    return fail(VN_EINVAL, "vn_a2c_returns: bad args");
  hipLaunchKernelGGL(returns_kernel, dim3((E + 255) / 256), dim3(256), 0, (hipStream_t)stream, rewards, dones,
                     bootstrap_out, T, E, num_actions, gamma, returns);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_a2c_loss_grad(const float* out, const int32_t* actions, const float* returns, int n, int num_actions,
                     float value_coef, float entropy_coef, float* dout, float* stats4, vn_stream_t stream) {
  if (!out || !actions || !returns || !dout || !stats4 || n <= 0 || num_actions < 1 || num_actions > 7)
    return fail(VN_EINVAL, "vn_a2c_loss_grad: bad args");
  hipStream_t st = (hipStream_t)stream;
  VN_HIP(hipMemsetAsync(stats4, 0, 4 * sizeof(float), st));
  hipLaunchKernelGGL(loss_grad_kernel, dim3((n + 255) / 256), dim3(256), 0, st, out, actions, returns, n,
                     num_actions, value_coef, entropy_coef, 1.0f / (float)n, dout, stats4);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_grad_norm(const float* grads, int64_t n, float scale, float max_norm, double* partial_512, float* scalars2,
                 vn_stream_t stream) {
  if (!grads || !partial_512 || !scalars2 || n <= 0) return fail(VN_EINVAL, "vn_grad_norm: bad args");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3(kNormBlocks), dim3(256), 0, st, grads, n, scale, partial_512);
  hipLaunchKernelGGL(norm_final_kernel, dim3(1), dim3(256), 0, st, partial_512, kNormBlocks, max_norm, scalars2);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_grad_norm_join(float* grads, int64_t n, const float* add0, int64_t lo0, int64_t hi0, const float* add1,
                      int64_t lo1, int64_t hi1, float scale, float max_norm, double* partial_512, float* scalars2,
                      vn_stream_t stream) {
  if (!grads || !partial_512 || !scalars2 || n <= 0) return fail(VN_EINVAL, "vn_grad_norm_join: bad args");
  if ((add0 && (lo0 < 0 || hi0 > n || lo0 > hi0)) || (add1 && (lo1 < 0 || hi1 > n || lo1 > hi1)))
    return fail(VN_EINVAL, "vn_grad_norm_join: addend range outside [0, n)");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(sumsq_join_partial_kernel, dim3(kNormBlocks), dim3(256), 0, st, grads, n, scale, add0, lo0, hi0,
                     add1, lo1, hi1, partial_512);
  hipLaunchKernelGGL(norm_final_kernel, dim3(1), dim3(256), 0, st, partial_512, kNormBlocks, max_norm, scalars2);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_rmsprop_step(float* params, const float* grads, float* square_avg, int64_t n, float scale,
                    const float* scalars2, float lr, float alpha, float eps, vn_stream_t stream) {
  if (!params || !grads || !square_avg || !scalars2 || n <= 0) return fail(VN_EINVAL, "vn_rmsprop_step: bad args");
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(rmsprop_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, params, grads, square_avg, n,
                     scale, scalars2, lr, (const float*)nullptr, alpha, eps);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_rmsprop_step_dev(float* params, const float* grads, float* square_avg, int64_t n, float scale,
                        const float* scalars2, const float* lr_dev, float alpha, float eps, vn_stream_t stream) {
  if (!params || !grads || !square_avg || !scalars2 || !lr_dev || n <= 0)
    return fail(VN_EINVAL, "vn_rmsprop_step_dev: bad args");
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(rmsprop_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, params, grads, square_avg, n,
                     scale, scalars2, 0.0f, lr_dev, alpha, eps);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_a2c_step_post(const int32_t* actions, const float* rewards, const uint8_t* dones, const float* ep_return,
                     const int32_t* ep_length, int E, int num_actions, int64_t* prev_action, float* prev_reward,
                     float* prev_mask, float* lra_next, float* mask_next, float* episode_stats3, vn_stream_t stream) {
  if (!actions || !rewards || !dones || !ep_return || !ep_length || !episode_stats3 || E <= 0 || num_actions < 1)
    return fail(VN_EINVAL, "vn_a2c_step_post: bad args");
  hipLaunchKernelGGL(step_post_kernel, dim3(1), dim3(kPostThreads), 0, (hipStream_t)stream, actions, rewards, dones,
                     ep_return, ep_length, E, num_actions, prev_action, prev_reward, prev_mask, lra_next, mask_next,
                     episode_stats3);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

}  // extern "C"
