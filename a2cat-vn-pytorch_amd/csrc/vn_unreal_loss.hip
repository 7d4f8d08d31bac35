// vn_unreal_loss.hip — the UNREAL auxiliary losses of the trainer on gfx950: pixel control
// (n-step Q-learning on pixel-change pseudo-rewards), reward prediction (3-class
// cross-entropy on three consecutive frames) and value replay, with the weights of
// experiments/thor_cached_auxiliary.py:39-41 (rp 1.0, pc 0.05, vr 1.0).
//
// The loss formulas live in deep_rl's UnrealTrainer (deep-rl==0.2.9, absent from the image):
// parity unpinned. The restatement follows the published UNREAL algorithm (Jaderberg et al.
// 2016) as deep_rl's call sites use it: the pseudo-reward of step t is the mean over each
// 4x4 cell (pc_cell_size, goal.py:72) and the 3 channels of |obs_{t+1} - obs_t| on the
// centre crop of 42 x 4 pixels of the image observation (_get_input_for_pixel_control,
// thor_cached_auxiliary.py:47-48; obs scaled to [0,1] by ScaledFloatFrame), Q targets
// R_T = max_a Q(s_T), R_t = r_t + gamma_pc (1 - done_t) R_{t+1}, loss mean (Q(s_t, a_t) - R_t)^2;
// on a done step r_t = 0: the frame after it is the auto-reset frame of the next episode, so
// the pixel change across the boundary is not an effect of a_t (recorded deviation: the
// frame that ends the episode is never emitted by the batched env, DESIGN.md "Deviations");
// reward prediction classes (r = 0, r > 0, r < 0) of the reward after frame t from frames
// t-2, t-1, t of one episode; value replay mean (V - R)^2 against the n-step returns. The
// oracle is oracle/unreal.py.
#include <hip/hip_runtime.h>

#include "vn_common.h"

namespace vn {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kPcCells = 42;  // BigGoalHouseModel's pixel-control map (goal.py:103-112)
constexpr int kPcCellsBig = 20;  // BigHouseModel's (bignet.py:77-91, one k4 s2 layer on 9x9)
constexpr int kPcCellPx = 4;
constexpr int kPcChunk = 8;  // rollout steps whose loads unreal_pc_loss_kernel issues together

// Mean |f1 - f0| / 255 over cell (cy, cx)'s 4 x 4 pixels and 3 channels (u8 HWC frames).
__device__ __forceinline__ float pc_cell_change(const uint8_t* __restrict__ f0, const uint8_t* __restrict__ f1, int W,
                                                int top, int left, int cy, int cx) {
  int s = 0;
#pragma unroll
  for (int dy = 0; dy < kPcCellPx; ++dy) {
    const int64_t o = ((int64_t)(top + cy * kPcCellPx + dy) * W + left + cx * kPcCellPx) * 3;
#pragma unroll
    for (int j = 0; j < 3 * kPcCellPx; ++j) s += abs((int)f1[o + j] - (int)f0[o + j]);
  }
  return (float)s * (1.0f / (255.0f * 3 * kPcCellPx * kPcCellPx));
}

template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float t = 0.0f;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) t += red[w];
  __syncthreads();
  return t;
}

// One thread per (env e < S, cell): the Q targets backwards over the rollout. Reads the
// heads' maps p2 [(T+1) S][42][42][8] of vn_pc_forward (value channels 0..A-1, action channel A,
// after their ReLUs) and forms q_c = (v_c + a) - a on the fly (goal.py:136); overwrites p2 with
// dL/dp2: the TD gradient of the taken action's value channel under its ReLU, 0 elsewhere (the
// action channel's gradient is exactly 0, pc_dq_kernel) and on the bootstrap rows T S + e.
__device__ __forceinline__ void pc_load8(const float* p, float (&v)[8]) {
  const f4 lo = reinterpret_cast<const f4*>(p)[0], hi = reinterpret_cast<const f4*>(p)[1];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    v[c] = lo[c];
    v[4 + c] = hi[c];
  }
}

__global__ __launch_bounds__(256) void unreal_pc_loss_kernel(float* __restrict__ p2, const int32_t* __restrict__ actions,
                                                             const uint8_t* __restrict__ dones,
                                                             const uint8_t* __restrict__ arena, int64_t frame_bytes,
                                                             int H, int W, const int32_t* __restrict__ rows_img,
                                                             const int32_t* __restrict__ rows_last, int T, int E, int S,
                                                             int A, int cells, float gamma, float coef,
                                                             float* __restrict__ stats) {
  __shared__ float red[4];
  const int PP = cells * cells;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  float sq = 0.0f;
  if (idx < S * PP) {
    const int e = idx / PP, pix = idx - e * PP, cy = pix / cells, cx = pix - cy * cells;
    const int top = (H - cells * kPcCellPx) / 2, left = (W - cells * kPcCellPx) / 2;
    float v[8];
    float* pb = p2 + ((int64_t)(T * S + e) * PP + pix) * 8;
    pc_load8(pb, v);
    float a = v[0];
#pragma unroll
    for (int c = 1; c < 8; ++c)
      if (c == A) a = v[c];
    float R = -INFINITY;
#pragma unroll
    for (int c = 0; c < 7; ++c)
      if (c < A) R = fmaxf(R, (v[c] + a) - a);
    reinterpret_cast<f4*>(pb)[0] = f4{0.f, 0.f, 0.f, 0.f};
    reinterpret_cast<f4*>(pb)[1] = f4{0.f, 0.f, 0.f, 0.f};
    // steps in chunks of kPcChunk, latest first: a chunk's loads (frame rows, dones, actions,
    // the two channels of p2 it needs, the cells of both frames) are all issued before its
    // sequential part (the target recursion and the gradient stores), so a rollout costs
    // T / kPcChunk memory round trips instead of T (33 -> ~10 us at 4 envs)
    const uint8_t* fn = arena + (int64_t)rows_last[e] * frame_bytes;  // the frame after step t1
    for (int t1 = T - 1; t1 >= 0; t1 -= kPcChunk) {
      int64_t rowi[kPcChunk];
      int act[kPcChunk];
      bool done[kPcChunk];
#pragma unroll
      for (int k = 0; k < kPcChunk; ++k) {
        const int t = max(t1 - k, 0);  // (a step past the chunk's start repeats step 0; unused)
        const int64_t r = (int64_t)t * E + e;
        rowi[k] = rows_img[r];
        act[k] = actions[r];
        done[k] = dones[r] != 0;
      }
      float rew[kPcChunk], va[kPcChunk], at[kPcChunk];
#pragma unroll
      for (int k = 0; k < kPcChunk; ++k) {
        const int t = max(t1 - k, 0);
        const uint8_t* f = arena + rowi[k] * frame_bytes;
        const uint8_t* fx = k == 0 ? fn : arena + rowi[k - 1] * frame_bytes;
        rew[k] = done[k] ? 0.0f : pc_cell_change(f, fx, W, top, left, cy, cx);
        pc_load8(p2 + ((int64_t)(t * S + e) * PP + pix) * 8, v);
        float a8 = v[0], v8 = v[0];
#pragma unroll
        for (int c = 1; c < 8; ++c) {
          if (c == A) a8 = v[c];
          if (c == act[k]) v8 = v[c];
        }
        at[k] = a8;
        va[k] = v8;
      }
#pragma unroll
      for (int k = 0; k < kPcChunk; ++k) {
        const int t = t1 - k;
        if (t < 0) break;
        R = rew[k] + (done[k] ? 0.0f : gamma * R);
        const float d = ((va[k] + at[k]) - at[k]) - R;
        sq += d * d;
        const float g = va[k] > 0.0f ? 2.0f * coef * d : 0.0f;
        float o[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) o[c] = c == act[k] ? g : 0.0f;
        float* pt = p2 + ((int64_t)(t * S + e) * PP + pix) * 8;
        reinterpret_cast<f4*>(pt)[0] = f4{o[0], o[1], o[2], o[3]};
        reinterpret_cast<f4*>(pt)[1] = f4{o[4], o[5], o[6], o[7]};
      }
      fn = arena + rowi[kPcChunk - 1] * frame_bytes;
    }
  }
  const float t = block_sum<256>(sq, red);
  if (threadIdx.x == 0 && t != 0.0f) atomicAdd(stats, t);
}

// Reward prediction, one workgroup: sample j = (ts - 2) S + e (frames ts-2, ts-1, ts of env
// e, 2 <= ts < T) is used when no episode ends at ts-2 or ts-1; dlogits of the mean
// cross-entropy over the used samples, times the weight; stats[0] = the mean CE, stats[1] =
// the sample count.
constexpr int kRpThreads = 1024;
__global__ __launch_bounds__(kRpThreads) void unreal_rp_loss_kernel(const float* __restrict__ logits,
                                                                    const float* __restrict__ rewards,
                                                                    const uint8_t* __restrict__ dones, int T, int E, int S,
                                                                    float weight, float* __restrict__ dlogits,
                                                                    float* __restrict__ stats) {
  __shared__ float red[kRpThreads / 64];
  const int n = (T - 2) * S;
  float cnt = 0.0f;
  for (int j = threadIdx.x; j < n; j += kRpThreads) {
    const int ts = 2 + j / S, e = j % S;
    cnt += (dones[(int64_t)(ts - 2) * E + e] || dones[(int64_t)(ts - 1) * E + e]) ? 0.0f : 1.0f;
  }
  const float count = block_sum<kRpThreads>(cnt, red);
  const float inv = count > 0.0f ? 1.0f / count : 0.0f;
  float ce = 0.0f;
  for (int j = threadIdx.x; j < n; j += kRpThreads) {
    const int ts = 2 + j / S, e = j % S;
    const bool used = !(dones[(int64_t)(ts - 2) * E + e] || dones[(int64_t)(ts - 1) * E + e]);
    const float r = rewards[(int64_t)ts * E + e];
    const int cls = r == 0.0f ? 0 : (r > 0.0f ? 1 : 2);
    const float* l = logits + (int64_t)j * 4;
    const float m = fmaxf(l[0], fmaxf(l[1], l[2]));
    const float ex[3] = {expf(l[0] - m), expf(l[1] - m), expf(l[2] - m)};
    const float z = ex[0] + ex[1] + ex[2];
    float* g = dlogits + (int64_t)j * 4;
#pragma unroll
    for (int c = 0; c < 3; ++c) g[c] = used ? (ex[c] / z - (c == cls ? 1.0f : 0.0f)) * weight * inv : 0.0f;
    g[3] = 0.0f;
    if (used) ce += logf(z) + m - l[cls];
  }
  const float total = block_sum<kRpThreads>(ce, red);
  if (threadIdx.x == 0) {
    stats[0] = total * inv;
    stats[1] = count;
  }
}

// dX4 rows t*E + e (e < S) from the rp input gradient dx [(T-2) S][3][F]: frame t is slot
// 2 - k of sample ts = t + k (k = 0..2, 2 <= ts < T), summed in that order.
__global__ __launch_bounds__(256) void unreal_rp_scatter_kernel(const float* __restrict__ dx, int T, int E, int S, int F,
                                                                float* __restrict__ dx4, int accumulate) {
  const int F4 = F / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)T * S * F4) return;
  const int q4 = (int)(i % F4);
  const int te = (int)(i / F4), t = te / S, e = te - (te / S) * S;
  f4 v = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int ts = t + k;
    if (ts < 2 || ts >= T) continue;
    v += reinterpret_cast<const f4*>(dx + (((int64_t)(ts - 2) * S + e) * 3 + (2 - k)) * F)[q4];
  }
  f4* d = reinterpret_cast<f4*>(dx4 + ((int64_t)t * E + e) * F) + q4;
  *d = accumulate ? *d + v : v;
}

// Value replay on rows t*E + e (e < S): dout[.][A] += coef (V - R), stats += (V - R)^2.
__global__ __launch_bounds__(256) void unreal_vr_kernel(const float* __restrict__ out, const float* __restrict__ returns,
                                                        int T, int E, int S, int A, float coef,
                                                        float* __restrict__ dout, float* __restrict__ stats) {
  __shared__ float red[4];
  const int i = blockIdx.x * 256 + threadIdx.x;
  float sq = 0.0f;
  if (i < T * S) {
    const int t = i / S, e = i - t * S;
    const int64_t r = (int64_t)t * E + e;
    const float d = out[r * 8 + A] - returns[r];
    dout[r * 8 + A] += coef * d;
    sq = d * d;
  }
  const float t = block_sum<256>(sq, red);
  if (threadIdx.x == 0 && t != 0.0f) atomicAdd(stats, t);
}

// The UNREAL losses' inputs in one launch (they were five framework copies): h_pc rows
// t*S + e = h_all row t*E + e (t < T, e < S), rows T*S + e = boot_h row e; rp_x row
// (t*S + e) slot k = x4 row (t+k)*E + e (t < T - 2, k < 3). One 16-B lane per 4 floats.
__global__ __launch_bounds__(256) void unreal_gather_kernel(const float* __restrict__ h_all,
                                                            const float* __restrict__ boot_h,
                                                            const float* __restrict__ x4, int T, int E, int S, int F,
                                                            int nh, float* __restrict__ h_pc, float* __restrict__ rp_x) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n_h = (int64_t)nh * S * 128;  // 512 floats = 128 lanes per h row (nh = T + 1, or 0)
  if (i < n_h) {
    const int j = (int)(i >> 7), q = (int)(i & 127);
    const float* src = j < T * S ? h_all + ((int64_t)(j / S) * E + j % S) * 512 : boot_h + (int64_t)(j - T * S) * 512;
    reinterpret_cast<f4*>(h_pc + (int64_t)j * 512)[q] = reinterpret_cast<const f4*>(src)[q];
    return;
  }
  const int F4 = F / 4;
  const int64_t r = i - n_h;
  if (r >= (int64_t)(T - 2) * S * 3 * F4) return;
  const int q = (int)(r % F4);
  const int64_t js = r / F4;  // (sample, slot)
  const int k = (int)(js % 3), j = (int)(js / 3), t = j / S, e = j - (j / S) * S;
  reinterpret_cast<f4*>(rp_x + js * F)[q] = reinterpret_cast<const f4*>(x4 + ((int64_t)(t + k) * E + e) * F)[q];
}

}  // namespace vn

using namespace vn;

extern "C" {

int vn_unreal_pc_loss_grad_ex(float* p2, int cells, const int32_t* actions, const uint8_t* dones,
                              const uint8_t* arena, int64_t frame_bytes, int height, int width,
                              const int32_t* rows_img, const int32_t* rows_last, int T, int E, int S, int num_actions,
                              float gamma, float weight, float* stats, vn_stream_t stream) {
  if (!p2 || !actions || !dones || !arena || !rows_img || !rows_last || !stats || T <= 0 || S <= 0 || S > E ||
      (cells != kPcCells && cells != kPcCellsBig) || num_actions < 1 || num_actions > 7 ||
      height < cells * kPcCellPx || width < cells * kPcCellPx || frame_bytes < (int64_t)height * width * 3)
    return fail(VN_EINVAL, "vn_unreal_pc_loss_grad: bad args");
  const int n = S * cells * cells;
  const float coef = weight / ((float)T * n);
  hipLaunchKernelGGL(unreal_pc_loss_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, p2, actions,
                     dones, arena, frame_bytes, height, width, rows_img, rows_last, T, E, S, num_actions, cells, gamma,
                     coef, stats);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_unreal_pc_loss_grad(float* p2, const int32_t* actions, const uint8_t* dones, const uint8_t* arena,
                           int64_t frame_bytes, int height, int width, const int32_t* rows_img,
                           const int32_t* rows_last, int T, int E, int S, int num_actions, float gamma, float weight,
                           float* stats, vn_stream_t stream) {
  return vn_unreal_pc_loss_grad_ex(p2, kPcCells, actions, dones, arena, frame_bytes, height, width, rows_img, rows_last,
                                   T, E, S, num_actions, gamma, weight, stats, stream);
}

int vn_unreal_rp_loss_grad(const float* logits, const float* rewards, const uint8_t* dones, int T, int E, int S,
                           float weight, float* dlogits, float* stats2, vn_stream_t stream) {
  if (!logits || !rewards || !dones || !dlogits || !stats2 || T < 3 || S <= 0 || S > E)
    return fail(VN_EINVAL, "vn_unreal_rp_loss_grad: bad args (needs T >= 3)");
  hipLaunchKernelGGL(unreal_rp_loss_kernel, dim3(1), dim3(kRpThreads), 0, (hipStream_t)stream, logits, rewards, dones,
                     T, E, S, weight, dlogits, stats2);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_unreal_rp_scatter(const float* dx, int T, int E, int S, int fcin, float* dx4, int accumulate,
                         vn_stream_t stream) {
  if (!dx || !dx4 || T < 3 || S <= 0 || S > E || fcin <= 0 || fcin % 4)
    return fail(VN_EINVAL, "vn_unreal_rp_scatter: bad args");
  const int64_t total = (int64_t)T * S * (fcin / 4);
  hipLaunchKernelGGL(unreal_rp_scatter_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     dx, T, E, S, fcin, dx4, accumulate);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_unreal_gather(const float* h_all, const float* boot_h, const float* x4, int T, int E, int S, int fcin,
                     float* h_pc, float* rp_x, vn_stream_t stream) {
  if ((h_pc && (!h_all || !boot_h)) || (!h_pc && !rp_x) || T <= 0 || S <= 0 || S > E ||
      (rp_x && (!x4 || T < 3 || fcin <= 0 || fcin % 4)))
    return fail(VN_EINVAL, "vn_unreal_gather: bad args");
  const int nh = h_pc ? T + 1 : 0;  // h rows to copy (none when h_pc == NULL)
  const int64_t total = (int64_t)nh * S * 128 + (rp_x ? (int64_t)(T - 2) * S * 3 * (fcin / 4) : 0);
  hipLaunchKernelGGL(unreal_gather_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     h_all, boot_h, x4, T, E, S, rp_x ? fcin : 0, nh, h_pc, rp_x);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_unreal_vr_grad(const float* out, const float* returns, int T, int E, int S, int num_actions, float weight,
                      float* dout, float* stats, vn_stream_t stream) {
  if (!out || !returns || !dout || !stats || T <= 0 || S <= 0 || S > E || num_actions < 1 || num_actions > 7)
    return fail(VN_EINVAL, "vn_unreal_vr_grad: bad args");
  const float coef = 2.0f * weight / ((float)T * S);
  hipLaunchKernelGGL(unreal_vr_kernel, dim3((T * S + 255) / 256), dim3(256), 0, (hipStream_t)stream, out, returns, T, E,
                     S, num_actions, coef, dout, stats);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

}  // extern "C"
