// vn_unreal.h — BigGoalHouseModel's UNREAL heads (models/goal.py:94-133): pixel control
// (pc_base Linear(512, 32*9*9) + ReLU, then pc_value / pc_action as two stacked k4 s2
// transposed convs with ReLUs, combined as value + action - mean(action)) and reward
// prediction (Linear(3 * 9*9*32, 3) on three frames' conv_base maps). Included by
// vn_policy.hip after the aux heads (vn_aux.h: deconv products, column sums).
//
// Layout of the pixel-control maps (NHWC, like the trunk):
//   pcb [n][9][9][32]      pc_base output (the reference views Linear's 2592 outputs as
//                          (32, 9, 9): our rows of W are permuted to (y, x, c) order),
//   a1  [n][20][20][64]    both first deconvs side by side: pc_value 0-31, pc_action 32-63,
//   p2  [n][42][42][8]     both second deconvs (block diagonal W2): pc_value's A channels
//                          0..A-1 from a1 channels 0-31, pc_action's one channel A from 32-63,
//                          A+1..7 padding,
//   q   [n][42][42][A]     (value + action) - action, in the reference's evaluation order.
// BigHouseModel's heads (models/bignet.py:77-111) have one k4 s2 layer per branch: pcb -> p2
// [n][20][20][8] directly (W1 [32][4][4][8] with the same channel roles), no a1; the same
// combination and loss kernels run on the 20x20 map (pc_forward_impl / pc_backward_impl).
#pragma once

namespace vn {

constexpr int kPcC1 = 64;   // pc_value 32 + pc_action 32 first-layer channels
constexpr int kPcC2 = 8;    // pc_value A + pc_action 1 + padding
constexpr int kPcMap = 9;   // pc_base map 9x9x32 (goal.py:96, 134)
constexpr int kPcA1 = 20;   // 2 * 9 + 2
constexpr int kPcP = 42;    // 2 * 20 + 2
constexpr int kPcBase = kPcMap * kPcMap * 32;  // 2592

// q = (v + a) - mean_c(a) with one action channel: mean(a) = a (goal.py:136).
__global__ __launch_bounds__(256) void pc_combine_kernel(const float* __restrict__ p2, int64_t npix, int A,
                                                         float* __restrict__ q) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= npix) return;
  const f4 lo = *reinterpret_cast<const f4*>(p2 + p * kPcC2);
  const f4 hi = *reinterpret_cast<const f4*>(p2 + p * kPcC2 + 4);
  const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  float a = v[0];
#pragma unroll
  for (int c = 1; c < 8; ++c)
    if (c == A) a = v[c];
  for (int c = 0; c < A; ++c) q[p * A + c] = (v[c] + a) - a;
}

// dP2 over p2 in place: dq under the value ReLU for channels 0..A-1; the action channel's
// gradient is dq summed over the channels (the broadcast add) minus the same sum (the mean):
// exactly 0, as torch's autograd computes it; padding 0.
__global__ __launch_bounds__(256) void pc_dq_kernel(float* __restrict__ p2, const float* __restrict__ dq, int64_t npix,
                                                    int A) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= npix) return;
  f4* pp = reinterpret_cast<f4*>(p2 + p * kPcC2);
  const f4 lo = pp[0], hi = pp[1];
  const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  float g[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) g[c] = (c < A && v[c] > 0.0f) ? dq[p * A + (c < A ? c : 0)] : 0.0f;
  pp[0] = f4{g[0], g[1], g[2], g[3]};
  pp[1] = f4{g[4], g[5], g[6], g[7]};
}

// Zero the off-block entries of dW2 [64][16][8]: value rows 0-31 feed channels 0..A-1,
// action rows 32-63 feed channel A.
__global__ void pc_blockdiag_mask_kernel(float* __restrict__ dW2, int A) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= kPcC1 * 16 * kPcC2) return;
  const int ci = idx / (16 * kPcC2), co = idx % kPcC2;
  const bool live = ci < 32 ? co < A : co == A;
  if (!live) dW2[idx] = 0.0f;
}

// Reward prediction's input gradient dx [n][K] = dout [n][4] (3 logits + pad) x W [3][K]:
// K 3-term dot products per row, a fixed order, float4 along K.
__global__ __launch_bounds__(256) void rp_dx_kernel(const float* __restrict__ dout, const float* __restrict__ W, int n,
                                                    int K, float* __restrict__ dx) {
  const int K4 = K / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)n * K4) return;
  const int r = (int)(i / K4), k4 = (int)(i - (int64_t)r * K4);
  const f4 d = *reinterpret_cast<const f4*>(dout + (int64_t)r * 4);
  const f4 w0 = reinterpret_cast<const f4*>(W)[k4];
  const f4 w1 = reinterpret_cast<const f4*>(W + K)[k4];
  const f4 w2 = reinterpret_cast<const f4*>(W + 2 * K)[k4];
  f4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = fmaf(d[2], w2[j], fmaf(d[1], w1[j], d[0] * w0[j]));
  reinterpret_cast<f4*>(dx + (int64_t)r * K)[k4] = o;
}

// Y (+)= v: the pixel-control input gradient, added to the caller's dh when accumulating.
struct EpiAcc {
  float* Y;
  int64_t ld;
  int acc;
  __device__ __forceinline__ void operator()(int row, int col, float v, int) const {
    float* y = Y + (int64_t)row * ld + col;
    *y = acc ? *y + v : v;
  }
};

// dst rows t*E + e (e < S) += src rows t*S + e: [T][S][C] into [T][E][C] (C % 4 == 0); the
// LSTM backward's extra output gradient of the first S envs (pixel control).
__global__ __launch_bounds__(256) void add_env_rows_kernel(const float* __restrict__ src, int T, int E, int S, int C,
                                                           float* __restrict__ dst) {
  const int C4 = C / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)T * S * C4) return;
  const int c4 = (int)(i % C4);
  const int ts = (int)(i / C4), t = ts / S, e = ts - (ts / S) * S;
  f4* d = reinterpret_cast<f4*>(dst + ((int64_t)t * E + e) * C) + c4;
  *d += reinterpret_cast<const f4*>(src + (int64_t)ts * C)[c4];
}

}  // namespace vn
