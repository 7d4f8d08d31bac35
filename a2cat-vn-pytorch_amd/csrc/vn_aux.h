// vn_aux.h — AuxiliaryBigGoalHouseModel's deconv heads (models/goal.py:144-189) and the
// auxiliary deconv loss of experiments/ai2_auxiliary/trainer.py:9-55, included by
// vn_policy.hip after the GEMM launch helpers.
//
// Heads: three TimeDistributed(ConvTranspose2d(32,16,k4,s2), ReLU, ConvTranspose2d(16,C,k4,s2))
// on the conv_base map X4 [n][h3][w3][32] for depth (C=1), segmentation (3) and goal
// segmentation (3). The three first layers share their input and run as ONE deconv with 48
// output channels; the second layers run as one deconv 48 -> 8 whose weight is block
// diagonal (head h reads channels 16h..16h+15 and writes depth 0, mask 1-3, goal mask 4-6;
// channel 7 is padding), so its off-block gradient is masked to keep them structural zeros.
//
// A stride-2 k4 transposed conv is computed as the parity-class "dgrad" product of the
// trunk's backward (DgradA/DgradB loaders): out pixel (2yy+py, 2xx+px) sums the 2x2 input
// taps that reach it. Its backward is a plain stride-2 conv (NhwcIm2col) for the input
// gradient and a split-K wgrad for the weights. Weights are stored [Cin][ky][kx][Cout].
#pragma once

namespace vn {

constexpr int kAuxC1 = 48;  // 3 heads x 16
constexpr int kAuxC2 = 8;   // depth 1 + mask 3 + goal mask 3 + pad
constexpr int kAuxCell = 4; // deconv_cell_size = pc_cell_size (goal.py:70,148)

// Output pixel (2yy + PY, 2xx + PX) of a transposed conv, bias (+ ReLU), NHWC.
template <int OH, int OW, int PY, int PX, int HYC, int WXC>
struct EpiDeconv {
  float* Y;
  int C;
  const float* bias;
  int relu;
  __device__ __forceinline__ void operator()(int row, int col, float v, int) const {
    constexpr int per = HYC * WXC;
    const int n = row / per;
    const int r = row - n * per;
    const int y = (r / WXC) * 2 + PY, x = (r % WXC) * 2 + PX;
    v += bias[col];
    Y[(((int64_t)n * OH + y) * OW + x) * C + col] = relu ? fmaxf(v, 0.0f) : v;
  }
};

// dX masked by the ReLU that produced X, plus an extra gradient on the same tensor (the
// aux heads' gradient w.r.t. the conv_base map), both under the mask.
struct EpiMaskAdd {
  float* out;
  const float* X;
  int64_t ld;
  const float* extra;
  __device__ __forceinline__ void operator()(int row, int col, float v, int) const {
    const int64_t i = (int64_t)row * ld + col;
    out[i] = X[i] > 0.0f ? v + extra[i] : 0.0f;
  }
};

// Head of output channel c of the second layer (-1 = padding channel).
__device__ __forceinline__ int aux_head_of_out(int c) { return c == 0 ? 0 : (c <= 3 ? 1 : (c <= 6 ? 2 : -1)); }

// Zero the off-block entries of dW2 [48][16][8] (block-diagonal second layer).
__global__ void aux_blockdiag_mask_kernel(float* __restrict__ dW2) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= kAuxC1 * 16 * kAuxC2) return;
  const int ci = idx / (16 * kAuxC2), co = idx % kAuxC2;
  if (aux_head_of_out(co) != ci / 16) dW2[idx] = 0.0f;
}

// Column sums of src [rows][cols] (cols <= 64), deterministic: per-block partials, then a
// fixed-order reduce.
__global__ void colsum_partial_kernel(const float* __restrict__ src, int64_t rows, int cols,
                                      float* __restrict__ partial) {
  __shared__ float sh[256];
  const int c = threadIdx.x % cols;
  const int lanes = blockDim.x / cols;  // row lanes per block
  const int l = threadIdx.x / cols;
  float s = 0.0f;
  if (l < lanes)
    for (int64_t r = (int64_t)blockIdx.x * lanes + l; r < rows; r += (int64_t)gridDim.x * lanes)
      s += src[r * cols + c];
  sh[threadIdx.x] = (l < lanes) ? s : 0.0f;
  __syncthreads();
  if (threadIdx.x < cols) {
    float t = 0.0f;
    for (int j = 0; j < lanes; ++j) t += sh[j * cols + threadIdx.x];
    partial[(int64_t)blockIdx.x * cols + threadIdx.x] = t;
  }
}

__global__ void colsum_final_kernel(const float* __restrict__ partial, int blocks, int cols, float* __restrict__ out) {
  const int c = threadIdx.x;
  if (c >= cols) return;
  float t = 0.0f;
  for (int b = 0; b < blocks; ++b) t += partial[(int64_t)b * cols + c];
  out[c] = t;
}

struct AuxTargets {
  const uint8_t* depth;   // [rows][H][W][1]
  const uint8_t* seg;     // [rows][H][W][3]
  const int32_t* img_rows;
  const int32_t* goal_rows;
  int H, W;
};

// Targets = avg_pool(centre crop(obs / 255), 4) (trainer.py:9-15) fused with the per-head
// MSE gradient: dP = weight * 2 (P - target) / numel(head); stats[h] += sum (P - target)^2.
__global__ void aux_loss_grad_kernel(int n, int PH, int PW, const float* __restrict__ P, AuxTargets tg, float weight,
                                     float* __restrict__ dP, float* __restrict__ stats) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float sq[3] = {0.0f, 0.0f, 0.0f};
  if (idx < (int64_t)n * PH * PW) {
    const int e = (int)(idx / (PH * PW));
    const int pix = (int)(idx - (int64_t)e * PH * PW);
    const int oy = pix / PW, ox = pix - (pix / PW) * PW;
    const int top = (tg.H - PH * kAuxCell) / 2, left = (tg.W - PW * kAuxCell) / 2;
    const int64_t HW = (int64_t)tg.H * tg.W;
    const uint8_t* dsrc = tg.depth + (int64_t)tg.img_rows[e] * HW;
    const uint8_t* ssrc = tg.seg + (int64_t)tg.img_rows[e] * HW * 3;
    const uint8_t* gsrc = tg.seg + (int64_t)tg.goal_rows[e] * HW * 3;
    float acc[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int dy = 0; dy < kAuxCell; ++dy) {
      const int64_t rowp = (int64_t)(top + oy * kAuxCell + dy) * tg.W + left + ox * kAuxCell;
      for (int dx = 0; dx < kAuxCell; ++dx) {
        const int64_t p = rowp + dx;
        acc[0] += (float)dsrc[p];
        for (int c = 0; c < 3; ++c) {
          acc[1 + c] += (float)ssrc[p * 3 + c];
          acc[4 + c] += (float)gsrc[p * 3 + c];
        }
      }
    }
    const float* pr = P + idx * kAuxC2;
    float* dp = dP + idx * kAuxC2;
    const float numel[3] = {(float)n * PH * PW, 3.0f * n * PH * PW, 3.0f * n * PH * PW};
    for (int c = 0; c < 7; ++c) {
      // avg_pool2d of x/255: sum / 16 of the float values (the reference divides first)
      const float t = acc[c] * (1.0f / 255.0f) * (1.0f / (kAuxCell * kAuxCell));
      const float d = pr[c] - t;
      const int h = c == 0 ? 0 : (c <= 3 ? 1 : 2);
      sq[h] += d * d;
      dp[c] = weight * 2.0f * d / numel[h];
    }
    dp[7] = 0.0f;
  }
  // wave reduction of the statistics, one atomic per wave and head
  for (int h = 0; h < 3; ++h) {
    float v = sq[h];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0 && v != 0.0f) atomicAdd(stats + h, v);
  }
}

}  // namespace vn
