// vn_lstm.h — the recurrent core MaskedRNN(nn.LSTM(512 + A + 1, 512)) of
// BigGoalHouseModel (models/goal.py:61-67, 91-92), included by vn_policy.hip.
//
// Step t (batch E): xcat_t = [features_t (512) | last reward/action (A+1) | pad | h_{t-1} m_t (512)]
// gates = xcat_t W_cat^T + b_ih + b_hh, W_cat = [W_ih | 0 | W_hh] (one GEMM, k-contiguous rows),
// PyTorch gate order (i, f, g, o); c_t = f (c_{t-1} m_t) + i g, h_t = o tanh(c_t).
// m_t = 0 where an episode starts at t (the MaskedRNN reset; its exact deep_rl semantics
// are not in the reference tree: parity unpinned). BPTT runs inside one rollout
// (states entering the rollout are constants). Only dh_{t-1} = m_t (dgates_t x W_hh) is
// sequential; the trunk's input gradient of all T steps (dgates x W_ih, features part) and
// the weight gradient (one split-K GEMM over T*E rows of [dgates | xcat]) run after the loop.
#pragma once

namespace vn {

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

__global__ void lstm_prep_kernel(int n, int A, int xcat, int xoff, const float* __restrict__ x5,
                                 const float* __restrict__ lra, const float* __restrict__ mask,
                                 const float* __restrict__ h_prev, float* __restrict__ xc) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)n * xcat) return;
  const int e = (int)(idx / xcat), j = (int)(idx - (idx / xcat) * xcat);
  float v = 0.0f;
  if (j < 512) {
    v = x5[(int64_t)e * 512 + j];
  } else if (j < 512 + A + 1) {
    v = lra ? lra[(int64_t)e * (A + 1) + (j - 512)] : 0.0f;
  } else if (j >= xoff) {
    const float m = mask ? mask[e] : 1.0f;
    v = h_prev ? h_prev[(int64_t)e * 512 + (j - xoff)] * m : 0.0f;
  }
  xc[idx] = v;
}

__global__ void lstm_cell_kernel(int n, const float* __restrict__ gates, const float* __restrict__ c_prev,
                                 const float* __restrict__ mask, float* __restrict__ acts, float* __restrict__ c_out,
                                 float* __restrict__ h_out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)n * 512) return;
  const int e = (int)(idx >> 9), j = (int)(idx & 511);
  const float m = mask ? mask[e] : 1.0f;
  const float cp = c_prev ? c_prev[idx] * m : 0.0f;
  const float* g4 = gates + (int64_t)e * 2048;
  const float i = sigmoidf_(g4[j]), f = sigmoidf_(g4[512 + j]), g = tanhf(g4[1024 + j]), o = sigmoidf_(g4[1536 + j]);
  const float c = f * cp + i * g;
  const float h = o * tanhf(c);
  float* a4 = acts + (int64_t)e * 2048;
  a4[j] = i;
  a4[512 + j] = f;
  a4[1024 + j] = g;
  a4[1536 + j] = o;
  c_out[idx] = c;
  h_out[idx] = h;
}

__global__ void lstm_cell_bwd_kernel(int n, const float* __restrict__ dh_heads, const float* __restrict__ dh_next,
                                     const float* __restrict__ dc_next, const float* __restrict__ acts,
                                     const float* __restrict__ c, const float* __restrict__ c_prev,
                                     const float* __restrict__ mask, float* __restrict__ dgates,
                                     float* __restrict__ dc_prev_out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)n * 512) return;
  const int e = (int)(idx >> 9), j = (int)(idx & 511);
  const float m = mask ? mask[e] : 1.0f;
  const float* a4 = acts + (int64_t)e * 2048;
  const float i = a4[j], f = a4[512 + j], g = a4[1024 + j], o = a4[1536 + j];
  const float tc = tanhf(c[idx]);
  const float dh = dh_heads[idx] + (dh_next ? dh_next[idx] : 0.0f);
  const float dc = (dc_next ? dc_next[idx] : 0.0f) + dh * o * (1.0f - tc * tc);
  const float cp = c_prev ? c_prev[idx] * m : 0.0f;
  float* d4 = dgates + (int64_t)e * 2048;
  d4[j] = dc * g * i * (1.0f - i);
  d4[512 + j] = dc * cp * f * (1.0f - f);
  d4[1024 + j] = dc * i * (1.0f - g * g);
  d4[1536 + j] = dh * tc * o * (1.0f - o);
  dc_prev_out[idx] = dc * f * m;
}

// Epilogue of the per-step recurrent product dh_{t-1} = m_t (dgates_t x W_hh).
struct EpiLstmDh {
  float* dh_prev;
  const float* mask;
  __device__ __forceinline__ float pre_row(int row) const { return mask ? mask[row] : 1.0f; }
  __device__ __forceinline__ void post(int row, int col, float v, float m, int) const {
    dh_prev[(int64_t)row * 512 + col] = v * m;
  }
};

struct EpiBias2 {
  float* Y;
  int64_t ld;
  const float* b0;
  const float* b1;
  __device__ __forceinline__ float2 pre_col(int col) const { return float2{b0[col], b1[col]}; }
  __device__ __forceinline__ void post(int row, int col, float v, float2 b, int) const {
    Y[(int64_t)row * ld + col] = v + b.x + b.y;
  }
};

struct EpiStore {
  float* Y;
  int64_t ld;
  __device__ __forceinline__ void operator()(int row, int col, float v, int) const { Y[(int64_t)row * ld + col] = v; }
};

}  // namespace vn
