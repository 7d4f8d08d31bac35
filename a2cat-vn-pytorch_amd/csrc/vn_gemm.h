// vn_gemm.h — fp32 MFMA tile core with operand-gather functors (gfx950).
//
// C[M][N] = sum_k A[m][k] * B[k][n], one 256-thread workgroup (4 waves, WM x WN) per
// BM x BN tile and K range. Both operands are staged in LDS k-contiguous
// ([row][k], row stride BK+4 floats) by "fill" functors that gather them straight
// from their producers (im2col of NHWC activations, uint8 frames addressed through
// scene-cache rows, transposed weights, ...). Each wave reads 16 B per lane
// (ds_read_b128: 4 consecutive k of one row) and issues four
// v_mfma_f32_16x16x4_f32 per read — MFMA j of a group covers k = {j, 4+j, 8+j, 12+j},
// the same permutation on both operands, so the product is unchanged. f32 in/f32
// accumulate is an exact fmaf chain (cdna_hip_programming.md §3). blockIdx.z splits the
// K range (split-K): the epilogue receives the split index so wgrad can write
// per-split slabs that a second pass reduces deterministically.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vn {

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 f4zero() { return f4{0.f, 0.f, 0.f, 0.f}; }

template <int BM, int BN, int BK, int WM, int WN, class FA, class FB, class EP>
__global__ __launch_bounds__(256) void gemm_kernel(FA fa, FB fb, EP ep, int M, int N, int K, int kchunk) {
  static_assert(WM * WN == 4, "4 waves per workgroup");
  static_assert(BK % 16 == 0, "BK multiple of 16");
  constexpr int LD = BK + 4;
  constexpr int TM = BM / (WM * 16), TN = BN / (WN * 16);
  static_assert(TM >= 1 && TN >= 1, "tile too small for the wave layout");
  __shared__ __attribute__((aligned(16))) float As[BM * LD];
  __shared__ __attribute__((aligned(16))) float Bs[BN * LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kb = blockIdx.z * kchunk;
  const int ke = min(K, kb + kchunk);
  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4zero();
  const int ra = (wm * TM * 16 + (lane & 15)) * LD + 4 * (lane >> 4);
  const int rb = (wn * TN * 16 + (lane & 15)) * LD + 4 * (lane >> 4);
  for (int k0 = kb; k0 < ke; k0 += BK) {
    fa.template fill<BM, BK>(As, m0, k0, ke, tid);
    fb.template fill<BN, BK>(Bs, n0, k0, ke, tid);
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; kk += 16) {
      f4 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = *reinterpret_cast<const f4*>(&As[ra + i * 16 * LD + kk]);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = *reinterpret_cast<const f4*>(&Bs[rb + j * 16 * LD + kk]);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][q], b[j][q], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * TM * 16 + i * 16 + (lane >> 4) * 4 + r;
        const int col = n0 + wn * TN * 16 + j * 16 + (lane & 15);
        if (row < M && col < N) ep(row, col, acc[i][j][r], (int)blockIdx.z);
      }
}

// ---- fill helpers -----------------------------------------------------------
// Row-major source: L::load4(row, k, kend) -> 4 consecutive k of one row (zeros past kend).
template <int ROWS, int BK, class L>
__device__ __forceinline__ void fill_rows(const L& l, float* s, int row0, int k0, int kend, int tid) {
  constexpr int LD = BK + 4, Q = BK / 4, SLOTS = ROWS * Q;
#pragma unroll
  for (int i = tid; i < SLOTS; i += 256) {
    const int r = i / Q, q = i - r * Q;
    *reinterpret_cast<f4*>(&s[r * LD + 4 * q]) = l.load4(row0 + r, k0 + 4 * q, kend);
  }
}

// Transposing source (wgrad): L::load4t(p, r) -> rows r..r+3 at reduction index p.
template <int ROWS, int BK, class L>
__device__ __forceinline__ void fill_trans(const L& l, float* s, int row0, int k0, int kend, int tid) {
  constexpr int LD = BK + 4, R4 = ROWS / 4, SLOTS = R4 * BK;
#pragma unroll
  for (int i = tid; i < SLOTS; i += 256) {
    const int kk = i / R4, rq = i - kk * R4;
    const int p = k0 + kk;
    const f4 v = (p < kend) ? l.load4t(p, row0 + 4 * rq) : f4zero();
    s[(4 * rq + 0) * LD + kk] = v[0];
    s[(4 * rq + 1) * LD + kk] = v[1];
    s[(4 * rq + 2) * LD + kk] = v[2];
    s[(4 * rq + 3) * LD + kk] = v[3];
  }
}

}  // namespace vn
