// vn_gemm.h — fp32 MFMA tile core with operand-gather functors (gfx950).
//
// C[M][N] = sum_k A[m][k] * B[k][n], one 256-thread workgroup (4 waves, WM x WN) per
// BM x BN tile and K range. Both operands are staged in LDS k-contiguous
// ([row][k], row stride BK+8 floats: with it the four 16-lane groups of a
// ds_read_b128 hit 16 distinct 4-bank slots, MI355X_MICROARCH.md §LDS) by loader functors that gather them straight
// from their producers (im2col of NHWC activations, uint8 frames addressed through
// scene-cache rows, transposed weights, ...): fetch() issues the next K tile's global
// loads into registers before the current tile's MFMAs, commit() writes them to LDS
// after the barrier (a register-staged software pipeline). Each wave reads 16 B per lane
// (ds_read_b128: 4 consecutive k of one row) and issues four
// v_mfma_f32_16x16x4_f32 per read — MFMA j of a group covers k = {j, 4+j, 8+j, 12+j},
// the same permutation on both operands, so the product is unchanged. f32 in/f32
// accumulate is an exact fmaf chain (cdna_hip_programming.md §3). blockIdx.z splits the
// K range (split-K): the epilogue receives the split index so wgrad can write
// per-split slabs that a second pass reduces deterministically.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace vn {

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 f4zero() { return f4{0.f, 0.f, 0.f, 0.f}; }

// Two-phase epilogues: a functor's side inputs (bias, the producing activation of a ReLU
// mask, ...) are all loaded before the stores that use them, then post(row, col, v, side,
// split) stores. With one load per element inside the store loop, every load waited on
// vmcnt, which on gfx950 also counts the tile's earlier stores: the epilogue ran one memory
// round trip per element. A functor says what its side input depends on: pre_col(col) (one
// value per tile column: loaded once per j), pre_row(row) (once per row), or pre(row, col)
// (per element: loaded one i-slice of the tile at a time to bound the registers held).
template <class E, class = void>
struct has_pre : std::false_type {};
template <class E>
struct has_pre<E, std::void_t<decltype(&E::pre)>> : std::true_type {};
template <class E, class = void>
struct has_pre_col : std::false_type {};
template <class E>
struct has_pre_col<E, std::void_t<decltype(&E::pre_col)>> : std::true_type {};
template <class E, class = void>
struct has_pre_row : std::false_type {};
template <class E>
struct has_pre_row<E, std::void_t<decltype(&E::pre_row)>> : std::true_type {};
// A loader whose valid rows end at a device-side count (row_limit(), wave-uniform): tiles at
// or past it return at once and the epilogue stores no row at or past it (the grid is sized
// for the host's upper bound — goal-frame deduplication's device-side frame counts).
template <class L, class = void>
struct has_row_limit : std::false_type {};
template <class L>
struct has_row_limit<L, std::void_t<decltype(&L::row_limit)>> : std::true_type {};

// Epilogue over an accumulator tile: NR values per (i, j) whose (row, col) come from rc; the
// column of a value depends on j (and the lane) only, its row on i and r only.
template <int TM, int TN, int NR, class EP, class ACC, class RC>
__device__ __forceinline__ void run_epilogue(const EP& ep, const ACC& acc, int M, int N, int z, RC rc) {
  if constexpr (has_pre_col<EP>::value) {
    using PT = decltype(ep.pre_col(0));
    PT pv[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int row, col;
      rc(0, j, 0, row, col);
      if (col < N) pv[j] = ep.pre_col(col);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          int row, col;
          rc(i, j, r, row, col);
          if (row < M && col < N) ep.post(row, col, acc[i][j][r], pv[j], z);
        }
  } else if constexpr (has_pre_row<EP>::value) {
    using PT = decltype(ep.pre_row(0));
    PT pv[TM][NR];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        int row, col;
        rc(i, 0, r, row, col);
        if (row < M) pv[i][r] = ep.pre_row(row);
      }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          int row, col;
          rc(i, j, r, row, col);
          if (row < M && col < N) ep.post(row, col, acc[i][j][r], pv[i][r], z);
        }
  } else if constexpr (has_pre<EP>::value) {
    using PT = decltype(ep.pre(0, 0));
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      PT pv[TN][NR];
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          int row, col;
          rc(i, j, r, row, col);
          if (row < M && col < N) pv[j][r] = ep.pre(row, col);
        }
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          int row, col;
          rc(i, j, r, row, col);
          if (row < M && col < N) ep.post(row, col, acc[i][j][r], pv[j][r], z);
        }
    }
  } else {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          int row, col;
          rc(i, j, r, row, col);
          if (row < M && col < N) ep(row, col, acc[i][j][r], z);
        }
  }
}

template <int BM, int BN, int BK, int WM, int WN, class FA, class FB, class EP>
__global__ __launch_bounds__(256) void gemm_kernel(FA fa, FB fb, EP ep, int M, int N, int K, int kchunk) {
  static_assert(WM * WN == 4, "4 waves per workgroup");
  static_assert(BK % 16 == 0, "BK multiple of 16");
  // LDS row stride: BK+8 makes the ds_read_b128 groups conflict-free; transposed fills
  // (wgrad) need BK+4 for conflict-free scalar writes (fetch_trans)
  constexpr int LD = (FA::kTrans || FB::kTrans) ? BK + 4 : BK + 8;
  constexpr int TM = BM / (WM * 16), TN = BN / (WN * 16);
  static_assert(TM >= 1 && TN >= 1, "tile too small for the wave layout");
  constexpr int NA = (FA::template slots<BM, BK>() + 255) / 256;
  constexpr int NB = (FB::template slots<BN, BK>() + 255) / 256;
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
  // software pipeline: the next K tile's global loads are in flight while this one computes
  f4 pa[NA], pb[NB];
  if (kb < ke) {
    fa.template fetch<BM, BK>(pa, m0, kb, ke, tid);
    fb.template fetch<BN, BK>(pb, n0, kb, ke, tid);
  }
  for (int k0 = kb; k0 < ke; k0 += BK) {
    FA::template commit<BM, BK, LD>(pa, As, tid);
    FB::template commit<BN, BK, LD>(pb, Bs, tid);
    __syncthreads();
    if (k0 + BK < ke) {
      fa.template fetch<BM, BK>(pa, m0, k0 + BK, ke, tid);
      fb.template fetch<BN, BK>(pb, n0, k0 + BK, ke, tid);
    }
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
  run_epilogue<TM, TN, 4>(ep, acc, M, N, (int)blockIdx.z, [&](int i, int j, int r, int& row, int& col) {
    row = m0 + wm * TM * 16 + i * 16 + (lane >> 4) * 4 + r;
    col = n0 + wn * TN * 16 + j * 16 + (lane & 15);
  });
}

// Same core on v_mfma_f32_32x32x2_f32 (64-cycle issue = 64-cycle latency: one accumulator
// chain per 32x32 block runs at the full rate). Lane l reads 4 consecutive k of row l&31
// at k offset 4*(l>>5) (ds_read_b128); MFMA j of a group covers k = {j, 4+j}. With the
// row stride BK+4 the four 16-lane groups of a ds_read_b128 hit 16 distinct 4-bank slots.
// C layout: row = (r&3) + 8*(r>>2) + 4*(l>>5), col = l&31.
template <int BM, int BN, int BK, int WM, int WN, class FA, class FB, class EP>
__global__ __launch_bounds__(256) void gemm32_kernel(FA fa, FB fb, EP ep, int M, int N, int K, int kchunk) {
  static_assert(WM * WN == 4, "4 waves per workgroup");
  static_assert(BK % 8 == 0, "BK multiple of 8");
  constexpr int LD = BK + 4;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  static_assert(TM >= 1 && TN >= 1, "tile too small for the wave layout");
  constexpr int NA = (FA::template slots<BM, BK>() + 255) / 256;
  constexpr int NB = (FB::template slots<BN, BK>() + 255) / 256;
  __shared__ __attribute__((aligned(16))) float As[BM * LD];
  __shared__ __attribute__((aligned(16))) float Bs[BN * LD];
  typedef float f16v_ __attribute__((ext_vector_type(16)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kb = blockIdx.z * kchunk;
  const int ke = min(K, kb + kchunk);
  f16v_ acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  const int ra = (wm * TM * 32 + (lane & 31)) * LD + 4 * (lane >> 5);
  const int rb = (wn * TN * 32 + (lane & 31)) * LD + 4 * (lane >> 5);
  f4 pa[NA], pb[NB];
  if (kb < ke) {
    fa.template fetch<BM, BK>(pa, m0, kb, ke, tid);
    fb.template fetch<BN, BK>(pb, n0, kb, ke, tid);
  }
  for (int k0 = kb; k0 < ke; k0 += BK) {
    FA::template commit<BM, BK, LD>(pa, As, tid);
    FB::template commit<BN, BK, LD>(pb, Bs, tid);
    __syncthreads();
    if (k0 + BK < ke) {
      fa.template fetch<BM, BK>(pa, m0, k0 + BK, ke, tid);
      fb.template fetch<BN, BK>(pb, n0, k0 + BK, ke, tid);
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += 8) {
      f4 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = *reinterpret_cast<const f4*>(&As[ra + i * 32 * LD + kk]);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = *reinterpret_cast<const f4*>(&Bs[rb + j * 32 * LD + kk]);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][q], b[j][q], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  run_epilogue<TM, TN, 16>(ep, acc, M, N, (int)blockIdx.z, [&](int i, int j, int r, int& row, int& col) {
    row = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    col = n0 + wn * TN * 32 + j * 32 + (lane & 31);
  });
}

// ---- fp32 GEMM on bf16 MFMA with split operands ("x6") ---------------------------
// Each fp32 operand value v is split by truncation into three bf16 terms v0 + v1 + v2 == v
// (exact, split3 below); a*b is summed as the six term products with i + j <= 2 (the three
// dropped ones are below 2^-24 |a b|), each exact in fp32, on v_mfma_f32_32x32x16_bf16 (16x
// the f32 MFMA rate; 6 of them cost 0.375 of the f32 path). Row-fill loaders only: commit
// splits a k-contiguous f4 into three 8-byte bf16 runs of planes [term][row][k] (row
// stride BK + 8 elements: 20-dword rows put the 16-lane groups of a ds_read_b128 on 16
// distinct slots). Lane l reads row l&31, k = 8*(l>>5)..+7 (the MFMA A/B layout).
typedef __bf16 bf16x8_ __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint32_t bf16_split_bits(float v, float& rest) {
  const uint32_t hb = __float_as_uint(v) & 0xffff0000u;
  rest = v - __uint_as_float(hb);
  return hb >> 16;
}

// Row-fill slot i -> (row rr, quad q). With 8 quads a row (BK = 32) the 16 lanes of a
// ds_write_b64 group hold rows rr and rr + 4 of an 8-row block, not rr and rr + 1: their
// 8-byte runs start 4 LDK / 2 = 80 dwords apart (16 mod 32, LDK = 40) instead of 20, so the
// two rows' 16 dwords each land on disjoint banks (tools/gemm_banks.py: 1 -> 0 extra cycles
// per group). Fetch and commit share it; global reads stay 128-B row runs.
template <int ROWS, int Q>
__device__ __forceinline__ void rows_slot(int i, int& rr, int& q) {
  if constexpr (Q == 8 && ROWS % 8 == 0) {
    rr = ((i >> 6) << 3) | (((i >> 3) & 1) << 2) | ((i >> 4) & 3);
    q = i & 7;
  } else {
    rr = i / Q;
    q = i - (i / Q) * Q;
  }
}

template <int ROWS, int BK, int LDK>
__device__ __forceinline__ void commit_rows_x6(const f4* r, uint16_t* s, int tid) {
  constexpr int Q = BK / 4, T = ROWS * Q, NS = (T + 255) / 256, PLANE = ROWS * LDK;
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int i = tid + j * 256;
    if (T % 256 == 0 || i < T) {
      int rr, q;
      rows_slot<ROWS, Q>(i, rr, q);
      uint32_t t0[4], t1[4], t2[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float r1, r2, r3;
        t0[e] = bf16_split_bits(r[j][e], r1);
        t1[e] = bf16_split_bits(r1, r2);
        t2[e] = bf16_split_bits(r2, r3);
      }
      uint16_t* d = s + rr * LDK + 4 * q;
      *reinterpret_cast<uint2*>(d) = uint2{t0[0] | (t0[1] << 16), t0[2] | (t0[3] << 16)};
      *reinterpret_cast<uint2*>(d + PLANE) = uint2{t1[0] | (t1[1] << 16), t1[2] | (t1[3] << 16)};
      *reinterpret_cast<uint2*>(d + 2 * PLANE) = uint2{t2[0] | (t2[1] << 16), t2[2] | (t2[3] << 16)};
    }
  }
}

// Transposing source (wgrad: both operands gathered along the reduction index): the 4 rows
// of slot i at k = kk are split and stored k-major — planes [term][k][row] with row stride
// trans_ld(ROWS) — as one 8-byte run per term (the former row-major image took twelve 2-byte
// LDS stores per slot); the MFMA loop reads its fragments back with the hardware transpose
// read (frag_tr below).
constexpr int trans_ld(int rows) {  // 4 rows of a 32-lane half of ds_read_b64_tr_b16 on distinct banks
  return (rows * 2) % 128 == 0 ? rows + 32 : rows;
}

// x6 slot i -> (k = kk, row quad rq): G = min(ROWS / 4, 16) consecutive lanes take G
// consecutive row quads of one k, so a 16-lane ds_write_b64 group writes 32 consecutive
// dwords of one k row (the f32 path's pairs of quads over 8 k put 4 lanes on each bank
// pair: 3 extra cycles per group, tools/gemm_banks.py); a lane group's global reads are
// G * 16 contiguous bytes of one reduction index.
template <int ROWS, int BK>
__device__ __forceinline__ void trans_slot_x6(int i, int& kk, int& rq) {
  constexpr int G = ROWS / 4 < 16 ? ROWS / 4 : 16;
  static_assert((ROWS / 4) % G == 0, "row quads in groups");
  kk = (i / G) % BK;
  rq = i % G + G * (i / (G * BK));
}

template <int ROWS, int BK, class L>
__device__ __forceinline__ void fetch_trans_x6(const L& l, f4* r, int row0, int k0, int kend, int tid) {
  constexpr int R4 = ROWS / 4, T = R4 * BK, NS = (T + 255) / 256;
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int i = tid + j * 256;
    if (T % 256 == 0 || i < T) {
      int kk, rq;
      trans_slot_x6<ROWS, BK>(i, kk, rq);
      const int p = k0 + kk;
      r[j] = (p < kend) ? l.load4t(p, row0 + 4 * rq) : f4zero();
    }
  }
}

template <int ROWS, int BK, class L>
__device__ __forceinline__ void fetch_x6(const L& l, f4* r, int row0, int k0, int kend, int tid) {
  if constexpr (L::kTrans)
    fetch_trans_x6<ROWS, BK>(l, r, row0, k0, kend, tid);
  else
    l.template fetch<ROWS, BK>(r, row0, k0, kend, tid);
}

template <int ROWS, int BK>
__device__ __forceinline__ void commit_trans_x6(const f4* r, uint16_t* s, int tid) {
  constexpr int R4 = ROWS / 4, T = R4 * BK, NS = (T + 255) / 256, LDT = trans_ld(ROWS), PLANE = BK * LDT;
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int i = tid + j * 256;
    if (T % 256 == 0 || i < T) {
      int kk, rq;
      trans_slot_x6<ROWS, BK>(i, kk, rq);
      uint32_t t0[4], t1[4], t2[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float r1, r2, r3;
        t0[e] = bf16_split_bits(r[j][e], r1);
        t1[e] = bf16_split_bits(r1, r2);
        t2[e] = bf16_split_bits(r2, r3);
      }
      uint16_t* d = s + kk * LDT + 4 * rq;
      *reinterpret_cast<uint2*>(d) = uint2{t0[0] | (t0[1] << 16), t0[2] | (t0[3] << 16)};
      *reinterpret_cast<uint2*>(d + PLANE) = uint2{t1[0] | (t1[1] << 16), t1[2] | (t1[3] << 16)};
      *reinterpret_cast<uint2*>(d + 2 * PLANE) = uint2{t2[0] | (t2[1] << 16), t2[2] | (t2[3] << 16)};
    }
  }
}

template <int ROWS, int BK, int LDK, class L>
__device__ __forceinline__ void commit_x6(const f4* r, uint16_t* s, int tid) {
  if constexpr (L::kTrans)
    commit_trans_x6<ROWS, BK>(r, s, tid);
  else
    commit_rows_x6<ROWS, BK, LDK>(r, s, tid);
}

// The 32x32x16 fragment (row m0 + (l & 31), k = kk + 8(l >> 5) .. +7) of a k-major plane
// [k][LDT] via two ds_read_b64_tr_b16: in each 16-lane group, lane 4q + p addresses row
// k0 + q, columns 4p .. 4p+3 of the group's 16 columns, and lane i receives column i of the
// four k rows (element q = k0 + q). Uniform control flow only (the read gathers across lanes).
typedef short s16x4_ __attribute__((ext_vector_type(4)));
template <int LDT>
__device__ __forceinline__ bf16x8_ frag_tr(const uint16_t* plane, int m0, int kk, int lane) {
  const int q = (lane >> 2) & 3, p = lane & 3, g = (lane >> 4) & 1, h = lane >> 5;
  const uint16_t* a = plane + (kk + 8 * h + q) * LDT + m0 + 16 * g + 4 * p;
  typedef __attribute__((address_space(3))) s16x4_ lds_s16x4;
  const s16x4_ lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a));
  const s16x4_ hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 4 * LDT));
  union { s16x4_ s[2]; bf16x8_ v; } u;
  u.s[0] = lo;
  u.s[1] = hi;
  return u.v;
}

template <int BM, int BN, int BK, int WM, int WN, class FA, class FB, class EP>
__global__ __launch_bounds__(256) void gemm_x6_kernel(FA fa, FB fb, EP ep, int M, int N, int K, int kchunk) {
  static_assert(WM * WN == 4, "4 waves per workgroup");
  static_assert(BK % 16 == 0, "BK multiple of 16");
  constexpr int LDK = BK + 8;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  static_assert(TM >= 1 && TN >= 1, "tile too small for the wave layout");
  constexpr int NA = (FA::template slots<BM, BK>() + 255) / 256;
  constexpr int NB = (FB::template slots<BN, BK>() + 255) / 256;
  // row-major planes [term][row][LDK], or k-major [term][k][trans_ld(rows)] for a transposing loader
  constexpr int LTA = trans_ld(BM), LTB = trans_ld(BN);
  constexpr int PA = FA::kTrans ? BK * LTA : BM * LDK, PB = FB::kTrans ? BK * LTB : BN * LDK;
  __shared__ __attribute__((aligned(16))) uint16_t As[3 * PA];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[3 * PB];
  typedef float f16v_ __attribute__((ext_vector_type(16)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  if constexpr (has_row_limit<FA>::value) {  // uniform: the whole workgroup leaves together
    const int lim = fa.row_limit();
    if (m0 >= lim) return;
    M = min(M, lim);
  }
  const int kb = blockIdx.z * kchunk;
  const int ke = min(K, kb + kchunk);
  f16v_ acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  const int ra = (wm * TM * 32 + (lane & 31)) * LDK + 8 * (lane >> 5);
  const int rb = (wn * TN * 32 + (lane & 31)) * LDK + 8 * (lane >> 5);
  f4 pa[NA], pb[NB];
  if (kb < ke) {
    fetch_x6<BM, BK>(fa, pa, m0, kb, ke, tid);
    fetch_x6<BN, BK>(fb, pb, n0, kb, ke, tid);
  }
  for (int k0 = kb; k0 < ke; k0 += BK) {
    commit_x6<BM, BK, LDK, FA>(pa, As, tid);
    commit_x6<BN, BK, LDK, FB>(pb, Bs, tid);
    __syncthreads();
    if (k0 + BK < ke) {
      fetch_x6<BM, BK>(fa, pa, m0, k0 + BK, ke, tid);
      fetch_x6<BN, BK>(fb, pb, n0, k0 + BK, ke, tid);
    }
    // the MFMA cluster at raised wave priority: the co-resident workgroup's wave on this SIMD
    // then runs its commit (VALU split, LDS writes) in this wave's MFMA gaps instead of
    // delaying its MFMA issue (tools/gemm_x6_bench.hip, LSTM gates shape: 117 -> 102 us)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 16) {
      bf16x8_ a[3][TM], b[3][TN];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          if constexpr (FA::kTrans)
            a[t][i] = frag_tr<LTA>(As + t * PA, wm * TM * 32 + i * 32, kk, lane);
          else
            a[t][i] = *reinterpret_cast<const bf16x8_*>(&As[t * PA + ra + i * 32 * LDK + kk]);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (FB::kTrans)
            b[t][j] = frag_tr<LTB>(Bs + t * PB, wn * TN * 32 + j * 32, kk, lane);
          else
            b[t][j] = *reinterpret_cast<const bf16x8_*>(&Bs[t * PB + rb + j * 32 * LDK + kk]);
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {  // small terms first
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
        }
    }
    __builtin_amdgcn_s_setprio(0);
    __syncthreads();
  }
  run_epilogue<TM, TN, 16>(ep, acc, M, N, (int)blockIdx.z, [&](int i, int j, int r, int& row, int& col) {
    row = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    col = n0 + wn * TN * 32 + j * 32 + (lane & 31);
  });
}

// ---- fill helpers: fetch (global -> registers) then commit (registers -> LDS) ----
// A loader with load4_fast(row, k) (no bounds checks) gets it for tiles wholly inside
// its rows and the K range (a wave-uniform test): the common case issues plain 16-B loads.
template <class L, class = void>
struct has_fast_load : std::false_type {};
template <class L>
struct has_fast_load<L, std::void_t<decltype(&L::load4_fast)>> : std::true_type {};

// Row-major source: L::load4(row, k, kend) -> 4 consecutive k of one row (zeros past kend).
template <int ROWS, int BK, class L>
__device__ __forceinline__ void fetch_rows(const L& l, f4* r, int row0, int k0, int kend, int tid) {
  constexpr int Q = BK / 4, T = ROWS * Q, NS = (T + 255) / 256;
  if constexpr (has_fast_load<L>::value) {
    if (k0 + BK <= kend && row0 + ROWS <= l.M) {
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        const int i = tid + j * 256;
        if (T % 256 == 0 || i < T) {
          int rr, q;
          rows_slot<ROWS, Q>(i, rr, q);
          r[j] = l.load4_fast(row0 + rr, k0 + 4 * q);
        }
      }
      return;
    }
  }
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int i = tid + j * 256;
    if (T % 256 == 0 || i < T) {
      int rr, q;
      rows_slot<ROWS, Q>(i, rr, q);
      r[j] = l.load4(row0 + rr, k0 + 4 * q, kend);
    }
  }
}
template <int ROWS, int BK, int LD>
__device__ __forceinline__ void commit_rows(const f4* r, float* s, int tid) {
  constexpr int Q = BK / 4, T = ROWS * Q, NS = (T + 255) / 256;
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int i = tid + j * 256;
    if (T % 256 == 0 || i < T) {
      int rr, q;
      rows_slot<ROWS, Q>(i, rr, q);
      *reinterpret_cast<f4*>(&s[rr * LD + 4 * q]) = r[j];
    }
  }
}

// Transposing source (wgrad): L::load4t(p, r) -> rows r..r+3 at reduction index p.
// Slot i holds rows 4*rq..4*rq+3 at k = kk with rq = (i & 1) + 2 * (i / (2*BK)),
// kk = (i >> 1) % BK: pairs of lanes read 32 contiguous bytes of one k, and the 32 lanes
// of a ds_write_b32 half cover kk 0..15 x two row quads, whose banks
// ((4 rq + c) * LD + kk) mod 32 are distinct when LD = BK + 4 (4 LD = 16 mod 32).
template <int ROWS, int BK, class L>
__device__ __forceinline__ void fetch_trans(const L& l, f4* r, int row0, int k0, int kend, int tid) {
  constexpr int R4 = ROWS / 4, T = R4 * BK, NS = (T + 255) / 256;
  static_assert(R4 % 2 == 0, "row quads in pairs");
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int i = tid + j * 256;
    if (T % 256 == 0 || i < T) {
      const int kk = (i >> 1) % BK, rq = (i & 1) + 2 * (i / (2 * BK));
      const int p = k0 + kk;
      r[j] = (p < kend) ? l.load4t(p, row0 + 4 * rq) : f4zero();
    }
  }
}
template <int ROWS, int BK, int LD>
__device__ __forceinline__ void commit_trans(const f4* r, float* s, int tid) {
  constexpr int R4 = ROWS / 4, T = R4 * BK, NS = (T + 255) / 256;
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int i = tid + j * 256;
    if (T % 256 == 0 || i < T) {
      const int kk = (i >> 1) % BK, rq = (i & 1) + 2 * (i / (2 * BK));
      s[(4 * rq + 0) * LD + kk] = r[j][0];
      s[(4 * rq + 1) * LD + kk] = r[j][1];
      s[(4 * rq + 2) * LD + kk] = r[j][2];
      s[(4 * rq + 3) * LD + kk] = r[j][3];
    }
  }
}

// Mix-ins giving a loader the fetch/commit/slots interface of the GEMM core.
#define VN_ROWS_LOADER                                                                     \
  static constexpr bool kTrans = false;                                                    \
  template <int ROWS, int BK>                                                              \
  static constexpr int slots() { return ROWS * (BK / 4); }                                 \
  template <int ROWS, int BK>                                                              \
  __device__ __forceinline__ void fetch(f4* r, int r0, int k0, int ke, int tid) const {    \
    fetch_rows<ROWS, BK>(*this, r, r0, k0, ke, tid);                                       \
  }                                                                                        \
  template <int ROWS, int BK, int LD>                                                      \
  __device__ __forceinline__ static void commit(const f4* r, float* s, int tid) {          \
    commit_rows<ROWS, BK, LD>(r, s, tid);                                                  \
  }

#define VN_TRANS_LOADER                                                                    \
  static constexpr bool kTrans = true;                                                     \
  template <int ROWS, int BK>                                                              \
  static constexpr int slots() { return (ROWS / 4) * BK; }                                 \
  template <int ROWS, int BK>                                                              \
  __device__ __forceinline__ void fetch(f4* r, int r0, int k0, int ke, int tid) const {    \
    fetch_trans<ROWS, BK>(*this, r, r0, k0, ke, tid);                                      \
  }                                                                                        \
  template <int ROWS, int BK, int LD>                                                      \
  __device__ __forceinline__ static void commit(const f4* r, float* s, int tid) {          \
    commit_trans<ROWS, BK, LD>(r, s, tid);                                                 \
  }

}  // namespace vn
