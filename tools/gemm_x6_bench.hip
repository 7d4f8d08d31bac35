// gemm_x6_bench.hip — where the time of the split-bf16 ("x6") GEMM core goes, at the LSTM
// gates shape (M 4096, N 2048, K 1032; DenseRows x DenseRows). Diagnostic tool, not part of
// the library. Variants of the core loop (flags of xk below):
//   LOADS 0: no global loads (LDS filled once: MFMA + LDS-read bound)
//   SPLIT 0: commit writes only the hi plane (the VALU split and two thirds of the LDS
//            writes removed; numerically wrong, timing only)
//   PF 2   : two register stages of global prefetch
//   PRIO 1 : s_setprio 1 around the MFMA cluster
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_x6_bench.hip -o tools/gemm_x6_bench
#include "../a2cat-vn-pytorch_amd/csrc/vn_policy.hip"

#include <cstdio>
#include <vector>

using namespace vn;

namespace vn {
int fail(int code, const std::string& msg) {
  fprintf(stderr, "%s\n", msg.c_str());
  return code;
}
int hip_fail(hipError_t e, const char* what) {
  fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
  return VN_EHIP;
}
}  // namespace vn

__global__ void fill_kernel(float* p, int64_t n, uint32_t seed, float lo) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint32_t h = frame_hash(seed, (uint32_t)(i >> 32), (uint32_t)i);
    p[i] = lo + (float)(h >> 8) * (1.0f / 16777216.0f);
  }
}

static float* dalloc(int64_t n, uint32_t seed, float lo) {
  float* p = nullptr;
  if (hipMalloc(&p, n * 4) != hipSuccess) {
    printf("alloc failed\n");
    exit(1);
  }
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, p, n, seed, lo);
  return p;
}

template <class F>
static float timeit(F f, int reps = 20) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) f();
  hipDeviceSynchronize();
  hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r) f();
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

// epilogue that stores only if a value is NaN (never): the kernel without its output stores
struct EpiNone {
  float* out;
  __device__ __forceinline__ void operator()(int row, int col, float v, int) const {
    if (v != v) out[0] = v;
  }
};

template <int ROWS, int BK, int LDK>
__device__ __forceinline__ void commit_hi_only(const f4* r, uint16_t* s, int tid) {
  constexpr int Q = BK / 4, T = ROWS * Q, NS = (T + 255) / 256;
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int i = tid + j * 256;
    if (T % 256 == 0 || i < T) {
      const int rr = i / Q, q = i - (i / Q) * Q;
      uint32_t t0[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) t0[e] = __float_as_uint(r[j][e]) >> 16;
      uint16_t* d = s + rr * LDK + 4 * q;
      *reinterpret_cast<uint2*>(d) = uint2{t0[0] | (t0[1] << 16), t0[2] | (t0[3] << 16)};
    }
  }
}

template <int BM, int BN, int BK, int WM, int WN, int LOADS, int SPLIT, int PF, int PRIO, class FA, class FB, class EP>
__global__ __launch_bounds__(256) void xk(FA fa, FB fb, EP ep, int M, int N, int K) {
  constexpr int LDK = BK + 8;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  constexpr int NA = (FA::template slots<BM, BK>() + 255) / 256;
  constexpr int NB = (FB::template slots<BN, BK>() + 255) / 256;
  __shared__ __attribute__((aligned(16))) uint16_t As[3 * BM * LDK];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[3 * BN * LDK];
  typedef float f16v_ __attribute__((ext_vector_type(16)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kb = 0, ke = K;
  f16v_ acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  const int ra = (wm * TM * 32 + (lane & 31)) * LDK + 8 * (lane >> 5);
  const int rb = (wn * TN * 32 + (lane & 31)) * LDK + 8 * (lane >> 5);
  f4 pa[PF][NA], pb[PF][NB];
  fa.template fetch<BM, BK>(pa[0], m0, kb, ke, tid);
  fb.template fetch<BN, BK>(pb[0], n0, kb, ke, tid);
  if constexpr (PF == 2) {
    fa.template fetch<BM, BK>(pa[1], m0, kb + BK, ke, tid);
    fb.template fetch<BN, BK>(pb[1], n0, kb + BK, ke, tid);
  }
  if constexpr (LOADS == 0) {
    commit_x6<BM, BK, LDK, FA>(pa[0], As, tid);
    commit_x6<BN, BK, LDK, FB>(pb[0], Bs, tid);
    __syncthreads();
  }
  auto tile = [&](auto stage, int k0) {
    constexpr int S = decltype(stage)::value;
    if constexpr (LOADS) {
      if constexpr (SPLIT) {
        commit_x6<BM, BK, LDK, FA>(pa[S], As, tid);
        commit_x6<BN, BK, LDK, FB>(pb[S], Bs, tid);
      } else {
        commit_hi_only<BM, BK, LDK>(pa[S], As, tid);
        commit_hi_only<BN, BK, LDK>(pb[S], Bs, tid);
      }
      __syncthreads();
      if (k0 + PF * BK < ke) {
        fa.template fetch<BM, BK>(pa[S], m0, k0 + PF * BK, ke, tid);
        fb.template fetch<BN, BK>(pb[S], n0, k0 + PF * BK, ke, tid);
      }
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 16) {
      bf16x8_ a[3][TM], b[3][TN];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
          a[t][i] = *reinterpret_cast<const bf16x8_*>(&As[t * BM * LDK + ra + i * 32 * LDK + kk]);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          b[t][j] = *reinterpret_cast<const bf16x8_*>(&Bs[t * BN * LDK + rb + j * 32 * LDK + kk]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
        }
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    if constexpr (LOADS) __syncthreads();
  };
  if constexpr (PF == 2) {
    for (int k0 = kb; k0 < ke; k0 += 2 * BK) {
      tile(std::integral_constant<int, 0>{}, k0);
      if (k0 + BK < ke) tile(std::integral_constant<int, 1>{}, k0 + BK);
    }
  } else {
    for (int k0 = kb; k0 < ke; k0 += BK) tile(std::integral_constant<int, 0>{}, k0);
  }
  run_epilogue<TM, TN, 16>(ep, acc, M, N, 0, [&](int i, int j, int r, int& row, int& col) {
    row = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    col = n0 + wn * TN * 32 + j * 32 + (lane & 31);
  });
}

// Double-buffered LDS: tile k's MFMAs run while tile k+1 (already in registers) is split
// into the other buffer and tile k+2's global loads are issued; one barrier per tile.
// SG: sched_group_barrier interleave pattern (0 = compiler's choice).
template <int BM, int BN, int BK, int WM, int WN, int SG, class FA, class FB, class EP>
__global__ __launch_bounds__(256) void xdb(FA fa, FB fb, EP ep, int M, int N, int K) {
  constexpr int LDK = BK + 8;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  constexpr int NA = (FA::template slots<BM, BK>() + 255) / 256;
  constexpr int NB = (FB::template slots<BN, BK>() + 255) / 256;
  constexpr int ASZ = 3 * BM * LDK, BSZ = 3 * BN * LDK;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem16[];
  typedef float f16v_ __attribute__((ext_vector_type(16)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int ke = K;
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
  fa.template fetch<BM, BK>(pa, m0, 0, ke, tid);
  fb.template fetch<BN, BK>(pb, n0, 0, ke, tid);
  commit_x6<BM, BK, LDK, FA>(pa, smem16, tid);
  commit_x6<BN, BK, LDK, FB>(pb, smem16 + ASZ, tid);
  if (BK < ke) {
    fa.template fetch<BM, BK>(pa, m0, BK, ke, tid);
    fb.template fetch<BN, BK>(pb, n0, BK, ke, tid);
  }
  __syncthreads();
  int cur = 0;
  for (int k0 = 0; k0 < ke; k0 += BK) {
    const uint16_t* As = smem16 + cur * (ASZ + BSZ);
    const uint16_t* Bs = As + ASZ;
    uint16_t* An = smem16 + (cur ^ 1) * (ASZ + BSZ);
    const bool more = k0 + BK < ke;
    bf16x8_ a[BK / 16][3][TM], b[BK / 16][3][TN];
#pragma unroll
    for (int kq = 0; kq < BK / 16; ++kq)
#pragma unroll
      for (int t = 0; t < 3; ++t) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
          a[kq][t][i] = *reinterpret_cast<const bf16x8_*>(&As[t * BM * LDK + ra + i * 32 * LDK + kq * 16]);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          b[kq][t][j] = *reinterpret_cast<const bf16x8_*>(&Bs[t * BN * LDK + rb + j * 32 * LDK + kq * 16]);
      }
    if (more) {
      commit_x6<BM, BK, LDK, FA>(pa, An, tid);
      commit_x6<BN, BK, LDK, FB>(pb, An + ASZ, tid);
    }
#pragma unroll
    for (int kq = 0; kq < BK / 16; ++kq)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[kq][2][i], b[kq][0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[kq][0][i], b[kq][2][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[kq][1][i], b[kq][1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[kq][1][i], b[kq][0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[kq][0][i], b[kq][1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[kq][0][i], b[kq][0][j], acc[i][j], 0, 0, 0);
        }
    if constexpr (SG == 1) {
      // per MFMA: 5 VALU, 1 DS write (the commit), then global loads at the end
#pragma unroll
      for (int q = 0; q < (BK / 16) * TM * TN * 6; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      }
    }
    if (k0 + 2 * BK < ke) {
      fa.template fetch<BM, BK>(pa, m0, k0 + 2 * BK, ke, tid);
      fb.template fetch<BN, BK>(pb, n0, k0 + 2 * BK, ke, tid);
    }
    __syncthreads();
    cur ^= 1;
  }
  run_epilogue<TM, TN, 16>(ep, acc, M, N, 0, [&](int i, int j, int r, int& row, int& col) {
    row = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    col = n0 + wn * TN * 32 + j * 32 + (lane & 31);
  });
}

// Loader/MFMA-wave core (gemm_x6pc_kernel) with diagnostic switches: LOAD 0 = the loader waves
// stage tile 0 once and then only meet the barriers (MFMA + LDS-read + barrier bound);
// HOIST 1 = the MFMA waves read both 16-k fragment sets of a K tile before its MFMAs.
template <int BM, int BN, int BK, int LOAD, int HOIST, class FA, class FB, class EP>
__global__ __launch_bounds__(512, 1) void xpc(FA fa, FB fb, EP ep, int M, int N, int K) {
  constexpr int LDK = BK + 8;
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int NA = (FA::template slots<BM, BK>() + 255) / 256;
  constexpr int NB = (FB::template slots<BN, BK>() + 255) / 256;
  constexpr int PA = BM * LDK, PB = BN * LDK;
  __shared__ __attribute__((aligned(16))) uint16_t As[2][3 * PA];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][3 * PB];
  typedef float f16v_ __attribute__((ext_vector_type(16)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool loader = wave >= 4;
  const int ltid = tid - 256;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kb = 0, ke = K;
  const int nk = (ke - kb + BK - 1) / BK;
  f4 pa[2][NA], pb[2][NB];
  auto fetch = [&](auto R, int j) {
    fa.template fetch<BM, BK>(pa[decltype(R)::value], m0, kb + j * BK, ke, ltid);
    fb.template fetch<BN, BK>(pb[decltype(R)::value], n0, kb + j * BK, ke, ltid);
  };
  auto commit = [&](auto R, int stage) {
    commit_x6<BM, BK, LDK, FA>(pa[decltype(R)::value], As[stage], ltid);
    commit_x6<BN, BK, LDK, FB>(pb[decltype(R)::value], Bs[stage], ltid);
  };
  using R0 = std::integral_constant<int, 0>;
  using R1 = std::integral_constant<int, 1>;
  if (loader) {
    fetch(R0{}, 0);
    if (nk > 1) fetch(R1{}, 1);
    commit(R0{}, 0);
    if (!LOAD) commit(R1{}, 1);
  }
  __syncthreads();
  const int wm = wave & 1, wn = (wave >> 1) & 1;
  f16v_ acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  const int ra = (wm * TM * 32 + (lane & 31)) * LDK + 8 * (lane >> 5);
  const int rb = (wn * TN * 32 + (lane & 31)) * LDK + 8 * (lane >> 5);
  auto iteration = [&](auto R, int it) {
    constexpr int P = decltype(R)::value;
    if (loader) {
      if constexpr (LOAD) {
        if (it + 2 < nk) fetch(R, it + 2);
        if (it + 1 < nk) commit(std::integral_constant<int, P ^ 1>{}, P ^ 1);
      }
    } else {
      const uint16_t* as = As[P];
      const uint16_t* bs = Bs[P];
      bf16x8_ a[BK / 16][3][TM], b[BK / 16][3][TN];
      auto rd = [&](int q) {
#pragma unroll
        for (int t = 0; t < 3; ++t) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
            a[q][t][i] = *reinterpret_cast<const bf16x8_*>(&as[t * PA + ra + i * 32 * LDK + q * 16]);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            b[q][t][j] = *reinterpret_cast<const bf16x8_*>(&bs[t * PB + rb + j * 32 * LDK + q * 16]);
        }
      };
      if constexpr (HOIST) {
#pragma unroll
        for (int q = 0; q < BK / 16; ++q) rd(q);
      }
#pragma unroll
      for (int q = 0; q < BK / 16; ++q) {
        if constexpr (!HOIST) rd(q);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[q][2][i], b[q][0][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[q][0][i], b[q][2][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[q][1][i], b[q][1][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[q][1][i], b[q][0][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[q][0][i], b[q][1][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[q][0][i], b[q][0][j], acc[i][j], 0, 0, 0);
          }
      }
    }
    __syncthreads();
  };
  for (int it = 0; it < nk; it += 2) {
    iteration(R0{}, it);
    if (it + 1 < nk) iteration(R1{}, it + 1);
  }
  if (!loader)
    run_epilogue<TM, TN, 16>(ep, acc, M, N, 0, [&](int i, int j, int r, int& row, int& col) {
      row = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      col = n0 + wn * TN * 32 + j * 32 + (lane & 31);
    });
}

template <int BM, int BN, int WM, int WN>
static void dh_shape(int M, int N, int K, const char* name) {
  float* a = dalloc((int64_t)M * K, 31, -0.5f);
  float* b = dalloc((int64_t)N * K, 32, -0.05f);
  float* c = dalloc((int64_t)M * N, 33, 0.f);
  float* bias = dalloc(N, 34, 0.f);
  DenseRows fa{a, K, M};
  DenseRows fb{b, K, N};
  EpiBias2 ep{c, N, bias, bias};
  const double fl = 2.0 * M * N * K;
  float ms = timeit([&] { launch_gemm_x6<BM, BN, 32, WM, WN>(fa, fb, ep, M, N, K, 0); });
  printf("%-12s M %6d N %5d K %5d <%3d,%3d,%d,%d>  %8.1f us %7.1f TF(f32-equiv) %5.1f%% x6 peak\n", name, M, N, K, BM, BN,
         WM, WN, ms * 1e3, fl / ms / 1e9, 100.0 * fl * 6 / (ms * 1e-3) / 2.5e15);
  hipFree(a);
  hipFree(b);
  hipFree(c);
  hipFree(bias);
}

// Mode 4: per-step products of the BPTT / rollout at 4096 envs against BK and split-K (the
// split form includes its slab write and splitk_epilogue_kernel launch).
template <int BM, int BN, int BK>
static void sk_shape(int M, int N, int K, int splits, const char* name) {
  float* a = dalloc((int64_t)M * K, 41, -0.5f);
  float* b = dalloc((int64_t)N * K, 42, -0.05f);
  float* c = dalloc((int64_t)M * N, 43, 0.f);
  float* bias = dalloc(N, 44, 0.f);
  float* slab = dalloc((int64_t)M * N * splits, 45, 0.f);
  DenseRows fa{a, K, M};
  DenseRows fb{b, K, N};
  EpiBias2 ep{c, N, bias, bias};
  const double fl = 2.0 * M * N * K;
  float ms;
  if (splits == 1) {
    ms = timeit([&] { launch_gemm_x6<BM, BN, BK, 2, 2>(fa, fb, ep, M, N, K, 0); });
  } else {
    const int kchunk = ((K + splits - 1) / splits + BK - 1) / BK * BK;
    const int sp = (K + kchunk - 1) / kchunk;
    EpiSlab es{slab, M, N};
    ms = timeit([&] {
      hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, BK, 2, 2, DenseRows, DenseRows, EpiSlab>), grid_for(M, N, BM, BN, sp),
                         dim3(256), 0, 0, fa, fb, es, M, N, K, kchunk);
      launch_splitk_epilogue(slab, sp, M, N, ep, 0);
    });
  }
  printf("%-10s M %6d N %5d K %5d <%3d,%3d,%2d> split %d  %8.1f us %7.1f TF(f32-equiv)\n", name, M, N, K, BM, BN, BK,
         splits, ms * 1e3, fl / ms / 1e9);
  hipFree(a);
  hipFree(b);
  hipFree(c);
  hipFree(bias);
  hipFree(slab);
}

int main(int argc, char** argv) {
  if (argc > 1 && atoi(argv[1]) == 4) {
    for (int rep = 0; rep < 2; ++rep) {
      sk_shape<64, 64, 32>(4096, 512, 2048, 1, "lstm dh");
      sk_shape<64, 64, 64>(4096, 512, 2048, 1, "lstm dh");
      sk_shape<64, 64, 32>(4096, 512, 2048, 2, "lstm dh");
      sk_shape<64, 64, 32>(4096, 512, 2048, 4, "lstm dh");
      sk_shape<64, 64, 64>(4096, 512, 2048, 2, "lstm dh");
      sk_shape<128, 128, 32>(4096, 2048, 1032, 1, "gates");
      sk_shape<128, 128, 64>(4096, 2048, 1032, 1, "gates");
      sk_shape<128, 128, 32>(4096, 2048, 1032, 2, "gates");
      sk_shape<64, 64, 32>(4096, 512, 2592, 1, "merge174");
      sk_shape<64, 64, 64>(4096, 512, 2592, 1, "merge174");
      sk_shape<64, 64, 32>(4096, 512, 2592, 2, "merge174");
      sk_shape<64, 64, 32>(4096, 512, 2592, 4, "merge174");
    }
    return 0;
  }
  if (argc > 1 && atoi(argv[1]) == 2) {
    for (int rep = 0; rep < 2; ++rep) {
      dh_shape<64, 64, 2, 2>(4096, 512, 2048, "lstm dh");
      dh_shape<128, 64, 2, 2>(4096, 512, 2048, "lstm dh");
      dh_shape<64, 128, 2, 2>(4096, 512, 2048, "lstm dh");
      dh_shape<128, 128, 2, 2>(4096, 512, 2048, "lstm dh");
      dh_shape<64, 64, 2, 2>(4096, 512, 288, "fc 84");
      dh_shape<128, 64, 2, 2>(4096, 512, 288, "fc 84");
      dh_shape<128, 128, 2, 2>(4096, 512, 288, "fc 84");
      dh_shape<128, 128, 2, 2>(81920, 512, 2048, "dz5 batched");
      dh_shape<128, 64, 2, 2>(81920, 512, 2048, "dz5 batched");
      dh_shape<128, 128, 2, 2>(4096, 2048, 1032, "gates");
      dh_shape<128, 64, 2, 2>(4096, 2048, 1032, "gates");
      dh_shape<64, 128, 2, 2>(4096, 2048, 1032, "gates");
    }
    return 0;
  }
  const int E = 4096, XC = 1032, N = 2048;
  float* xc = dalloc((int64_t)E * XC, 21, -0.5f);
  float* wc = dalloc((int64_t)N * XC, 22, -0.05f);
  float* gt = dalloc((int64_t)E * N, 23, 0.f);
  float* b0 = dalloc(N, 24, 0.f);
  hipStream_t st = 0;
  const double fl = 2.0 * E * N * XC;
  DenseRows fa{xc, XC, E};
  DenseRows fb{wc, XC, N};
  EpiBias2 ep{gt, N, b0, b0};
  auto rep = [&](const char* name, float ms) {
    printf("%-44s %8.1f us %7.1f TF(f32-equiv) %6.1f%% of x6 peak\n", name, ms * 1e3, fl / ms / 1e9,
           100.0 * fl * 6 / (ms * 1e-3) / 2.5e15);
  };
  rep("library gemm_x6 <128,128,32,2,2>", timeit([&] { launch_gemm_x6<128, 128, 32, 2, 2>(fa, fb, ep, E, N, XC, st); }));
  rep("library gemm_x6 <64,64,32,2,2>", timeit([&] { launch_gemm_x6<64, 64, 32, 2, 2>(fa, fb, ep, E, N, XC, st); }));

#define XK(BM, BN, BK, WM, WN, L, S, P, R)                                                                   \
  rep("xk<" #BM "," #BN "," #BK "> loads" #L " split" #S " pf" #P " prio" #R, timeit([&] {                  \
        hipLaunchKernelGGL((xk<BM, BN, BK, WM, WN, L, S, P, R, DenseRows, DenseRows, EpiBias2>),             \
                           grid_for(E, N, BM, BN), dim3(256), 0, st, fa, fb, ep, E, N, XC);                  \
      }));
  if (argc > 1 && atoi(argv[1]) == 3) {
    setenv("VN_GEMM_CLASSIC", "1", 1);
    rep("classic gemm_x6 <128,128,32,2,2>", timeit([&] { launch_gemm_x6<128, 128, 32, 2, 2>(fa, fb, ep, E, N, XC, st); }));
    unsetenv("VN_GEMM_CLASSIC");
    EpiNone en{gt};
#define XPC(BM, BN, L, H)                                                                                  \
    rep("xpc<" #BM "," #BN "> load" #L " hoist" #H, timeit([&] {                                           \
          hipLaunchKernelGGL((xpc<BM, BN, 32, L, H, DenseRows, DenseRows, EpiBias2>), grid_for(E, N, BM, BN), \
                             dim3(512), 0, st, fa, fb, ep, E, N, XC);                                      \
        }));
    XPC(128, 128, 1, 0)
    XPC(128, 128, 1, 1)
    XPC(128, 128, 0, 0)
    XPC(128, 128, 0, 1)
    rep("xpc<128,128> load0 hoist1 epilogue-none", timeit([&] {
          hipLaunchKernelGGL((xpc<128, 128, 32, 0, 1, DenseRows, DenseRows, EpiNone>), grid_for(E, N, 128, 128),
                             dim3(512), 0, st, fa, fb, en, E, N, XC);
        }));
    XK(128, 128, 32, 2, 2, 0, 1, 1, 0)
    XK(128, 128, 32, 2, 2, 1, 1, 1, 0)
    printf("done\n");
    return 0;
  }
  XK(128, 128, 32, 2, 2, 1, 1, 1, 0)
  XK(128, 128, 32, 2, 2, 0, 1, 1, 0)
  {
    EpiNone en{gt};
    rep("xk<128,128,32> loads0 epilogue-none", timeit([&] {
          hipLaunchKernelGGL((xk<128, 128, 32, 2, 2, 0, 1, 1, 0, DenseRows, DenseRows, EpiNone>), grid_for(E, N, 128, 128),
                             dim3(256), 0, st, fa, fb, en, E, N, XC);
        }));
    rep("xk<128,128,32> loads1 epilogue-none", timeit([&] {
          hipLaunchKernelGGL((xk<128, 128, 32, 2, 2, 1, 1, 1, 0, DenseRows, DenseRows, EpiNone>), grid_for(E, N, 128, 128),
                             dim3(256), 0, st, fa, fb, en, E, N, XC);
        }));
    rep("xk<128,128,32> loads1 prio1 epilogue-none", timeit([&] {
          hipLaunchKernelGGL((xk<128, 128, 32, 2, 2, 1, 1, 1, 1, DenseRows, DenseRows, EpiNone>), grid_for(E, N, 128, 128),
                             dim3(256), 0, st, fa, fb, en, E, N, XC);
        }));
  }
  XK(128, 128, 32, 2, 2, 1, 0, 1, 0)
  XK(128, 128, 32, 2, 2, 1, 1, 2, 0)
  XK(128, 128, 32, 2, 2, 1, 1, 1, 1)
  XK(128, 128, 64, 2, 2, 1, 1, 1, 0)
  XK(128, 128, 64, 2, 2, 0, 1, 1, 0)
  XK(64, 64, 32, 2, 2, 0, 1, 1, 0)
#define XDB(BM, BN, BK, WM, WN, SG)                                                                       \
  {                                                                                                        \
    auto kf = xdb<BM, BN, BK, WM, WN, SG, DenseRows, DenseRows, EpiBias2>;                                 \
    const int lds = 2 * 3 * (BM + BN) * (BK + 8) * 2;                                                      \
    hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, lds);                \
    rep("xdb<" #BM "," #BN "," #BK "> sg" #SG, timeit([&] {                                                 \
          hipLaunchKernelGGL(kf, grid_for(E, N, BM, BN), dim3(256), lds, st, fa, fb, ep, E, N, XC);         \
        }));                                                                                               \
    hipError_t e = hipGetLastError();                                                                      \
    if (e != hipSuccess) printf("  launch error %s\n", hipGetErrorString(e));                              \
  }
  XDB(128, 128, 32, 2, 2, 0)
  XDB(128, 128, 32, 2, 2, 1)
  XDB(128, 128, 16, 2, 2, 0)
  XDB(128, 128, 16, 2, 2, 1)
  XDB(64, 128, 32, 2, 2, 0)
  XDB(64, 64, 32, 2, 2, 0)
  // correctness of xdb vs the library kernel (same products, same order per accumulator)
  {
    std::vector<float> h1((size_t)E * N), h2((size_t)E * N);
    launch_gemm_x6<128, 128, 32, 2, 2>(fa, fb, ep, E, N, XC, st);
    hipMemcpy(h1.data(), gt, h1.size() * 4, hipMemcpyDeviceToHost);
    auto kf = xdb<128, 128, 32, 2, 2, 0, DenseRows, DenseRows, EpiBias2>;
    hipLaunchKernelGGL(kf, grid_for(E, N, 128, 128), dim3(256), 2 * 3 * 256 * 40 * 2, st, fa, fb, ep, E, N, XC);
    hipMemcpy(h2.data(), gt, h2.size() * 4, hipMemcpyDeviceToHost);
    size_t bad = 0;
    for (size_t q = 0; q < h1.size(); ++q) bad += (h1[q] != h2[q]);
    printf("xdb vs library: %zu of %zu differ\n", bad, h1.size());
  }
  printf("done\n");
  return 0;
}
