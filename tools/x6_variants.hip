// x6_variants.hip — diagnostic: the x6 GEMM core (vn_gemm.h gemm_x6_kernel) against a
// variant that stages the A operand in LDS as fp32 (16-B stores, 4 B per value) and splits
// it into the three bf16 terms after the fragment read, B staged as split planes as in the
// core. LDS store bytes per A value 6 -> 4, fragment read bytes 48 -> 32 per lane; the split
// VALU is unchanged when one wave reads each A row (WN == 1). Shapes: conv2 forward at
// 174x174 (im2col, N = 32) and the LSTM gates product. Outputs must match bit for bit.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/x6_variants.hip -o tools/x6_variants
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

__device__ __forceinline__ void split8(const f4& x0, const f4& x1, bf16x8_& t0, bf16x8_& t1, bf16x8_& t2) {
  union { uint16_t u[8]; bf16x8_ v; } a, b, c;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    split3_bf16(x0[e], a.u[e], b.u[e], c.u[e]);
    split3_bf16(x1[e], a.u[4 + e], b.u[4 + e], c.u[4 + e]);
  }
  t0 = a.v;
  t1 = b.v;
  t2 = c.v;
}

template <int BM, int BN, int BK, int WM, int WN, class FA, class FB, class EP>
__global__ __launch_bounds__(256) void gemm_x6a_kernel(FA fa, FB fb, EP ep, int M, int N, int K, int kchunk) {
  constexpr int LDA = BK + 4;  // fp32 row stride: the 16-lane groups of a ds_read_b128 on distinct quads
  constexpr int LDK = BK + 8;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  constexpr int NA = (FA::template slots<BM, BK>() + 255) / 256;
  constexpr int NB = (FB::template slots<BN, BK>() + 255) / 256;
  __shared__ __attribute__((aligned(16))) float As[BM * LDA];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[3 * BN * LDK];
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
  const int ra = (wm * TM * 32 + (lane & 31)) * LDA + 8 * (lane >> 5);
  const int rb = (wn * TN * 32 + (lane & 31)) * LDK + 8 * (lane >> 5);
  f4 pa[NA], pb[NB];
  if (kb < ke) {
    fa.template fetch<BM, BK>(pa, m0, kb, ke, tid);
    fb.template fetch<BN, BK>(pb, n0, kb, ke, tid);
  }
  for (int k0 = kb; k0 < ke; k0 += BK) {
    commit_rows<BM, BK, LDA>(pa, As, tid);
    commit_x6<BN, BK, LDK, FB>(pb, Bs, tid);
    __syncthreads();
    if (k0 + BK < ke) {
      fa.template fetch<BM, BK>(pa, m0, k0 + BK, ke, tid);
      fb.template fetch<BN, BK>(pb, n0, k0 + BK, ke, tid);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 16) {
      bf16x8_ a[3][TM], b[3][TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const f4 x0 = *reinterpret_cast<const f4*>(&As[ra + i * 32 * LDA + kk]);
        const f4 x1 = *reinterpret_cast<const f4*>(&As[ra + i * 32 * LDA + kk + 4]);
        split8(x0, x1, a[0][i], a[1][i], a[2][i]);
      }
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          b[t][j] = *reinterpret_cast<const bf16x8_*>(&Bs[t * BN * LDK + rb + j * 32 * LDK + kk]);
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
    __builtin_amdgcn_s_setprio(0);
    __syncthreads();
  }
  run_epilogue<TM, TN, 16>(ep, acc, M, N, (int)blockIdx.z, [&](int i, int j, int r, int& row, int& col) {
    row = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    col = n0 + wn * TN * 32 + j * 32 + (lane & 31);
  });
}

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
  f();
  hipDeviceSynchronize();
  hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r) f();
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

static double maxdiff(const float* a, const float* b, int64_t n) {
  std::vector<float> x(n), y(n);
  hipMemcpy(x.data(), a, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(y.data(), b, n * 4, hipMemcpyDeviceToHost);
  double m = 0;
  for (int64_t i = 0; i < n; ++i) m = std::max(m, (double)std::fabs(x[i] - y[i]));
  return m;
}

int main() {
  {  // conv2 forward, 174x174: 8192 frames, 42x42x32 -> 20x20x32
    const int frames = 8192;
    const int64_t X1n = (int64_t)frames * 42 * 42 * 32, X2n = (int64_t)frames * 400 * 32;
    float* X1 = dalloc(X1n, 1, -0.5f);
    float* W2 = dalloc(32 * 512, 5, -0.05f);
    float* b = dalloc(32, 8, 0.f);
    float* o1 = dalloc(X2n, 9, 0.f);
    float* o2 = dalloc(X2n, 9, 0.f);
    const double fl = 2.0 * frames * 400 * 32 * 512;
    NhwcIm2col<32, 4, 4, 2, 42, 42, 20, 20, 1> fa{X1, frames * 400};
    DenseRows fb{W2, 512, 32};
    const int M = fa.M;
    for (int rep = 0; rep < 2; ++rep) {
      float t0 = timeit([&] { launch_gemm_x6<128, 32, 32, 4, 1>(fa, fb, EpiBiasAct{o1, 32, b, 1}, M, 32, 512, 0); });
      float t1 = timeit([&] {
        hipLaunchKernelGGL((gemm_x6a_kernel<128, 32, 32, 4, 1, decltype(fa), DenseRows, EpiBiasAct>), grid_for(M, 32, 128, 32),
                           dim3(256), 0, 0, fa, fb, EpiBiasAct{o2, 32, b, 1}, M, 32, 512, 512);
      });
      printf("conv2 fwd 174: core %.3f ms (%.1f TF)  A-fp32 %.3f ms (%.1f TF)\n", t0, fl / t0 / 1e9, t1, fl / t1 / 1e9);
    }
    hipDeviceSynchronize();
    printf("conv2 fwd 174: max |core - variant| = %g\n", maxdiff(o1, o2, X2n));
    hipFree(X1), hipFree(o1), hipFree(o2);
  }
  {  // LSTM gates: [4096 x 1032] x [2048 x 1032]^T
    const int E = 4096, XC = 1032;
    float* X = dalloc((int64_t)E * XC, 11, -1.f);
    float* W = dalloc((int64_t)2048 * XC, 12, -0.05f);
    float* o1 = dalloc((int64_t)E * 2048, 9, 0.f);
    float* o2 = dalloc((int64_t)E * 2048, 9, 0.f);
    float* b = dalloc(2048, 8, 0.f);
    const double fl = 2.0 * E * 2048 * XC;
    DenseRows fa{X, XC, E}, fb{W, XC, 2048};
    for (int rep = 0; rep < 2; ++rep) {
      float t0 = timeit([&] { launch_gemm_x6<128, 128, 32, 2, 2>(fa, fb, EpiBiasAct{o1, 2048, b, 0}, E, 2048, XC, 0); });
      float t1 = timeit([&] {
        hipLaunchKernelGGL((gemm_x6a_kernel<128, 128, 32, 2, 2, DenseRows, DenseRows, EpiBiasAct>), grid_for(E, 2048, 128, 128),
                           dim3(256), 0, 0, fa, fb, EpiBiasAct{o2, 2048, b, 0}, E, 2048, XC, XC);
      });
      float t2 = timeit([&] {
        hipLaunchKernelGGL((gemm_x6a_kernel<128, 64, 32, 4, 1, DenseRows, DenseRows, EpiBiasAct>), grid_for(E, 2048, 128, 64),
                           dim3(256), 0, 0, fa, fb, EpiBiasAct{o2, 2048, b, 0}, E, 2048, XC, XC);
      });
      printf("lstm gates: core 128x128 %.3f ms (%.1f TF)  A-fp32 128x128 %.3f ms (%.1f TF)  A-fp32 128x64 4x1 %.3f ms (%.1f TF)\n",
             t0, fl / t0 / 1e9, t1, fl / t1 / 1e9, t2, fl / t2 / 1e9);
    }
    hipDeviceSynchronize();
    printf("lstm gates: max |core - variant| = %g\n", maxdiff(o1, o2, (int64_t)E * 2048));
  }
  printf("done\n");
  return 0;
}
