// tile_sweep.hip — time the conv2/conv3 GEMM tile configurations at the training shapes
// (diagnostic tool, not part of the library). Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tile_sweep.hip -o tools/tile_sweep
// Includes the library TU so the same loaders/epilogues are timed.
#include "../a2cat-vn-pytorch_amd/csrc/vn_policy.hip"

#include <cstdio>
#include <vector>

using namespace vn;

namespace vn {  // the library's error helpers live in vn_env.hip
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
static float timeit(F f, int reps = 5) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    hipEventRecord(a, 0);
    f();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    best = std::min(best, ms);
  }
  return best;
}

int main(int argc, char** argv) {
  const bool dense_only = argc > 3 && atoi(argv[3]) == 1;
  const int n = argc > 1 ? atoi(argv[1]) : 81920;    // backward batch (T*E)
  const int nf = argc > 2 ? atoi(argv[2]) : 4096;    // forward batch (E)
  using G = Geo<84, 84>;
  const int64_t X1n = 2ll * n * 400 * 32, X2n = 2ll * n * 81 * 32, X3n = (int64_t)n * 9 * 64;
  float* X1 = dalloc(X1n, 1, -0.5f);
  float* X2 = dalloc(X2n, 2, -0.5f);
  float* dz2 = dalloc(X2n, 3, -0.5f);
  float* dz3 = dalloc(X3n, 4, -0.5f);
  float* W2 = dalloc(32 * 512, 5, -0.5f);
  float* W2T = dalloc(32 * 512, 6, -0.5f);
  float* W3 = dalloc(64 * 1024, 7, -0.5f);
  float* b = dalloc(64, 8, 0.f);
  float* out = dalloc(X1n, 9, 0.f);
  float* slab = dalloc(8ll << 20, 10, 0.f);
  float* dW = dalloc(64 * 1025, 11, 0.f);
  float* db = dalloc(64, 12, 0.f);
  hipStream_t st = 0;
  {  // LSTM gates GEMM: [4096 x 1032] x [2048 x 1032]^T
    const int E = nf, XC = 1032;
    float* xc = dalloc((int64_t)E * XC, 21, -0.5f);
    float* wc = dalloc(2048ll * XC, 22, -0.05f);
    float* gt = dalloc((int64_t)E * 2048, 23, 0.f);
    float* b0 = dalloc(2048, 24, 0.f);
    const double fl = 2.0 * E * 2048 * XC;
#define DENSE(BM, BN, BK, WM, WN)                                                                            \
    {                                                                                                        \
      DenseRows fa{xc, XC, E};                                                                               \
      DenseRows fb{wc, XC, 2048};                                                                            \
      EpiBias2 ep{gt, 2048, b0, b0};                                                                         \
      float ms = timeit([&] { launch_gemm<BM, BN, BK, WM, WN>(fa, fb, ep, E, 2048, XC, st); });              \
      printf("lstm gates  <%3d,%3d,%2d,%d,%d> %8.3f ms %7.1f TF\n", BM, BN, BK, WM, WN, ms, fl / ms / 1e9);    \
    }
#define DENSE32(BM, BN, BK, WM, WN)                                                                          \
    {                                                                                                        \
      DenseRows fa{xc, XC, E};                                                                               \
      DenseRows fb{wc, XC, 2048};                                                                            \
      EpiBias2 ep{gt, 2048, b0, b0};                                                                         \
      float ms = timeit([&] { launch_gemm32<BM, BN, BK, WM, WN>(fa, fb, ep, E, 2048, XC, st); });            \
      printf("lstm gates32<%3d,%3d,%2d,%d,%d> %8.3f ms %7.1f TF\n", BM, BN, BK, WM, WN, ms, fl / ms / 1e9);    \
    }
    {  // LSTM weight gradient: dgates^T [2048 x P] x xcat [P x 1032] (split-K over P)
      const int P = 4 * E;
      float* dg = dalloc((int64_t)P * 2048, 25, -0.5f);
      float* xa = dalloc((int64_t)P * XC, 26, -0.5f);
      float* slab = dalloc(12ll << 20, 27, 0.f);
      float* dW = dalloc(2048ll * XC, 28, 0.f);
      float* db = dalloc(2048, 29, 0.f);
      const double fw = 2.0 * P * 2048 * XC;
#define WGL(BM, BN, WM, WN)                                                                                   \
      {                                                                                                       \
        Im2colT<DenseRows> fbw{DenseRows{xa, XC, P}, XC};                                                     \
        float ms = timeit([&] { launch_wgrad<BM, BN, WM, WN>(dg, 2048, 2048, fbw, XC, P, slab, 12ll << 20, dW, db, st); }); \
        printf("lstm wgrad  <%3d,%3d,32,%d,%d> %8.3f ms %7.1f TF\n", BM, BN, WM, WN, ms, fw / ms / 1e9);        \
      }
      WGL(64, 64, 2, 2)
      WGL(128, 64, 2, 2)
      WGL(128, 128, 2, 2)
      WGL(64, 128, 2, 2)
    }
#define DENSEX6(BM, BN, BK, WM, WN)                                                                          \
    {                                                                                                        \
      DenseRows fa{xc, XC, E};                                                                               \
      DenseRows fb{wc, XC, 2048};                                                                            \
      EpiBias2 ep{gt2, 2048, b0, b0};                                                                        \
      float ms = timeit([&] { launch_gemm_x6<BM, BN, BK, WM, WN>(fa, fb, ep, E, 2048, XC, st); });           \
      hipMemcpy(h2.data(), gt2, h2.size() * 4, hipMemcpyDeviceToHost);                                       \
      double md = 0, mx = 0;                                                                                 \
      for (size_t q = 0; q < h2.size(); ++q) { md = std::max(md, (double)fabsf(h2[q] - h1[q])); mx = std::max(mx, (double)fabsf(h1[q])); } \
      double e6 = 0, e1 = 0;                                                                                 \
      for (int q = 0; q < 2048; ++q) {                                                                       \
        const int rr = (q * 7919) % E, cc = (q * 104729) % 2048;                                             \
        double ex = 2.0 * hb[cc];                                                                            \
        for (int kx = 0; kx < XC; ++kx) ex += (double)hx[(size_t)rr * XC + kx] * (double)hw[(size_t)cc * XC + kx]; \
        e6 = std::max(e6, fabs(h2[(size_t)rr * 2048 + cc] - ex));                                            \
        e1 = std::max(e1, fabs(h1[(size_t)rr * 2048 + cc] - ex));                                            \
      }                                                                                                      \
      printf("lstm gatesX6<%3d,%3d,%2d,%d,%d> %8.3f ms %7.1f TF  max|x6-f32|/max %.2e  fp64 err x6 %.2e f32 %.2e\n", BM, BN, BK, WM, WN, ms, fl / ms / 1e9, md / mx, e6 / mx, e1 / mx); \
    }
    std::vector<float> h1((size_t)E * 2048), h2((size_t)E * 2048), hx((size_t)E * XC), hw(2048ll * XC);
    hipMemcpy(hx.data(), xc, hx.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hw.data(), wc, hw.size() * 4, hipMemcpyDeviceToHost);
    std::vector<float> hb(2048);
    hipMemcpy(hb.data(), b0, hb.size() * 4, hipMemcpyDeviceToHost);
    float* gt2 = dalloc((int64_t)E * 2048, 30, 0.f);
    {
      DenseRows fa{xc, XC, E};
      DenseRows fb{wc, XC, 2048};
      EpiBias2 ep{gt, 2048, b0, b0};
      launch_gemm<64, 64, 32, 2, 2>(fa, fb, ep, E, 2048, XC, st);
      hipMemcpy(h1.data(), gt, h1.size() * 4, hipMemcpyDeviceToHost);
    }
    DENSEX6(64, 64, 32, 2, 2)
    DENSEX6(128, 128, 32, 2, 2)
    DENSEX6(128, 128, 16, 2, 2)
    DENSEX6(128, 64, 32, 2, 2)
    DENSEX6(64, 128, 32, 2, 2)
    DENSEX6(256, 128, 16, 2, 2)
    DENSE32(64, 64, 32, 2, 2)
    DENSE32(128, 128, 32, 2, 2)
    DENSE32(128, 128, 16, 2, 2)
    DENSE32(128, 64, 32, 2, 2)
    DENSE32(64, 128, 32, 2, 2)
    DENSE32(128, 128, 64, 2, 2)
    DENSE32(256, 128, 16, 2, 2)
    DENSE(64, 64, 32, 2, 2)
    DENSE(128, 64, 32, 2, 2)
    DENSE(64, 128, 32, 2, 2)
    DENSE(128, 128, 32, 2, 2)
    DENSE(128, 128, 16, 2, 2)
    DENSE(64, 64, 64, 2, 2)
    DENSE(128, 64, 64, 2, 2)
  }

  const double f2 = 2.0 * 81 * 32 * 512;  // per frame flops of conv2
  if (dense_only) { hipDeviceSynchronize(); printf("done\n"); return 0; }

#define FWD2(BM, BN, BK, WM, WN)                                                                                  \
  {                                                                                                               \
    NhwcIm2col<32, 4, 4, 2, 20, 20, 9, 9, 1> fa{X1, 2 * nf * 81};                                                 \
    DenseRows fb{W2, 512, 32};                                                                                    \
    EpiBiasAct ep{out, 32, b, 1};                                                                                 \
    float ms = timeit([&] { launch_gemm<BM, BN, BK, WM, WN>(fa, fb, ep, fa.M, 32, 512, st); });                     \
    printf("conv2 fwd   <%3d,%3d,%2d,%d,%d> %8.3f ms %7.1f TF\n", BM, BN, BK, WM, WN, ms, f2 * 2 * nf / ms / 1e9); \
  }
  FWD2(64, 32, 32, 4, 1)
  FWD2(64, 32, 64, 4, 1)
  FWD2(128, 32, 32, 4, 1)
  FWD2(128, 32, 64, 4, 1)
  FWD2(128, 32, 32, 2, 2)
  FWD2(256, 32, 32, 4, 1)

  {
    float ms = timeit([&] { dgrad_all_classes<32, 32, 20, 20, 9, 9>(dz2, W2T, out, X1, 2 * n, 0, 1, 32, st); });
    printf("conv2 dgrad <64,32,32,4,1> %8.3f ms %7.1f TF\n", ms, f2 * 2 * n / ms / 1e9);
  }
  {
    const int frames = 2 * n;
    const int blocks = std::min(frames, resident_blocks((const void*)conv2_dgrad_kernel<20, 20, 9, 9, false>, 256, 0));
    float ms = timeit([&] {
      hipLaunchKernelGGL((conv2_dgrad_kernel<20, 20, 9, 9, false>), dim3(blocks), dim3(256), 0, st, dz2, W2T, X1, nullptr, out, frames);
    });
    printf("conv2 dgrad specialised   %8.3f ms %7.1f TF (%d blocks)\n", ms, f2 * 2 * n / ms / 1e9, blocks);
  }
  {
    const int frames = 2 * n, blocks = std::min(frames, kConv2WgradBlocks);
    constexpr size_t lds = conv2_wgrad_lds<20, 20, 9, 9>();
    hipFuncSetAttribute((const void*)conv2_wgrad_kernel<20, 20, 9, 9>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    float ms = timeit([&] {
      hipLaunchKernelGGL((conv2_wgrad_kernel<20, 20, 9, 9>), dim3(blocks), dim3(256), lds, st, X1, dz2, frames, slab,
                         slab + (int64_t)blocks * 32 * 512, FrameList{});
    });
    printf("conv2 wgrad specialised   %8.3f ms %7.1f TF\n", ms, f2 * 2 * n / ms / 1e9);
  }

#define WG2(BM, BN, WM, WN)                                                                                       \
  {                                                                                                               \
    using Im = NhwcIm2col<32, 4, 4, 2, 20, 20, 9, 9, 1>;                                                          \
    const int P2 = 2 * n * 81;                                                                                    \
    Im2colT<Im> fbw{Im{X1, P2}, 512};                                                                             \
    float ms = timeit([&] { launch_wgrad<BM, BN, WM, WN>(dz2, 32, 32, fbw, 512, P2, slab, 8ll << 20, dW, db, st); }); \
    printf("conv2 wgrad <%3d,%3d,32,%d,%d> %8.3f ms %7.1f TF\n", BM, BN, WM, WN, ms, f2 * 2 * n / ms / 1e9);      \
  }
  WG2(32, 64, 2, 2)
  WG2(32, 128, 2, 2)
  WG2(32, 128, 1, 4)
  WG2(32, 256, 1, 4)
  WG2(32, 64, 1, 4)

  const double f3 = 2.0 * 9 * 64 * 1024;
  {
    float ms = timeit([&] {
      for (int g = 0; g < 2; ++g) dgrad_all_classes<64, 64, 9, 9, 3, 3>(dz3, W3, out, X2, n, g, 2, 32, st);
    });
    printf("conv3 dgrad <64,32,32,4,1> %8.3f ms %7.1f TF\n", ms, f3 * n / ms / 1e9);
  }
  hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
