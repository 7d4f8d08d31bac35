// sweep_c2f174.hip — x6 tile shapes of conv2's forward product at 174x174 (42x42x32 ->
// 20x20x32, one rollout step of 4096 envs = 8192 frames). Diagnostic tool. Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/sweep_c2f174.hip -o tools/sweep_c2f174
#include "../a2cat-vn-pytorch_amd/csrc/vn_policy.hip"

#include <cstdio>

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
static float timeit(F f, int reps = 10) {
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

int main() {
  const int frames = 8192;
  const int64_t X1n = (int64_t)frames * 42 * 42 * 32, X2n = (int64_t)frames * 400 * 32;
  float* X1 = dalloc(X1n, 1, -0.5f);
  float* W2 = dalloc(32 * 512, 5, -0.05f);
  float* b = dalloc(32, 8, 0.f);
  float* out = dalloc(X2n, 9, 0.f);
  hipStream_t st = 0;
  const double fl = 2.0 * frames * 400 * 32 * 512;
#define X6(BM, BN, BK, WM, WN)                                                                                  \
  {                                                                                                             \
    NhwcIm2col<32, 4, 4, 2, 42, 42, 20, 20, 1> fa{X1, frames * 400};                                            \
    DenseRows fb{W2, 512, 32};                                                                                  \
    EpiBiasAct ep{out, 32, b, 1};                                                                               \
    float ms = timeit([&] { launch_gemm_x6<BM, BN, BK, WM, WN>(fa, fb, ep, fa.M, 32, 512, st); });             \
    printf("conv2 fwd x6 <%3d,%3d,%2d,%d,%d> %8.3f ms %7.1f TF\n", BM, BN, BK, WM, WN, ms, fl / ms / 1e9);      \
  }
  X6(128, 32, 32, 4, 1)
  X6(128, 32, 64, 4, 1)
  X6(256, 32, 32, 4, 1)
  X6(256, 32, 16, 4, 1)
  X6(128, 32, 16, 4, 1)
  hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
