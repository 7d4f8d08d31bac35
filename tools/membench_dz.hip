// Read-pattern microbenchmark for conv1_wgrad_x3's dZ stream: 163840 frames x 400 pixels x 32
// fp32 (8.4 GB). A: the MFMA-layout dword loads (lane (co, h) reads 8 pixels of one channel,
// 2 x 128 B per instruction); B: 16-B loads (1 KB per instruction). 512 workgroups x 256.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(256) void rdA(const float* __restrict__ dz, int frames, float* out, int depth) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  float acc = 0.f;
  for (int f = blockIdx.x; f < frames; f += gridDim.x) {
    const float* zf = dz + (size_t)f * 400 * 32 + c32;
    for (int s = wave; s < 25; s += 4) {
      const float* p = zf + (16 * s + 8 * h) * 32;
      float z[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) z[j] = p[j * 32];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += z[j];
    }
  }
  if (acc == 1.2345f) out[0] = acc;
}

__global__ __launch_bounds__(256) void rdB(const float* __restrict__ dz, int frames, float* out, int depth) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc = 0.f;
  for (int f = blockIdx.x; f < frames; f += gridDim.x) {
    const f4* zf = reinterpret_cast<const f4*>(dz + (size_t)f * 400 * 32);
    for (int s = wave; s < 25; s += 4) {
      const f4* p = zf + s * 128;  // 16 pixels x 32 floats = 128 f4
      f4 a = p[lane], b = p[64 + lane];
      acc += a[0] + a[1] + a[2] + a[3] + b[0] + b[1] + b[2] + b[3];
    }
  }
  if (acc == 1.2345f) out[0] = acc;
}

int main() {
  const int frames = 163840;
  const size_t n = (size_t)frames * 400 * 32;
  float *dz, *out;
  CK(hipMalloc(&dz, n * 4));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(dz, 0, n * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int k = 0; k < 2; ++k)
    for (int grid : {256, 512, 1024, 2048}) {
      for (int v = 0; v < 2; ++v) {
        auto fn = v == 0 ? rdA : rdB;
        hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, 0, dz, frames, out, 0);
        CK(hipEventRecord(a));
        for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, 0, dz, frames, out, 0);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= 3;
        if (k) printf("%s grid %5d: %.3f ms  %.2f TB/s\n", v ? "B(16B)" : "A(dword)", grid, ms, n * 4 / ms / 1e9);
      }
    }
  return 0;
}
