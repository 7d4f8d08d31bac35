// mfma_clock.hip — the chip's sustained bf16 MFMA rate and shader clock under a dense
// v_mfma_f32_32x32x16_bf16 load (every SIMD busy, random operands), to price the x6 GEMM
// core against what the part sustains rather than the 2.4 GHz datasheet peak.
// Clock = d(s_memtime) / d(s_memrealtime) x 100 MHz (MI355X_MICROARCH.md, timing recipe).
//   hipcc -O3 --offload-arch=gfx950 -o tools/mfma_clock tools/mfma_clock.hip && tools/mfma_clock
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void mfma_loop(const uint4* __restrict__ seed, int iters, float* out,
                                                 unsigned long long* clk) {
  const int tid = threadIdx.x;
  union { uint4 q; bf16x8 v; } a0, a1, b0, b1;
  a0.q = seed[tid];
  a1.q = seed[tid + 256];
  b0.q = seed[tid + 512];
  b1.q = seed[tid + 768];
  f16v acc[4];
  for (int j = 0; j < 4; ++j)
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0.v, b0.v, acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1.v, b0.v, acc[1], 0, 0, 0);
    acc[2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0.v, b1.v, acc[2], 0, 0, 0);
    acc[3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1.v, b1.v, acc[3], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.0f;
  for (int j = 0; j < 4; ++j)
    for (int r = 0; r < 16; ++r) s += acc[j][r];
  out[blockIdx.x * 256 + tid] = s;
  if (tid == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 2;  // 8 waves per CU: 2 per SIMD
  std::vector<uint4> h(1024);
  unsigned x = 12345;
  for (auto& q : h) {
    unsigned w[4];
    for (int k = 0; k < 4; ++k) {
      x = x * 1664525u + 1013904223u;
      w[k] = (x & 0x7f7f7f7fu) | 0x3c003c00u;  // finite, non-zero bf16 pairs
    }
    q = make_uint4(w[0], w[1], w[2], w[3]);
  }
  uint4* d_seed;
  float* d_out;
  unsigned long long* d_clk;
  (void)hipMalloc(&d_seed, 1024 * sizeof(uint4));
  (void)hipMalloc(&d_out, (size_t)blocks * 256 * 4);
  (void)hipMalloc(&d_clk, (size_t)blocks * 16);
  (void)hipMemcpy(d_seed, h.data(), 1024 * sizeof(uint4), hipMemcpyHostToDevice);
  const int iters = 20000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 800; ++rep) hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, d_seed, iters, d_out, d_clk);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0, 0);
  const int reps = 200;
  for (int rep = 0; rep < reps; ++rep)
    hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, d_seed, iters, d_out, d_clk);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> c((size_t)blocks * 2);
  (void)hipMemcpy(c.data(), d_clk, c.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> mhz;
  for (int b = 0; b < blocks; ++b)
    if (c[2 * b + 1]) mhz.push_back((double)c[2 * b] / (double)c[2 * b + 1] * 100.0);
  std::sort(mhz.begin(), mhz.end());
  const double flops = (double)reps * blocks * 4 /*waves*/ * iters * 4 * 32768.0;
  printf("CUs %d, %d workgroups x 4 waves, %d x 4 MFMA 32x32x16 bf16 per wave per launch\n", cus, blocks, iters);
  printf("sustained: %.0f TFLOP/s bf16 (%.1f%% of 2.5 PF), clock median %.0f MHz (min %.0f, max %.0f)\n",
         flops / (ms * 1e-3) / 1e12, 100.0 * flops / (ms * 1e-3) / 2.5e15, mhz[mhz.size() / 2], mhz.front(), mhz.back());
  return 0;
}
