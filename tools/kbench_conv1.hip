// Standalone timing harness for the conv1 kernels of vn_conv1.h on synthetic frames and dZ
// (the 84x84 training shape: 2 x 81920 frames). Build:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I a2cat-vn-pytorch_amd/csrc tools/kbench_conv1.hip -o tools/kbench_conv1
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "vn_common.h"
#include "vn_gemm.h"
#include "vn_frames.h"
#include "vn_conv1.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

using namespace vn;

__global__ void fill_u8(uint8_t* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] = (uint8_t)((i * 2654435761u) >> 13);
}
__global__ void fill_f(float* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] = (float)((int)((i * 2654435761u) >> 9 & 1023) - 512) * 1e-3f;
}
__global__ void fill_rows(int32_t* r, int n, int rows) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) r[i] = (int)((i * 2654435761u) % rows);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 81920, frames = 2 * n, arena = 30000;
  const int64_t fb = 84 * 84 * 3;
  uint8_t* ar; int32_t *ri, *rg; float *dz, *slab;
  CK(hipMalloc(&ar, arena * fb));
  CK(hipMalloc(&ri, n * 4)); CK(hipMalloc(&rg, n * 4));
  CK(hipMalloc(&dz, (size_t)frames * 400 * 32 * 4));
  CK(hipMalloc(&slab, (size_t)4096 * 32 * 160 * 4));
  hipLaunchKernelGGL(fill_u8, dim3((arena * fb + 255) / 256), dim3(256), 0, 0, ar, (size_t)arena * fb);
  hipLaunchKernelGGL(fill_f, dim3(((size_t)frames * 12800 + 255) / 256), dim3(256), 0, 0, dz, (size_t)frames * 12800);
  hipLaunchKernelGGL(fill_rows, dim3((n + 255) / 256), dim3(256), 0, 0, ri, n, arena);
  hipLaunchKernelGGL(fill_rows, dim3((n + 255) / 256), dim3(256), 0, 0, rg, n, arena - 7);
  FrameSrc src{{ar, ar}, {ri, rg}, fb, {nullptr, nullptr}};
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const char* which = argc > 2 ? argv[2] : "wgrad";
  float *dz2, *wt, *dx1; uint32_t* msk;
  CK(hipMalloc(&dz2, (size_t)frames * 81 * 32 * 4));
  CK(hipMalloc(&wt, 16 * 32 * 32 * 4));
  CK(hipMalloc(&msk, (size_t)frames * 400 * 4));
  dx1 = dz;  // reuse: frames x 400 x 32
  hipLaunchKernelGGL(fill_f, dim3(((size_t)frames * 81 * 32 + 255) / 256), dim3(256), 0, 0, dz2, (size_t)frames * 81 * 32);
  hipLaunchKernelGGL(fill_f, dim3((16 * 32 * 32 + 255) / 256), dim3(256), 0, 0, wt, (size_t)16 * 32 * 32);
  hipLaunchKernelGGL(fill_f, dim3(((size_t)frames * 400 + 255) / 256), dim3(256), 0, 0, (float*)msk, (size_t)frames * 400);
  constexpr size_t dlds = conv2_dgrad_x6_lds<20, 20, 9, 9>();
  CK(hipFuncSetAttribute((const void*)conv2_dgrad_x6_kernel<20, 20, 9, 9, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dlds));
  for (int grid : {512, 768, 1024}) {
    auto run = [&]() {
      if (which[0] == 'w')
        hipLaunchKernelGGL((conv1_wgrad_x3_kernel<84, 84, 20, 20>), dim3(grid), dim3(256), (Conv1WgBand<84, 84>::LDS), 0, src, frames, FrameList{}, dz, slab);
      else if (which[0] == 'd')
        hipLaunchKernelGGL((conv2_dgrad_x6_kernel<20, 20, 9, 9, 4>), dim3(grid), dim3(256), dlds, 0, dz2, wt, msk, dx1, frames, FrameList{}, slab);
      else
        hipLaunchKernelGGL((conv2_dgrad_kernel<20, 20, 9, 9, true>), dim3(grid), dim3(256), 0, 0, dz2, wt, dx1, msk, dx1, frames);
    };
    run();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) run();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    printf("%s grid %d: %.3f ms\n", which, grid, ms / 5);
  }
  return 0;
}
