// copybench — the vn_step frame-gather pattern in isolation: 4096 envs each copy one random
// image row and one fixed goal row (21,168 B at 84x84x3) of a 626 MB arena into two batch
// buffers. Variants of the copy loop, timed with one event pair around R launches, next to a
// plain float4 copy of the same byte count (the chip's copy ceiling).
//   hipcc -O3 --offload-arch=gfx950 -o tools/copybench tools/copybench.hip && tools/copybench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

static int E = 4096;  // envs (argv[2])
constexpr int F = 21168;  // 84*84*3
constexpr int NV = F / 16;  // 1323 uint4 per frame
constexpr int ROWS = 29564;
constexpr int SETS = 64;

struct Args {
  const uint8_t* arena;
  const int* img_rows;   // [SETS][E]
  const int* goal_rows;  // [E]
  uint8_t* obs;
  uint8_t* goal;
  int set;
  int n;
};

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// K0: current vn_step loop (one wave per env, 4 envs / WG, 4 x 2 loads in flight per lane)
template <int U>
__global__ __launch_bounds__(256) void k_wave_env(Args a) {
  const int lane = threadIdx.x & 63;
  const int e = uni(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int64_t ir = a.img_rows[a.set * a.n + e], gr = a.goal_rows[e];
  const uint4* s1 = reinterpret_cast<const uint4*>(a.arena + ir * F);
  const uint4* s2 = reinterpret_cast<const uint4*>(a.arena + gr * F);
  uint4* d1 = reinterpret_cast<uint4*>(a.obs + (int64_t)e * F);
  uint4* d2 = reinterpret_cast<uint4*>(a.goal + (int64_t)e * F);
  int i = lane;
  for (; i + 64 * (U - 1) < NV; i += 64 * U) {
    uint4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = s1[i + 64 * u];
#pragma unroll
    for (int u = 0; u < U; ++u) y[u] = s2[i + 64 * u];
#pragma unroll
    for (int u = 0; u < U; ++u) d1[i + 64 * u] = x[u];
#pragma unroll
    for (int u = 0; u < U; ++u) d2[i + 64 * u] = y[u];
  }
  for (; i < NV; i += 64) {
    const uint4 x = s1[i], y = s2[i];
    d1[i] = x;
    d2[i] = y;
  }
}

// K1: nontemporal stores (and optionally loads)
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_wave_env_nt(Args a) {
  const int lane = threadIdx.x & 63;
  const int e = uni(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int64_t ir = a.img_rows[a.set * a.n + e], gr = a.goal_rows[e];
  const uint4* s1 = reinterpret_cast<const uint4*>(a.arena + ir * F);
  const uint4* s2 = reinterpret_cast<const uint4*>(a.arena + gr * F);
  uint4* d1 = reinterpret_cast<uint4*>(a.obs + (int64_t)e * F);
  uint4* d2 = reinterpret_cast<uint4*>(a.goal + (int64_t)e * F);
  auto ld = [](const uint4* p) -> uint4 {
    if constexpr (NTL) {
      uint4 v;
      v.x = __builtin_nontemporal_load(&p->x);
      v.y = __builtin_nontemporal_load(&p->y);
      v.z = __builtin_nontemporal_load(&p->z);
      v.w = __builtin_nontemporal_load(&p->w);
      return v;
    } else {
      return *p;
    }
  };
  auto stv = [](uint4* p, uint4 v) {
    if constexpr (NTS) {
      __builtin_nontemporal_store(v.x, &p->x);
      __builtin_nontemporal_store(v.y, &p->y);
      __builtin_nontemporal_store(v.z, &p->z);
      __builtin_nontemporal_store(v.w, &p->w);
    } else {
      *p = v;
    }
  };
  int i = lane;
  for (; i + 64 * (U - 1) < NV; i += 64 * U) {
    uint4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = ld(s1 + i + 64 * u);
#pragma unroll
    for (int u = 0; u < U; ++u) y[u] = ld(s2 + i + 64 * u);
#pragma unroll
    for (int u = 0; u < U; ++u) stv(d1 + i + 64 * u, x[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) stv(d2 + i + 64 * u, y[u]);
  }
  for (; i < NV; i += 64) {
    const uint4 x = ld(s1 + i), y = ld(s2 + i);
    stv(d1 + i, x);
    stv(d2 + i, y);
  }
}

// K1b: per-stream policy, CV bits: 1/2 = nt store image/goal output, 4/8 = nt load image/goal
template <bool NT>
__device__ __forceinline__ uint4 ldp(const uint4* p) {
  if constexpr (NT) {
    uint4 v;
    v.x = __builtin_nontemporal_load(&p->x);
    v.y = __builtin_nontemporal_load(&p->y);
    v.z = __builtin_nontemporal_load(&p->z);
    v.w = __builtin_nontemporal_load(&p->w);
    return v;
  } else {
    return *p;
  }
}
template <bool NT>
__device__ __forceinline__ void stp(uint4* p, uint4 v) {
  if constexpr (NT) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
    __builtin_nontemporal_store(v.z, &p->z);
    __builtin_nontemporal_store(v.w, &p->w);
  } else {
    *p = v;
  }
}
template <int CV>
__global__ __launch_bounds__(256) void k_policy(Args a) {
  constexpr int U = 4;
  const int lane = threadIdx.x & 63;
  const int e = uni(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int64_t ir = a.img_rows[a.set * a.n + e], gr = a.goal_rows[e];
  const uint4* s1 = reinterpret_cast<const uint4*>(a.arena + ir * F);
  const uint4* s2 = reinterpret_cast<const uint4*>(a.arena + gr * F);
  uint4* d1 = reinterpret_cast<uint4*>(a.obs + (int64_t)e * F);
  uint4* d2 = reinterpret_cast<uint4*>(a.goal + (int64_t)e * F);
  int i = lane;
  for (; i + 64 * (U - 1) < NV; i += 64 * U) {
    uint4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = ldp<(CV & 4) != 0>(s1 + i + 64 * u);
#pragma unroll
    for (int u = 0; u < U; ++u) y[u] = ldp<(CV & 8) != 0>(s2 + i + 64 * u);
#pragma unroll
    for (int u = 0; u < U; ++u) stp<(CV & 1) != 0>(d1 + i + 64 * u, x[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) stp<(CV & 2) != 0>(d2 + i + 64 * u, y[u]);
  }
  for (; i < NV; i += 64) {
    const uint4 x = ldp<(CV & 4) != 0>(s1 + i), y = ldp<(CV & 8) != 0>(s2 + i);
    stp<(CV & 1) != 0>(d1 + i, x);
    stp<(CV & 2) != 0>(d2 + i, y);
  }
}

// K2: one wave per frame (2 waves per env), WG = 4 waves = 2 envs
template <int U>
__global__ __launch_bounds__(256) void k_wave_frame(Args a) {
  const int lane = threadIdx.x & 63;
  const int w = uni(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int e = w >> 1, which = w & 1;
  const int64_t r = which ? a.goal_rows[e] : a.img_rows[a.set * a.n + e];
  const uint4* s = reinterpret_cast<const uint4*>(a.arena + r * F);
  uint4* d = reinterpret_cast<uint4*>((which ? a.goal : a.obs) + (int64_t)e * F);
  int i = lane;
  for (; i + 64 * (U - 1) < NV; i += 64 * U) {
    uint4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = s[i + 64 * u];
#pragma unroll
    for (int u = 0; u < U; ++u) d[i + 64 * u] = x[u];
  }
  for (; i < NV; i += 64) d[i] = s[i];
}

// K3: whole workgroup (256 thr) per env: 4 waves share the two frames (1323 uint4 per frame)
template <int U>
__global__ __launch_bounds__(256) void k_wg_env(Args a) {
  const int t = threadIdx.x;
  const int e = blockIdx.x;
  const int64_t ir = a.img_rows[a.set * a.n + e], gr = a.goal_rows[e];
  const uint4* s1 = reinterpret_cast<const uint4*>(a.arena + ir * F);
  const uint4* s2 = reinterpret_cast<const uint4*>(a.arena + gr * F);
  uint4* d1 = reinterpret_cast<uint4*>(a.obs + (int64_t)e * F);
  uint4* d2 = reinterpret_cast<uint4*>(a.goal + (int64_t)e * F);
  int i = t;
  for (; i + 256 * (U - 1) < NV; i += 256 * U) {
    uint4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = s1[i + 256 * u];
#pragma unroll
    for (int u = 0; u < U; ++u) y[u] = s2[i + 256 * u];
#pragma unroll
    for (int u = 0; u < U; ++u) d1[i + 256 * u] = x[u];
#pragma unroll
    for (int u = 0; u < U; ++u) d2[i + 256 * u] = y[u];
  }
  for (; i < NV; i += 256) {
    const uint4 x = s1[i], y = s2[i];
    d1[i] = x;
    d2[i] = y;
  }
}

// K6: traffic split probes (same geometry as K0, nt image loads): MODE 0 = read both frames,
// write image output only; 1 = read image only, write both outputs; 2 = write both outputs
// only (no reads); 3 = read both only (xor into one dword per lane)
template <int MODE>
__global__ __launch_bounds__(256) void k_probe(Args a) {
  const int lane = threadIdx.x & 63;
  const int e = uni(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int64_t ir = a.img_rows[a.set * a.n + e], gr = a.goal_rows[e];
  const uint4* s1 = reinterpret_cast<const uint4*>(a.arena + ir * F);
  const uint4* s2 = reinterpret_cast<const uint4*>(a.arena + gr * F);
  uint4* d1 = reinterpret_cast<uint4*>(a.obs + (int64_t)e * F);
  uint4* d2 = reinterpret_cast<uint4*>(a.goal + (int64_t)e * F);
  uint32_t acc = 0;
  for (int i = lane; i < NV; i += 64) {
    if constexpr (MODE == 0) {
      const uint4 x = s1[i], y = s2[i];
      d1[i] = make_uint4(x.x ^ y.x, x.y ^ y.y, x.z ^ y.z, x.w ^ y.w);
    } else if constexpr (MODE == 1) {
      const uint4 x = s1[i];
      d1[i] = x;
      d2[i] = x;
    } else if constexpr (MODE == 2) {
      const uint4 x = make_uint4(i, e, 0, 0);
      d1[i] = x;
      d2[i] = x;
    } else {
      const uint4 x = s1[i], y = s2[i];
      acc ^= x.x ^ y.y ^ x.z ^ y.w;
    }
  }
  if constexpr (MODE == 3) if (acc == 0x12345678u) d1[lane] = make_uint4(acc, 0, 0, 0);
}

// K4: flat float4 copy of the same byte count (2 x E x F read, same written), grid-stride
__global__ __launch_bounds__(256) void k_flat(const uint4* __restrict__ s, uint4* __restrict__ d, int64_t n) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) d[i] = s[i];
}

// K5: flat copy, one pass, exact grid (each thread U elements)
template <int U>
__global__ __launch_bounds__(256) void k_flat_exact(const uint4* __restrict__ s, uint4* __restrict__ d, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  uint4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (base + 256 * u < n) x[u] = s[base + 256 * u];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (base + 256 * u < n) d[base + 256 * u] = x[u];
}

template <typename L>
float time_it(L launch, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 20; ++i) launch(i);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) launch(i);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms * 1000.f / reps;  // us per launch
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 300;
  if (argc > 2) E = atoi(argv[2]);
  const int quick = argc > 3 ? atoi(argv[3]) : 0;
  uint8_t *arena, *obs, *goal;
  int *img_rows, *goal_rows;
  CK(hipMalloc(&arena, (size_t)ROWS * F));
  CK(hipMalloc(&obs, (size_t)E * F));
  CK(hipMalloc(&goal, (size_t)E * F));
  CK(hipMalloc(&img_rows, (size_t)SETS * E * 4));
  CK(hipMalloc(&goal_rows, (size_t)E * 4));
  CK(hipMemset(arena, 7, (size_t)ROWS * F));
  std::vector<int> h(SETS * E), g(E);
  srand(1);
  for (auto& v : h) v = rand() % ROWS;
  for (auto& v : g) v = rand() % ROWS;
  CK(hipMemcpy(img_rows, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(goal_rows, g.data(), g.size() * 4, hipMemcpyHostToDevice));
  const double bytes = 4.0 * E * F;
  auto rep = [&](const char* name, float us) {
    printf("%-34s %8.2f us  %7.0f GB/s  frac %.3f\n", name, us, bytes / (us * 1e-6) / 1e9, bytes / (us * 1e-6) / 8e12);
  };
  Args A{arena, img_rows, goal_rows, obs, goal, 0, E};
  printf("E = %d envs\n", E);
  auto envk = [&](auto kern, int grid) {
    return [=](int i) mutable {
      Args b = A;
      b.set = i % SETS;
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, b);
    };
  };
  {
    char nm[64];
#define POL(cv)                                                         \
  snprintf(nm, sizeof nm, "policy cv%-2d (st i%d g%d, nt-ld i%d g%d)", cv, cv & 1, (cv >> 1) & 1, (cv >> 2) & 1, \
           (cv >> 3) & 1);                                              \
  rep(nm, time_it(envk(k_policy<cv>, E / 4), reps));
    for (int round = 0; round < (quick ? 1 : 2); ++round) {
      POL(0) POL(1) POL(2) POL(3) POL(4) POL(5) POL(6) POL(7) POL(8) POL(9) POL(10) POL(11) POL(12) POL(13) POL(14) POL(15)
    }
  }
  rep("wave/env U4 (vn_step)", time_it(envk(k_wave_env<4>, E / 4), reps));
  rep("wave/env U2", time_it(envk(k_wave_env<2>, E / 4), reps));
  rep("wave/env U8", time_it(envk(k_wave_env<8>, E / 4), reps));
  rep("wave/env U4 nt-store", time_it(envk(k_wave_env_nt<4, false, true>, E / 4), reps));
  rep("wave/env U4 nt-load", time_it(envk(k_wave_env_nt<4, true, false>, E / 4), reps));
  rep("wave/env U4 nt-both", time_it(envk(k_wave_env_nt<4, true, true>, E / 4), reps));
  rep("wave/frame U4", time_it(envk(k_wave_frame<4>, E / 2), reps));
  rep("wave/frame U8", time_it(envk(k_wave_frame<8>, E / 2), reps));
  rep("wg/env U2", time_it(envk(k_wg_env<2>, E), reps));
  rep("wg/env U1", time_it(envk(k_wg_env<1>, E), reps));
  rep("wave/env U4 (again)", time_it(envk(k_wave_env<4>, E / 4), reps));
  if (!quick) {  // traffic probes; bytes column still counts the full 4F per env
    rep("probe rd2 wr1 (3F)", time_it(envk(k_probe<0>, E / 4), reps));
    rep("probe rd1 wr2 (3F)", time_it(envk(k_probe<1>, E / 4), reps));
    rep("probe wr2 only (2F)", time_it(envk(k_probe<2>, E / 4), reps));
    rep("probe rd2 only (2F)", time_it(envk(k_probe<3>, E / 4), reps));
    // hot goal rows: every env's goal among 64 rows (L2/MALL resident)
    std::vector<int> hot(E);
    for (int i = 0; i < E; ++i) hot[i] = g[i % 64];
    int* hot_rows;
    CK(hipMalloc(&hot_rows, (size_t)E * 4));
    CK(hipMemcpy(hot_rows, hot.data(), hot.size() * 4, hipMemcpyHostToDevice));
    Args H = A;
    H.goal_rows = hot_rows;
    auto hk = [&](auto kern) {
      return [=](int i) mutable {
        Args b = H;
        b.set = i % SETS;
        hipLaunchKernelGGL(kern, dim3(E / 4), dim3(256), 0, 0, b);
      };
    };
    rep("hot goals U4", time_it(hk(k_wave_env<4>), reps));
    rep("hot goals U4 nt-store", time_it(hk(k_wave_env_nt<4, false, true>), reps));
    rep("hot goals U4 nt-load", time_it(hk(k_wave_env_nt<4, true, false>), reps));
  }
  // flat copies of 2*E*F bytes (src = first rows of the arena; dst = obs..goal contiguous? use obs+goal as one)
  // flat copies of 2*E*F bytes from a source of that size (the arena is smaller at large E)
  uint8_t *dst, *src;
  CK(hipMalloc(&dst, (size_t)2 * E * F));
  CK(hipMalloc(&src, (size_t)2 * E * F));
  CK(hipMemset(src, 3, (size_t)2 * E * F));
  const int64_t n = (int64_t)2 * E * F / 16;
  for (int blocks : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, sizeof nm, "flat grid-stride %d WGs", blocks);
    rep(nm, time_it([=](int) { hipLaunchKernelGGL(k_flat, dim3(blocks), dim3(256), 0, 0, (const uint4*)src, (uint4*)dst, n); }, reps));
  }
  rep("flat exact U4", time_it([=](int) {
        hipLaunchKernelGGL(k_flat_exact<4>, dim3((n + 1023) / 1024), dim3(256), 0, 0, (const uint4*)src, (uint4*)dst, n);
      }, reps));
  rep("flat exact U8", time_it([=](int) {
        hipLaunchKernelGGL(k_flat_exact<8>, dim3((n + 2047) / 2048), dim3(256), 0, 0, (const uint4*)src, (uint4*)dst, n);
      }, reps));
  rep("hipMemcpyAsync D2D", time_it([=](int) { (void)hipMemcpyAsync(dst, src, (size_t)2 * E * F, hipMemcpyDeviceToDevice, 0); }, reps));
  // flat copy of 8x the bytes: steady-state ceiling without launch ramp
  {
    uint8_t* big;  // copy its first half (4 x the bytes) into its second half
    CK(hipMalloc(&big, (size_t)16 * E * F));
    const int64_t nb = (int64_t)8 * E * F / 16;
    float us = time_it([=](int) { hipLaunchKernelGGL(k_flat, dim3(8192), dim3(256), 0, 0, (const uint4*)big, (uint4*)(big + (size_t)8 * E * F), nb); }, reps / 4);
    printf("%-34s %8.2f us  %7.0f GB/s (4x bytes, steady state)\n", "flat grid-stride 8192 WGs x4", us,
           4 * bytes / (us * 1e-6) / 1e9);
  }
  printf("done\n");
  return 0;
}
