// Shared helpers of libvnav: error reporting and the counter-based RNG.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/vnav.h"

namespace vn {

// Thread-local last-error text (vn_last_error).
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

#define VN_HIP(call)                                  \
  do {                                                \
    hipError_t _e = (call);                           \
    if (_e != hipSuccess) return vn::hip_fail(_e, #call); \
  } while (0)

// ---- Philox4x32-10 (Salmon et al., SC'11) ----------------------------------
// Counter layout used by the engine (DESIGN.md "RNG streams"):
//   ctr = (env, episode, attempt, stream), key = (seed_lo, seed_hi).
struct u32x4 {
  uint32_t x, y, z, w;
};

enum : uint32_t {
  STREAM_GOAL = 0,    // goal / task draw of a reset
  STREAM_START = 1,   // start-state rejection attempts of a reset
  STREAM_ACTION = 2,  // synthetic random actions
  STREAM_POLICY = 3,  // categorical sampling from the policy
  STREAM_REPLAY = 4,  // the replay ring's slot draw (vn_replay_push_draw)
};

__host__ __device__ inline void mulhilo32(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

__host__ __device__ inline u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo32(0xD2511F53u, c.x, hi0, lo0);
    mulhilo32(0xCD9E8D57u, c.z, hi1, lo1);
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Uniform integer in [0, n): multiply-high (bias <= n / 2^32, documented).
__host__ __device__ inline uint32_t uniform_below(uint32_t r, uint32_t n) {
  return (uint32_t)(((uint64_t)r * (uint64_t)n) >> 32);
}

// ---- the policy's categorical draw (vn_a2c.hip sample_kernel, vn_env.hip's fused A2C step) --
__device__ __forceinline__ void softmax_stats(const float* lg, int A, float* p, float* logp, float& H) {
  float mx = lg[0];
  for (int j = 1; j < A; ++j) mx = fmaxf(mx, lg[j]);
  float s = 0.0f;
  for (int j = 0; j < A; ++j) s += expf(lg[j] - mx);
  const float ls = logf(s);
  H = 0.0f;
  for (int j = 0; j < A; ++j) {
    logp[j] = lg[j] - mx - ls;
    p[j] = expf(logp[j]);
    H -= p[j] * logp[j];
  }
}

// Inverse-CDF draw of sample i from the logits lg[0..A-1] (A <= 7): u = the top 24 bits of
// Philox4x32-10 (i, ctr_lo, ctr_hi, STREAM_POLICY) under key (k0, k1). Returns the action;
// p / lp / H receive the distribution, its log and its entropy.
__device__ __forceinline__ int sample_action(const float* lg, int A, uint32_t k0, uint32_t k1, uint64_t ctr,
                                             uint32_t i, float* p, float* lp, float& H) {
  softmax_stats(lg, A, p, lp, H);
  const u32x4 r = philox4x32_10(u32x4{i, (uint32_t)ctr, (uint32_t)(ctr >> 32), STREAM_POLICY}, k0, k1);
  const float u = (float)(r.x >> 8) * (1.0f / 16777216.0f);
  int a = A - 1;
  float c = 0.0f;
  for (int j = 0; j < A - 1; ++j) {
    c += p[j];
    if (u < c) {
      a = j;
      break;
    }
  }
  return a;
}

// Synthetic frame hash: 32-bit word w of frame (scene, state).
__host__ __device__ inline uint32_t frame_hash(uint32_t scene, uint32_t state, uint32_t w) {
  uint32_t x = (w * 0x9E3779B1u) ^ (state * 0x85EBCA77u) ^ (scene * 0xC2B2AE3Du) ^ 0x27D4EB2Fu;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

}  // namespace vn
