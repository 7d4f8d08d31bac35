// vn_frames.h — the frame operand of the policy kernels: uint8 scene-cache rows gathered by
// index (image and goal), or dense float NCHW frames.
#pragma once
#include <cstdint>

namespace vn {

struct FrameSrc {
  const uint8_t* base[2];
  const int32_t* rows[2];
  int64_t stride;
  const float* f32[2];  // optional dense float NCHW frames (TransposeImage+ScaledFloatFrame output)
};

// The frames a frame-level kernel (conv1 / conv2 forward, conv2 input / weight gradient,
// conv1 weight gradient) processes. Frame f = 2 * sample + {0: image, 1: goal}.
//   goals == nullptr: every frame 0 .. n_frames - 1 (item i = frame i).
//   goals != nullptr (goal-frame deduplication): items 0 .. nimg - 1 are the image frames
//   2i; items nimg .. nimg + *count - 1 are the goal frames 2 goals[j] + 1 of the samples that
//   start a goal run (the goal frame is the same for every later step of the episode, so its
//   conv1 / conv2 maps are computed once and its gradients summed before the conv2 / conv1
//   backward: vn_goal_runs in include/vnav.h).
struct FrameList {
  const int32_t* goals;
  const int32_t* count;
  int nimg;
};

#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
// Scalar (constant address space) loads: a wave-uniform index read with s_load keeps the
// kernels' vector-memory wait counts exact (a vector load here would make later waits drain
// every prefetch in flight).
__device__ __forceinline__ int fl_sload(const int32_t* p) {
  typedef __attribute__((address_space(4))) const int32_t cint32;
  return *(cint32*)p;
}

// Items of the list (n_frames: the host's count of the identity list / the upper bound).
__device__ __forceinline__ int fl_count(const FrameList& fl, int n_frames) {
  return fl.goals ? fl.nimg + fl_sload(fl.count) : n_frames;
}

// Frame of item i (wave-uniform). An image item still loads goals[0] (allocated: the list
// buffer holds one entry per sample) and discards it, so no branch hides the load.
__device__ __forceinline__ int fl_frame(const FrameList& fl, int i) {
  i = __builtin_amdgcn_readfirstlane(i);
  if (!fl.goals) return i;
  const int j = i - fl.nimg;
  const int g = fl_sload(fl.goals + (j > 0 ? j : 0));
  return j >= 0 ? 2 * g + 1 : 2 * i;
}

// Per-lane form (i differs between lanes: an im2col row's frame), plain vector loads.
__device__ __forceinline__ int fl_frame_v(const FrameList& fl, int i) {
  if (!fl.goals) return i;
  return i < fl.nimg ? 2 * i : 2 * fl.goals[i - fl.nimg] + 1;
}
#endif

}  // namespace vn
