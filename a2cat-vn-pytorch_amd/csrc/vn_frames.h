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

}  // namespace vn
