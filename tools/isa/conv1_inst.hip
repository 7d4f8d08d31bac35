// ISA / register check of the conv1 kernels alone (fast compile):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -I a2cat-vn-pytorch_amd/csrc \
//     -Rpass-analysis=kernel-resource-usage tools/isa/conv1_inst.hip -o /tmp/isa/conv1.s
#include <hip/hip_runtime.h>
#include "vn_common.h"
#include "vn_gemm.h"
#include "vn_frames.h"
#include "vn_conv1.h"
namespace vn {
template __global__ void conv1_fwd_x3r_kernel<174, 174, 42, 42>(FrameSrc, int, FrameList, const float*, const float*, float*, uint32_t*);
template __global__ void conv1_fwd_x3r_kernel<84, 84, 20, 20>(FrameSrc, int, FrameList, const float*, const float*, float*, uint32_t*);
template __global__ void conv1_fwd_x3r_kernel<300, 400, 74, 99>(FrameSrc, int, FrameList, const float*, const float*, float*, uint32_t*);
template __global__ void conv2_fwd_ring2_kernel<true>(const float*, const float*, const float*, float*, int, FrameList);
template __global__ void conv2_fwd_ring2_kernel<false>(const float*, const float*, const float*, float*, int, FrameList);
template __global__ void conv1_wgrad_x3_kernel<174, 174, 42, 42, true>(FrameSrc, int, FrameList, const float*, float*);
template __global__ void conv1_wgrad_x3_kernel<174, 174, 42, 42, false>(FrameSrc, int, FrameList, const float*, float*);
template __global__ void conv1_wgrad_x3_kernel<84, 84, 20, 20, true>(FrameSrc, int, FrameList, const float*, float*);
template __global__ void conv1_wgrad_x3_kernel<300, 400, 74, 99, true>(FrameSrc, int, FrameList, const float*, float*);
template __global__ void conv2_dgrad_x6_kernel<42, 42, 20, 20, 8, true>(const float*, const float*, const uint32_t*, float*, int, FrameList, float*);
template __global__ void conv2_dgrad_x6_kernel<20, 20, 9, 9, 4, true>(const float*, const float*, const uint32_t*, float*, int, FrameList, float*);
}  // namespace vn
