// ISA / register check of the aux second-layer kernels alone (fast compile):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -I a2cat-vn-pytorch_amd/csrc \
//     -Rpass-analysis=kernel-resource-usage tools/isa/aux_inst.hip -o /tmp/isa/aux.s
#include <hip/hip_runtime.h>
#include "vn_common.h"
#include "vn_gemm.h"
#include "vn_aux.h"
namespace vn {
template __global__ void aux_deconv2_kernel<20, 20, 42, 42, true>(const float*, int, const float*, const float*, float*, const f4*, const int32_t*, const int32_t*, float, float*, float*);
}  // namespace vn
