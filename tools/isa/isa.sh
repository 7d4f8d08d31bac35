#!/bin/bash
# tools/isa/isa.sh [extra hipcc flags]: compile tools/isa/conv1_inst.hip to /tmp/isa/conv1.s and print
# each kernel's registers, spills and occupancy
mkdir -p /tmp/isa
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -I a2cat-vn-pytorch_amd/csrc \
  -Rpass-analysis=kernel-resource-usage "$@" tools/isa/conv1_inst.hip -o /tmp/isa/conv1.s 2>&1 |
  grep -E "error|Function Name|VGPRs|AGPRs|Spill: [1-9]|Occupancy|ScratchSize" | sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//'
