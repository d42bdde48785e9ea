#!/bin/bash
# Per-kernel VGPR / LDS / occupancy of one kernel source as the production build compiles it:
#   scripts/r5/kres.sh alphago_amd/csrc/kernels/conv.hip [name-filter]
src=$1; filt=${2:-.}
TORCH_INC=$(python -c "import torch.utils.cpp_extension as c; print(' '.join('-I'+p for p in c.include_paths(device_type='cuda')))")
PY_INC=$(python -c "import sysconfig; print(sysconfig.get_paths()['include'])")
/opt/rocm/bin/hipcc -x hip -O3 -std=c++17 -fPIC -DUSE_ROCM=1 -D__HIP_PLATFORM_AMD__=1 -Wno-unused-result \
  -Wno-deprecated-declarations --offload-arch=gfx950 -fno-gpu-rdc -munsafe-fp-atomics $TORCH_INC -I$PY_INC \
  -Ialphago_amd/csrc/kernels -c "$src" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep -E "remark: .*(Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size)" \
  | sed -E 's/.*remark: //' | awk -v f="$filt" '/Function Name/{keep = ($0 ~ f)} keep'
