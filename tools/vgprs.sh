#!/bin/bash
# Register / occupancy report of the device kernels (CPU only: hipcc resource-usage remarks).
#   tools/vgprs.sh [extra hipcc flags]  -> kernel, VGPRs, AGPRs, spills, LDS, occupancy
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -fno-gpu-rdc \
  --cuda-device-only -c directcomputeraytracing_amd/csrc/device/tracer.hip -o /tmp/vgprs.o "$@" \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m: cur = m.group(1); continue
    for key in ("VGPRs:", "AGPRs:", "ScratchSize", "Occupancy", "VGPRs Spill"):
        if key in line and cur and ("cast_kernel" in cur or "material_kernel" in cur or "control_kernel" in cur or "megakernel" in cur or "drain_kernel" in cur):
            print(cur[:60], line.split("remark:")[-1].strip())
'
