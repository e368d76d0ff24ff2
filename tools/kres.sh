#!/bin/bash
# resource usage (VGPRs, spills, scratch, occupancy) of the library's kernels: a device-only compile with
# the kernel-resource-usage remarks.   usage: tools/kres.sh [kernel-name-regex] [extra hipcc flags]
cd "$(dirname "$0")/.."
pat=${1:-enc_mb_kernel}; shift
hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -c -o /tmp/kres.o -Wno-unused-result -Wno-pass-failed \
  -Rpass-analysis=kernel-resource-usage "$@" openh264-wasm_amd/csrc/h264mi_kernels.hip 2>&1 |
  awk -v pat="$pat" '/Function Name:/ {on = ($0 ~ pat)} on && /remark/ {sub(/.*remark: /, ""); print}'
