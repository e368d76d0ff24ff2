#!/bin/bash
# vmcnt waits and vector loads of enc_mb_kernel's P path start (between the H264MI_ISA_MARK markers, an asm-comment
# build): a device-only -S compile, the lean (<false>) instance.   usage: tools/isa_waits.sh tag [extra hipcc flags]
cd "$(dirname "$0")/.."
tag=${1:-base}; shift
hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o /tmp/isa_$tag.s -Wno-unused-result -Wno-pass-failed \
  -DH264MI_ISA_MARK "$@" openh264-wasm_amd/csrc/h264mi_kernels.hip 2>/dev/null || exit 1
awk '/^_ZN6h264mi13enc_mb_kernelILb0/{on=1} on' /tmp/isa_$tag.s > /tmp/isa_${tag}_lean.s
echo "vmcnt waits in the kernel: $(grep -c 'vmcnt' /tmp/isa_${tag}_lean.s)"
awk '/MARK_PSTART/{on=1} on{print NR": "$0} /MARK_JUDGE/{exit}' /tmp/isa_${tag}_lean.s | grep -E "MARK|vmcnt|global_load"
