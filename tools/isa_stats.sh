#!/bin/bash
# Device ISA statistics of one kernel of libh264mi (register counts, spills, selected opcodes).
# usage: tools/isa_stats.sh <kernel-substring>   e.g. tools/isa_stats.sh 16dec_parse_kernel
set -e
k=$1
mkdir -p /tmp/isa
hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o /tmp/isa/all.s openh264-wasm_amd/csrc/h264mi_kernels.hip -Wno-unused-result 2>/dev/null
name=$(grep -o "^_ZN6h264mi[0-9]*${k}[A-Za-z0-9_]*:" /tmp/isa/all.s | head -1 | tr -d :)
s=$(grep -n "^${name}:" /tmp/isa/all.s | cut -d: -f1)
e=$(grep -n "${name}.uses_flat_scratch" /tmp/isa/all.s | cut -d: -f1)
sed -n "${s},${e}p" /tmp/isa/all.s > /tmp/isa/k.s
echo "$name lines $(wc -l < /tmp/isa/k.s)"
grep -A40 "\.name:           ${name}$" /tmp/isa/all.s | grep -E "sgpr_count|vgpr_count|spill_count|private_segment" | head -6
for op in v_readlane v_writelane s_waitcnt v_cmp_ v_cndmask s_load ds_read flat_ scratch_ s_cbranch; do echo "$op $(grep -c "$op" /tmp/isa/k.s)"; done
