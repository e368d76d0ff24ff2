#!/bin/bash
# build libh264mi variants with extra -D flags: tools/build_variants.sh name="-DX=1 -DY=2" ...
set -e
mkdir -p openh264-wasm_amd/lib/variants
for kv in "$@"; do
  name=${kv%%=*}; flags=${kv#*=}
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -Wno-pass-failed $flags \
    -o openh264-wasm_amd/lib/variants/$name.so openh264-wasm_amd/csrc/h264mi_kernels.hip &
done
wait
ls -la openh264-wasm_amd/lib/variants
