#!/bin/bash
# enc_prof.py section profile (32 streams) for variant libraries lib/var_<name>.so
set -o pipefail
root=$(pwd)
for v in "$@"; do
  echo "== $v"
  H264MI_LIB=$root/openh264-wasm_amd/lib/var_$v.so timeout -k 10 300 python3 tools/enc_prof.py 1920 1080 1000000 32 4 2>&1 | grep -v amdgpu | tail -2 || exit 1
done
