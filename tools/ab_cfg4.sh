#!/bin/bash
# config-4 (decode-only) bench for variant libraries (lib/var_<name>.so, "base" = lib/libh264mi.so)
set -o pipefail
root=$(pwd); out=gpurun_out/abc4; mkdir -p $out
for v in "$@"; do
  lib=$root/openh264-wasm_amd/lib/libh264mi.so; [ $v != base ] && lib=$root/openh264-wasm_amd/lib/var_$v.so
  H264MI_LIB=$lib timeout -k 10 300 python3 bench.py --config 4 --no-cpu-baseline --no-traffic > $out/$v.log 2>&1 || { echo "$v failed"; tail -5 $out/$v.log; exit 1; }
  echo "$v config4: $(grep -o '"value": [0-9.]*' $out/$v.log | head -1) $(grep -o '"dec_recon_kernel": {"avg_ms": [0-9.]*' $out/$v.log)"
done
