#!/bin/bash
# A/B of variant libraries (lib/var_<name>.so, "base" = lib/libh264mi.so) on the 240-step bench, interleaved
set -o pipefail
root=$(pwd); out=gpurun_out/abb; mkdir -p $out; rounds=${ROUNDS:-2}
for r in $(seq $rounds); do for v in "$@"; do
  lib=$root/openh264-wasm_amd/lib/libh264mi.so; [ $v != base ] && lib=$root/openh264-wasm_amd/lib/var_$v.so
  H264MI_LIB=$lib timeout -k 10 300 python3 bench.py --steps 240 --warmup 16 --no-cpu-baseline --no-traffic > $out/${v}_$r.log 2>&1 || { echo "$v failed"; tail -5 $out/${v}_$r.log; exit 1; }
  echo "$v round $r: $(grep -o '"value": [0-9.]*' $out/${v}_$r.log | head -1) $(grep -o '"enc_mb_kernel": {"avg_ms": [0-9.]*' $out/${v}_$r.log)"
done; done
