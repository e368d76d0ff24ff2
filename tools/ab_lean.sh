#!/bin/bash
# enc_mb_kernel build choice: auto (by launch size) vs forced lean (H264MI_ENC_LEAN=1) on the low-stream configs
set -o pipefail
out=gpurun_out/ablean; mkdir -p $out
for cfg in 3 5 2; do for v in auto 1; do
  if [ $v = auto ]; then unset H264MI_ENC_LEAN; else export H264MI_ENC_LEAN=$v; fi
  timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline --no-traffic > $out/c${cfg}_$v.log 2>&1 || { echo "config $cfg $v failed"; tail -5 $out/c${cfg}_$v.log; exit 1; }
  echo "config $cfg lean=$v: $(grep -o '"value": [0-9.]*' $out/c${cfg}_$v.log | head -1) $(grep -o '"enc_mb_kernel": {"avg_ms": [0-9.]*' $out/c${cfg}_$v.log)"
done; done
unset H264MI_ENC_LEAN
