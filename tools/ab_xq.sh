#!/bin/bash
# encoder ticket queues: one global queue (H264MI_ENC_XQ=0) vs per-XCD queues (default), 240 and 20 steps
set -o pipefail
out=gpurun_out/abxq; mkdir -p $out
for r in 1 2; do for v in 0 1; do for st in 240:16 20:5; do
  k=${st%%:*}; w=${st##*:}
  H264MI_ENC_XQ=$v timeout -k 10 300 python3 bench.py --steps $k --warmup $w --no-cpu-baseline --no-traffic > $out/xq${v}_${k}_$r.log 2>&1 || { echo "xq $v failed"; tail -5 $out/xq${v}_${k}_$r.log; exit 1; }
  echo "xq=$v steps $k round $r: $(grep -o '"value": [0-9.]*' $out/xq${v}_${k}_$r.log | head -1) $(grep -o '"enc_mb_kernel": {"avg_ms": [0-9.]*' $out/xq${v}_${k}_$r.log)"
done; done; done
