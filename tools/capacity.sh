#!/bin/bash
# per-GPU throughput vs independent streams per GPU (1080p IPPP encode+decode, 1 Mbps) -> gpurun_out/<out>/
set -o pipefail
out=gpurun_out/${1:-capacity}; mkdir -p $out
for s in 4 8 16 32 48; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic --streams $s --steps 96 --warmup 16 > $out/s$s.log 2>&1 || { echo "streams $s failed"; tail -5 $out/s$s.log; exit 1; }
  echo "streams $s: $(grep -o '"value": [0-9.]*' $out/s$s.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $out/s$s.log) $(grep -o '"enc_mb_kernel": {"avg_ms": [0-9.]*' $out/s$s.log)"
done
