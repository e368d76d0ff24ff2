#!/bin/bash
# same-box A/B of the per-XCD ticket queues (H264MI_ENC_XQ) with the in-run traffic passes, interleaved
cd "$(dirname "$0")/../../.."
out=gpurun_out/r5_xq.txt; : > $out
for r in 1 2; do
  for xq in 0 1; do
    H264MI_ENC_XQ=$xq timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5_xq_${xq}_$r.json 2> gpurun_out/r5_xq_${xq}_$r.err || { echo "xq=$xq failed" >> $out; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r5_xq_${xq}_$r.json')); r=d['roofline']; print('$r xq=$xq', round(d['value'],1), round(d['ms_per_step'],3), round(r['avg_launch_ms'],3), r['traffic_range'], round(r['traffic_x_alg'],2), d['parity']['vs_oracle'][-4:])" >> $out
  done
done
cat $out
