#!/bin/bash
# per-XCD ticket queues at higher stream counts (no CPU leg, no PMC), interleaved
cd "$(dirname "$0")/../../.."
out=gpurun_out/r5_xq_cap.txt; : > $out
for S in 64 128; do
  for r in 1 2; do
    for xq in 0 1; do
      H264MI_ENC_XQ=$xq timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --streams $S --parse-cus 48 --no-cpu-baseline --no-traffic > gpurun_out/r5_xqc_${S}_${xq}_$r.json 2> gpurun_out/r5_xqc_${S}_${xq}_$r.err || { echo "S=$S xq=$xq failed" >> $out; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/r5_xqc_${S}_${xq}_$r.json')); print('S=$S $r xq=$xq', round(d['value'],1), round(d['ms_per_step'],3), d['kernels']['enc_mb_kernel'])" >> $out
    done
  done
done
cat $out
