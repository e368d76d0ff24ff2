#!/bin/bash
# encoder rows' wave priority (H264MI_ENC_PRIO) in the full pipeline (decoder beside), interleaved, no CPU leg / PMC
cd "$(dirname "$0")/../../.."
out=gpurun_out/r5_prio_bench.txt; : > $out
for r in 1 2; do
  for p in ${PRIOS:-0 2 3 4}; do
    H264MI_ENC_PRIO=$p timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/r5_pb_${p}_$r.json 2> gpurun_out/r5_pb_${p}_$r.err || { echo "prio=$p failed" >> $out; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r5_pb_${p}_$r.json')); print('$r prio=$p', round(d['value'],1), round(d['ms_per_step'],3), d['kernels']['enc_mb_kernel'], d['kernels']['dec_recon_kernel'])" >> $out
  done
done
cat $out
