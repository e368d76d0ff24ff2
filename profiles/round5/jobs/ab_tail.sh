#!/bin/bash
# same-box A/B of the streamed tail (bench --tail-streamed 0 / 1) at the driver's invocation, interleaved
cd "$(dirname "$0")/../../.."
out=gpurun_out/r5_tail.txt; : > $out
for r in 1 2; do
  for ts in 0 1; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --tail-streamed $ts > gpurun_out/r5_tail_${ts}_$r.json 2> gpurun_out/r5_tail_${ts}_$r.err || { echo "ts=$ts failed" >> $out; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r5_tail_${ts}_$r.json')); print('$r tail_streamed=$ts', round(d['value'],1), round(d['ms_per_step'],3), d['kernels']['enc_mb_kernel'], d['config'].get('tail_streamed'), d['parity']['vs_oracle'][-4:], d['parity']['selfcheck'][-30:])" >> $out
  done
done
cat $out
