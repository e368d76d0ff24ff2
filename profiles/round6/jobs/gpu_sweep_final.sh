#!/bin/bash
# round 6, end: streams per GPU after the MB-loop wait fixes (the driver's 20 / 5 steps, no CPU leg / PMC), interleaved
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6sweepf; mkdir -p $d; out=$d/sweep.txt; : > $out
for r in 1 2; do
  for S in 128 192 256; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --streams $S --no-cpu-baseline --no-traffic > $d/s${S}_$r.json 2> $d/s${S}_$r.err || { echo "$S $r failed" >> $out; tail -5 $d/s${S}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$d/s${S}_$r.json')); print('$r $S', round(d['value'],1), round(d['ms_per_step'],3), round(d['kernels']['enc_mb_kernel']['avg_ms'],3), d['parity']['selfcheck'][-4:])" >> $out
  done
done
cat $out
