#!/bin/bash
# encoder / decoder group sweep at the driver's invocation (no CPU leg, no PMC), interleaved rounds
cd "$(dirname "$0")/../../.."
out=gpurun_out/r5_groups.txt; : > $out
for r in 1 2; do
  for cfg in ${CFGS:-1:1 2:1 4:1}; do
    eg=${cfg%%:*}; dg=${cfg##*:}
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --enc-groups $eg --dec-groups $dg > gpurun_out/r5_groups_${eg}_${dg}_$r.json 2> gpurun_out/r5_groups_${eg}_${dg}_$r.err || { echo "eg=$eg dg=$dg failed" >> $out; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r5_groups_${eg}_${dg}_$r.json')); print('$r eg=$eg dg=$dg', round(d['value'],1), round(d['ms_per_step'],3), d['kernels']['enc_mb_kernel'], d['parity']['vs_oracle'][-4:])" >> $out
  done
done
cat $out
