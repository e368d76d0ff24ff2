#!/bin/bash
# what slows the encoder inside the pipeline: the bench as is, encode only on the masked wavefront CUs, encode
# only on every CU (no CPU leg / PMC)
cd "$(dirname "$0")/../../.."
out=gpurun_out/r5_contention.txt; : > $out
for r in 1 2; do
  for cfg in "full:" "enc-masked:--no-decode" "enc-all:--no-decode --parse-cus 0"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic $args > gpurun_out/r5_ct_${name}_$r.json 2> gpurun_out/r5_ct_${name}_$r.err || { echo "$name failed" >> $out; tail -3 gpurun_out/r5_ct_${name}_$r.err >> $out; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r5_ct_${name}_$r.json')); print('$r $name', round(d['value'],1), round(d['ms_per_step'],3), d['kernels'].get('enc_mb_kernel'), d['kernels'].get('dec_recon_kernel'))" >> $out
  done
done
cat $out
