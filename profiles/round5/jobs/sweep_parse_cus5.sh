#!/bin/bash
# parse-CU reservation sweep at the driver's invocation (no CPU leg / PMC), interleaved rounds
cd "$(dirname "$0")/../../.."
out=gpurun_out/r5_parse_cus.txt; : > $out
for r in ${RS:-1 2}; do
  for pc in ${PCS:-24 32 40}; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --parse-cus $pc > gpurun_out/r5pc_${pc}_$r.json 2> gpurun_out/r5pc_${pc}_$r.err || { echo "pc $pc failed" >> $out; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r5pc_${pc}_$r.json')); print('$r parse_cus=$pc', round(d['value'],1), round(d['ms_per_step'],3), round(d['kernels']['enc_mb_kernel']['avg_ms'],3), round(d['kernels']['dec_recon_kernel']['avg_ms'],3), d['parity']['vs_oracle'][-4:])" >> $out
  done
done
cat $out
