#!/bin/bash
# round-5 capacity sweep: streams per GPU x reserved parse CUs, the driver's 20 / 5 steps (no CPU leg, no PMC)
cd "$(dirname "$0")/../../.."
out=gpurun_out/r5_cap_sweep.txt; : > $out
for cfg in "64 48" "64 64" "96 48" "96 64" "128 64" "128 96"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --streams $1 --parse-cus $2 --no-cpu-baseline --no-traffic > gpurun_out/r5_cap_s$1_p$2.json 2> gpurun_out/r5_cap_s$1_p$2.err || { echo "S=$1 P=$2 failed rc=$?" >> $out; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5_cap_s$1_p$2.json')); print('S=$1 parse_cus=$2', round(d['value'],1), round(d['ms_per_step'],3), round(d['kernels']['enc_mb_kernel']['avg_ms'],3), round(d['kernels']['dec_recon_kernel']['avg_ms'],3), round(d['kernels']['dec_parse_kernel']['avg_ms'],3), d['parity']['vs_oracle'][-30:])" >> $out
done
cat $out
