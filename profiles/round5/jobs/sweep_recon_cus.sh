#!/bin/bash
# reconstruction on its own CU lane (bench --recon-cus) against sharing the encoder's CUs (no CPU leg / PMC)
cd "$(dirname "$0")/../../.."
out=gpurun_out/r5_recon_cus.txt; : > $out
for r in 1 2; do
  for rc in ${RCS:-0 32 64 96}; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --recon-cus $rc > gpurun_out/r5_rc_${rc}_$r.json 2> gpurun_out/r5_rc_${rc}_$r.err || { echo "rc=$rc failed" >> $out; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r5_rc_${rc}_$r.json')); print('$r recon_cus=$rc', round(d['value'],1), round(d['ms_per_step'],3), round(d['kernels']['enc_mb_kernel']['avg_ms'],3), round(d['kernels']['dec_recon_kernel']['avg_ms'],3), d['parity']['vs_oracle'][-4:])" >> $out
  done
done
cat $out
