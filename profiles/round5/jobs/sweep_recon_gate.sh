#!/bin/bash
# bench --recon-gate fraction sweep (no CPU leg / PMC), interleaved rounds
cd "$(dirname "$0")/../../.."
out=gpurun_out/r5_recon_gate_frac.txt; : > $out
for r in 1 2; do
  for f in ${FRACS:-off 0.5 0.75 1.0}; do
    if [ $f = off ]; then args="--recon-gate 0"; else args="--recon-gate 1 --recon-gate-frac $f"; fi
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic $args > gpurun_out/r5_rgf_${f}_$r.json 2> gpurun_out/r5_rgf_${f}_$r.err || { echo "f=$f failed" >> $out; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r5_rgf_${f}_$r.json')); print('$r frac=$f', round(d['value'],1), round(d['ms_per_step'],3), round(d['kernels']['enc_mb_kernel']['avg_ms'],3), round(d['kernels']['dec_recon_kernel']['avg_ms'],3), d['parity']['vs_oracle'][-4:])" >> $out
  done
done
cat $out
