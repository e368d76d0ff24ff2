#!/bin/bash
# parse-stream count sweep (HIP streams the decoder rotates entropy decoding over) at the driver's invocation (no CPU leg / PMC), interleaved
cd "$(dirname "$0")/../../.."
out=gpurun_out/r5_pstreams.txt; : > $out
for r in 1 2; do
  for g in ${GS:-2 3 4}; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --parse-streams $g > gpurun_out/r5ps_${g}_$r.json 2> gpurun_out/r5ps_${g}_$r.err || { echo "g $g failed" >> $out; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r5ps_${g}_$r.json')); c=d['config']; print('$r parse_streams=$g', round(d['value'],1), round(d['ms_per_step'],3), c.get('parse_cus'), round(d['kernels']['enc_mb_kernel']['avg_ms'],3), round(d['kernels']['dec_recon_kernel']['avg_ms'],3), d['parity']['vs_oracle'][-4:])" >> $out
  done
done
cat $out
