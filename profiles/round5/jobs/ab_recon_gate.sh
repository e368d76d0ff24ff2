#!/bin/bash
# the recon-gate test, then a same-box A/B of bench --recon-gate 0 / 1 at the driver's invocation (no CPU leg / PMC)
cd "$(dirname "$0")/../../.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -q -k "recon_gate or 1080p-s4 or pipelined" --timeout 120 --timeout-method thread > gpurun_out/r5_rg_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_rg_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/r5_recon_gate.txt; : > $out
for r in 1 2; do
  for g in 0 1; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --recon-gate $g > gpurun_out/r5_rg_${g}_$r.json 2> gpurun_out/r5_rg_${g}_$r.err || { echo "gate=$g failed" >> $out; tail -3 gpurun_out/r5_rg_${g}_$r.err >> $out; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r5_rg_${g}_$r.json')); print('$r gate=$g', round(d['value'],1), round(d['ms_per_step'],3), d['kernels']['enc_mb_kernel'], d['kernels']['dec_recon_kernel'], d['parity']['vs_oracle'][-4:], d['parity']['selfcheck'][-20:])" >> $out
  done
done
cat $out
