#!/bin/bash
# driver-invocation (20 steps) and 240-step bench at a few reserved parse-CU counts -> gpurun_out/pcus2/
set -o pipefail
out=gpurun_out/pcus2; mkdir -p $out
for n in "$@"; do for st in 20:5 240:16; do
  s=${st%%:*}; w=${st##*:}
  timeout -k 10 400 python3 bench.py --no-traffic --no-cpu-baseline --parse-cus $n --steps $s --warmup $w > $out/pcus_${n}_$s.log 2>&1 || { echo "parse-cus $n failed"; tail -5 $out/pcus_${n}_$s.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$out/pcus_${n}_$s.log').read().strip().splitlines()[-1]); print('parse_cus', $n, 'steps', $s, round(d['value'],1), 'frames/s', round(d['ms_per_step'],2), 'ms/step', 'parse', round(d['kernels']['dec_parse_kernel']['avg_ms'],1), 'enc', round(d['kernels']['enc_mb_kernel']['avg_ms'],2), 'recon', round(d['kernels']['dec_recon_kernel']['avg_ms'],2))"
done; done
