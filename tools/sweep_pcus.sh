#!/bin/bash
# default bench at a few reserved parse-CU counts -> gpurun_out/pcus_<n>.log (last line: the JSON)
set -o pipefail
for n in "$@"; do
  timeout -k 10 400 python3 bench.py --no-traffic --no-cpu-baseline --parse-cus $n > gpurun_out/pcus_$n.log 2>&1 || { echo "parse-cus $n failed"; tail -5 gpurun_out/pcus_$n.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/pcus_$n.log').read().strip().splitlines()[-1]); print('parse_cus', $n, round(d['value'],1), 'frames/s', round(d['ms_per_step'],2), 'ms/step', 'parse', round(d['kernels']['dec_parse_kernel']['avg_ms'],1), 'enc', round(d['kernels']['enc_mb_kernel']['avg_ms'],2))"
done
