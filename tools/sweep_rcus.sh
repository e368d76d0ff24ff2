#!/bin/bash
# default bench (240 steps) with the reconstruction on its own CU lane of n CUs -> gpurun_out/rcus_<n>.log
set -o pipefail
for n in "$@"; do
  timeout -k 10 400 python3 bench.py --no-traffic --no-cpu-baseline --recon-cus $n > gpurun_out/rcus_$n.log 2>&1 || { echo "recon-cus $n failed"; tail -5 gpurun_out/rcus_$n.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/rcus_$n.log').read().strip().splitlines()[-1]); k=d['kernels']; print('recon_cus', $n, round(d['value'],1), 'frames/s', round(d['ms_per_step'],2), 'ms/step', 'enc', round(k['enc_mb_kernel']['avg_ms'],2), 'recon', round(k['dec_recon_kernel']['avg_ms'],2), 'parse', round(k['dec_parse_kernel']['avg_ms'],1))"
done
