#!/bin/bash
# round 6, job F: the full bench (CPU leg, parity, traffic) at 128 streams per GPU; its wall time
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6f; mkdir -p $d
s=$(date +%s)
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --streams 128 --parse-cus 32 > $d/bench_s128.json 2> $d/bench_s128.err || { tail -5 $d/bench_s128.err; exit 1; }
echo "wall $(( $(date +%s) - s )) s"
python3 -c "import json; d=json.load(open('$d/bench_s128.json')); r=d['roofline']; c=d['cpu_baseline']; print(d['value'], d['ms_per_step'], r['frac'], r['traffic'], c['value'], c.get('sample','')[:200], str(d['parity'])[:400])"
