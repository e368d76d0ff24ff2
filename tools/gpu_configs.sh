#!/bin/bash
# bench.py per BASELINE.json config + the driver's short invocation at several decode-group sizes
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
for g in 1 2 8; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --group $g > $out/g$g.log 2>&1 || exit 1
  echo "group $g: $(grep -o '"value": [0-9.]*' $out/g$g.log)"
done
for c in 2 3 4 5; do
  timeout -k 10 300 python -u bench.py --config $c > $out/config$c.log 2>&1 || exit 1
  grep '^{' $out/config$c.log | tail -1 > $out/config$c.json
  echo "config $c: $(grep -o '"value": [0-9.]*' $out/config$c.json) $(grep -o '"ms_per_step": [0-9.]*' $out/config$c.json)"
done
