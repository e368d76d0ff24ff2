#!/bin/bash
# capacity: streams per GPU (and parse lane) at the driver's 20 steps and at 240 steps -> gpurun_out/cap/
# usage: bash tools/sweep_cap.sh "16" "48 --parse-cus 48" ...
set -o pipefail
out=gpurun_out/cap; mkdir -p $out
for cfg in "$@"; do
  n=$(echo "s$cfg" | tr -d ' -'); s=${cfg%% *}; rest=${cfg#$s}
  for st in 20:5 240:16; do
    k=${st%%:*}; w=${st##*:}
    timeout -k 10 300 python3 bench.py --no-traffic --no-cpu-baseline --streams $s $rest --steps $k --warmup $w > $out/${n}_$k.log 2>&1 || { echo "$cfg failed"; tail -5 $out/${n}_$k.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/${n}_$k.log').read().strip().splitlines()[-1]); print('$cfg', 'steps', $k, round(d['value'],1), 'frames/s', round(d['ms_per_step'],2), 'ms/step', {k: round(v['avg_ms'],2) for k, v in d['kernels'].items()})"
  done
done
