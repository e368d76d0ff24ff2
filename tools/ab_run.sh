set -o pipefail
mkdir -p gpurun_out/cap3
for S in 8 16 32; do
  for st in "20 5" "120 16"; do set -- $st
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-traffic --streams $S --steps $1 --warmup $2 > gpurun_out/cap3/b_${S}_$1.log 2>&1 || { echo FAIL $S; tail -5 gpurun_out/cap3/b_${S}_$1.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/cap3/b_${S}_$1.log') if l.startswith('{')][-1])
print('S $S steps $1', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['avg_ms'],3) for k,v in d['kernels'].items()})"
  done
done
