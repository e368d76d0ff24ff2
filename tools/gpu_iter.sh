#!/bin/bash
# iteration loop on the GPU box: selected gpu tests, the driver's bench line, optional extra bench args
# usage: tools/gpu_iter.sh <outdir> "<pytest -k expr or ALL or NONE>" [extra bench.py args...]
set -o pipefail
out=gpurun_out/$1; mkdir -p $out; k="$2"; shift 2
if [ "$k" = "ALL" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest FAILED"; tail -30 $out/pytest.log; exit 1; }
  tail -2 $out/pytest.log
elif [ "$k" != "NONE" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$k" > $out/pytest.log 2>&1 || { echo "pytest FAILED"; tail -30 $out/pytest.log; exit 1; }
  tail -2 $out/pytest.log
fi
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 "$@" > $out/b20.log 2>&1 || { echo "bench FAILED"; tail -20 $out/b20.log; exit 1; }
python3 - $out/b20.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('b20', round(d['value'] or 0,1), 'ms/step', round(d['ms_per_step'],3), {k:round(v['avg_ms'],3) for k,v in d['kernels'].items()}, d['parity']['selfcheck'][-4:])
PY
timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > $out/b240.log 2>&1 || { echo "bench240 FAILED"; tail -20 $out/b240.log; exit 1; }
python3 - $out/b240.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('b240', round(d['value'] or 0,1), 'ms/step', round(d['ms_per_step'],3), {k:round(v['avg_ms'],3) for k,v in d['kernels'].items()})
PY
