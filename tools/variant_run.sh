#!/bin/bash
# A/B libh264mi variants (openh264-wasm_amd/lib/variants/<name>.so via H264MI_LIB) on the driver's
# short bench and on config 4.  usage: tools/variant_run.sh <outdir> <name>... [-- extra bench args]
set -o pipefail
out=gpurun_out/$1; shift; mkdir -p $out
names=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do names+=("$1"); shift; done; [ "$1" = "--" ] && shift
for n in "${names[@]}"; do
  for cfg in ${CFGS:-0 4}; do
    H264MI_LIB=$PWD/openh264-wasm_amd/lib/variants/$n.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --config $cfg "$@" > $out/$n.c$cfg.log 2>&1 || { echo "$n c$cfg FAILED"; tail -5 $out/$n.c$cfg.log; exit 1; }
    python3 - $out/$n.c$cfg.log $n $cfg <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'c'+sys.argv[3], round(d['value'] or 0,1), 'ms/step', round(d['ms_per_step'],3), {k:round(v['avg_ms'],3) for k,v in d['kernels'].items()}, d['parity']['selfcheck'][-4:])
PY
  done
done
