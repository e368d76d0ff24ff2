#!/bin/bash
# round 6, job E: the metric pipeline at higher stream counts (row plan / exact GOM, parse CU reservation),
# no CPU leg or traffic passes (throughput sweep only; parity is checked by the full runs)
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6e; mkdir -p $d
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-traffic --no-cpu-baseline --clip 30 "$@" > $d/$n.json 2> $d/$n.err || { tail -5 $d/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('$d/$n.json')); k=d['kernels']; print('$n', round(d['value']), round(d['ms_per_step'],1), {a: round(b['avg_ms'],1) for a, b in k.items()}, d['config']['parse_cus'])"
}
if [ -n "$SWEEP" ]; then eval "$SWEEP"; exit $?; fi
run s64_row --streams 64 && run s64_exact --streams 64 --gom-exact && \
run s128_row --streams 128 && run s128_row_p40 --streams 128 --parse-cus 40 && run s128_exact --streams 128 --gom-exact && run s128_exact_p40 --streams 128 --gom-exact --parse-cus 40 && \
run s256_row_p40 --streams 256 --parse-cus 40 && run s256_row_p80 --streams 256 --parse-cus 80 && run s256_exact_p40 --streams 256 --gom-exact --parse-cus 40 && run s256_exact_p80 --streams 256 --gom-exact --parse-cus 80
