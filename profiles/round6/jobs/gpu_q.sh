#!/bin/bash
# round 6, job Q: parse-side record resolution -- the decoder GPU tests, then the pipeline A/B (H264MI_DEC_PRERES 1 / 0)
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6q; mkdir -p $d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -k "dec or multislice or syntax or batch or ring or napi or configs" > $d/gpu_tests.txt 2>&1
rc=$?; tail -5 $d/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for v in 1 0; do
  H264MI_DEC_PRERES=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-traffic --no-cpu-baseline --clip 30 > $d/b_$v_$rep.json 2> $d/b.err || { tail -3 $d/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$d/b_$v_$rep.json')); k=d['kernels']; print('preres $v rep $rep', round(d['value']), round(d['ms_per_step'],2), {a: round(b['avg_ms'],2) for a, b in k.items() if 'avg_ms' in b}, d['parity']['selfcheck'][-5:])"
done; done
