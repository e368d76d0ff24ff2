#!/bin/bash
# round-5 final evidence, part A: the whole GPU test suite, smoke(), the driver's bench invocation (CPU leg + PMC passes)
cd "$(dirname "$0")/../../.."
d=gpurun_out/final5; mkdir -p $d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $d/gpu_tests.txt 2>&1
rc=$?; tail -3 $d/gpu_tests.txt; [ $rc -ne 0 ] && { echo "tests rc=$rc"; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $d/smoke.txt 2>&1 || { tail -5 $d/smoke.txt; exit 1; }
tail -1 $d/smoke.txt
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $d/bench_default.json 2> $d/bench_default.err || { tail -5 $d/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$d/bench_default.json')); r=d['roofline']; c=d['cpu_baseline']; print(d['value'], d['ms_per_step'], r['frac'], r['traffic'], r.get('traffic_x_alg'), c['value'], d['parity']['vs_oracle'][-60:])"
