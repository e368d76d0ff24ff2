#!/bin/bash
# round 6: GPU suite, then the bench at 128 / 192 / 256 streams per GPU with the pinned P-slice decisions
cd "$GRAFT_REPO_ROOT"
d=gpurun_out/sweep_judge; mkdir -p $d
timeout -k 10 800 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $d/gpu_tests.txt 2>&1
rc=$?; tail -2 $d/gpu_tests.txt; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $d/gpu_tests.txt | head; exit $rc; }
for s in 128 192 256; do
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --streams $s --no-cpu-baseline --no-traffic > $d/bench_s$s.json 2> $d/bench_s$s.err || { tail -5 $d/bench_s$s.err; exit 1; }
  python3 -c "import json; d=json.load(open('$d/bench_s$s.json')); print($s, d['value'], d['ms_per_step'], {k: v.get('avg_ms') for k, v in d['kernels'].items()}, str(d['parity']['vs_oracle'])[-40:])"
done
