#!/bin/bash
# round 6: 16-stream self-consistency check, GPU suite and bench after pinning WelsMdFirstIntraMode (intra MBs in P slices)
cd "$GRAFT_REPO_ROOT"
d=gpurun_out/intra_p; mkdir -p $d
NF=25 timeout -k 10 500 python -u tools/debug/intra_p_diff.py 0 1 2 3 4 5 6 7 8 9 10 11 12 13 14 15 > $d/diff16.txt 2>&1 || { tail -5 $d/diff16.txt; exit 1; }
grep -c "bytes == oracle" $d/diff16.txt; grep -m3 "!=" $d/diff16.txt
grep -q "!=" $d/diff16.txt && exit 3
timeout -k 10 800 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > $d/gpu_tests.txt 2>&1
rc=$?; tail -3 $d/gpu_tests.txt; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $d/gpu_tests.txt | head; exit $rc; }
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $d/bench_default.json 2> $d/bench_default.err || { tail -5 $d/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$d/bench_default.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r.get('traffic_x_alg'), {k: v.get('avg_ms') for k, v in d['kernels'].items()}, str(d['parity'])[:300])"
