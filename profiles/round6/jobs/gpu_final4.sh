#!/bin/bash
# round 6, final (after the granule-poll wait and Intra4x4 table fixes): the whole GPU suite, smoke(), the driver's bench invocation, and rocprofv3 --kernel-trace --stats of the bench
cd "$(dirname "$0")/../../.." && mkdir -p gpurun_out/eprof
d=gpurun_out/r6final4; mkdir -p $d
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $d/gpu_tests.txt 2>&1
rc=$?; tail -3 $d/gpu_tests.txt; [ $rc -ne 0 ] && { echo "tests rc=$rc"; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $d/smoke.txt 2>&1 || { tail -5 $d/smoke.txt; exit 1; }
tail -1 $d/smoke.txt
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $d/bench_default.json 2> $d/bench_default.err || { tail -5 $d/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$d/bench_default.json')); r=d['roofline']; k=d['kernels']['dec_parse_kernel']; print(d['value'], d['ms_per_step'], r['frac'], r['traffic_x_alg'], d['cpu_baseline']['value'], k['busy_share_of_timed_wall'], k['sq']['issue_frac'] if k.get('sq') else None)"
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $root/$d/prof -o run --output-format csv -- python3 $root/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $root/$d/bench_prof.json 2> $root/$d/bench_prof.err || { tail -5 $root/$d/bench_prof.err; exit 1; }
cd $root && head -6 $d/prof/run_kernel_stats.csv | cut -c1-160
timeout -k 10 600 python -u bench.py --gpus 1 > $d/bench_240.json 2> $d/bench_240.err || { tail -5 $d/bench_240.err; exit 1; }
python3 -c "import json; d=json.load(open('$d/bench_240.json')); print('240 steps', d['value'], d['ms_per_step'], str(d['parity']['vs_oracle'])[:160])"

exit 0
