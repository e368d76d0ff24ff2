#!/bin/bash
# One GPU call: gpu tests, the driver's bench invocation, a rocprofv3 kernel-trace summary of it.
# usage: tools/gpu_round.sh <outdir> [skip-tests]
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
root=$(pwd)
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $out/pytest.log; exit 1; }
  tail -3 $out/pytest.log
fi
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_20_5.log 2>&1 || { echo "bench failed"; tail -20 $out/bench_20_5.log; exit 1; }
grep '^{' $out/bench_20_5.log | tail -1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $root/$out/stats -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --steps 240 --warmup 16 > $root/$out/stats.log 2>&1 || { echo "rocprof failed"; tail -20 $root/$out/stats.log; exit 1; }
cd $root && python3 tools/prof_summary.py $out/stats > $out/kernel_stats_summary.txt; head -30 $out/kernel_stats_summary.txt
