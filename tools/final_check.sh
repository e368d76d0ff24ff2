#!/bin/bash
# exact final build: the driver's bench invocation + rocprofv3 kernel stats of the same command -> gpurun_out/final7/
set -o pipefail
out=gpurun_out/final7; root=$(pwd); mkdir -p $out
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_default.log 2>&1 || { echo "bench failed"; tail $out/bench_default.log; exit 1; }
grep '^{' $out/bench_default.log | tail -1 > $out/bench_default.json
echo "bench_default: $(grep -o '"value": [0-9.]*' $out/bench_default.json | head -1)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $root/$out/stats -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --no-traffic --steps 20 --warmup 5 > $root/$out/stats.log 2>&1
echo "profiled bench exit status $?"
cd $root && python3 tools/prof_summary.py $out/stats > $out/kernel_stats_summary.txt
python3 tools/drain.py $(ls $out/stats/*kernel_trace.csv | head -1) 20 > $out/timeline_20steps.txt
head -4 $out/kernel_stats_summary.txt; head -1 $out/timeline_20steps.txt; tail -1 $out/timeline_20steps.txt
