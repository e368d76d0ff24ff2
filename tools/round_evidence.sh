#!/bin/bash
# Round evidence on one GPU box -> gpurun_out/<name>/ (copied into profiles/<name>/ afterwards):
#   bench_default.json/.log   the driver's invocation (python3 bench.py --gpus 1 --steps 20 --warmup 5)
#   bench_240.json            the same workload at 240 steps (steady state)
#   config{2,3,4,5}.json      BASELINE.json configs, one bench line each (CPU baseline + in-run traffic)
#   capi_{1m,8m}.json         single-call C-ABI latency at 1080p (tools/capi_latency.py)
#   stats/ + kernel_stats_summary.txt   rocprofv3 --kernel-trace --stats of the default bench
set -o pipefail
name=${1:-round2}; out=gpurun_out/$name; root=$(pwd); mkdir -p $out
j() { grep '^{' $1 | tail -1; }
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_default.log 2>&1 || { echo "default bench failed"; tail $out/bench_default.log; exit 1; }
j $out/bench_default.log > $out/bench_default.json
timeout -k 10 400 python3 bench.py --steps 240 --warmup 16 > $out/bench_240.log 2>&1 || { echo "240 bench failed"; exit 1; }
j $out/bench_240.log > $out/bench_240.json
for c in 2 3 4 5; do
  timeout -k 10 400 python3 bench.py --config $c > $out/config$c.log 2>&1 || { echo "config $c failed"; tail $out/config$c.log; exit 1; }
  j $out/config$c.log > $out/config$c.json
done
timeout -k 10 200 python3 tools/capi_latency.py 1920 1080 1000000 12 > $out/capi_1m.log 2>&1 && j $out/capi_1m.log > $out/capi_1m.json
timeout -k 10 200 python3 tools/capi_latency.py 1920 1080 8000000 12 > $out/capi_8m.log 2>&1 && j $out/capi_8m.log > $out/capi_8m.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $root/$out/stats -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --no-traffic --steps 20 --warmup 5 > $root/$out/stats.log 2>&1
cd $root && python3 tools/prof_summary.py $out/stats > $out/kernel_stats_summary.txt
python3 tools/drain.py $(ls $out/stats/*kernel_trace.csv | head -1) 20 > $out/timeline_20steps.txt
for f in $out/*.json; do echo "$f: $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
