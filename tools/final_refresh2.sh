#!/bin/bash
# final refresh after the loop-filter changes -> gpurun_out/final3/
set -o pipefail
out=gpurun_out/final3; root=$(pwd); mkdir -p $out
j() { grep '^{' $1 | tail -1; }
b() { tag=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $out/$tag.log 2>&1 || { echo "$tag failed"; tail $out/$tag.log; exit 1; }
      j $out/$tag.log > $out/$tag.json; echo "$tag: $(grep -o '"value": [0-9.]*' $out/$tag.json | head -1) $(grep -o '"ms_per_step": [0-9.]*' $out/$tag.json)"; }
b bench_default --gpus 1 --steps 20 --warmup 5
b bench_240 --steps 240 --warmup 16 --no-cpu-baseline --no-traffic
b bench_8m --steps 20 --warmup 5 --bitrate 8000000
b bench_s8 --steps 20 --warmup 5 --streams 8 --no-cpu-baseline --no-traffic
for c in 2 3 4 5; do b config$c --config $c; done
b config2_8m --config 2 --bitrate 8000000 --no-traffic
timeout -k 10 200 python3 tools/capi_latency.py 1920 1080 8000000 12 > $out/capi_8m.log 2>&1 && j $out/capi_8m.log > $out/capi_8m.json
timeout -k 10 200 python3 tools/capi_latency.py 1920 1080 1000000 12 > $out/capi_1m.log 2>&1 && j $out/capi_1m.log > $out/capi_1m.json
timeout -k 10 300 python3 tools/enc_prof.py 1920 1080 1000000 8 6 > $out/enc_sections.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $root/$out/stats -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --no-traffic --steps 20 --warmup 5 > $root/$out/stats.log 2>&1
echo "profiled bench exit status $?"
cd $root && python3 tools/prof_summary.py $out/stats > $out/kernel_stats_summary.txt
python3 tools/drain.py $(ls $out/stats/*kernel_trace.csv | head -1) 20 > $out/timeline_20steps.txt
head -4 $out/kernel_stats_summary.txt; head -1 $out/timeline_20steps.txt; tail -3 $out/timeline_20steps.txt
