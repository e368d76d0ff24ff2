#!/bin/bash
# Round-3 evidence on one GPU box -> gpurun_out/<name>/ (copied into profiles/round3/ afterwards).
# part A: bench lines (each with its CPU baseline and in-run PMC traffic)
# part B: C-ABI latency, rocprofv3 kernel stats + timeline, parse / encoder section profiles, SQ states
set -o pipefail
name=${1:-round3}; part=${2:-A}; out=gpurun_out/$name; root=$(pwd); mkdir -p $out
j() { grep '^{' $1 | tail -1; }
b() { tag=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $out/$tag.log 2>&1 || { echo "$tag failed"; tail $out/$tag.log; exit 1; }
      j $out/$tag.log > $out/$tag.json; echo "$tag: $(grep -o '"value": [0-9.]*' $out/$tag.json | head -1) $(grep -o '"ms_per_step": [0-9.]*' $out/$tag.json)"; }
if [ "$part" = A ]; then
  b bench_default --gpus 1 --steps 20 --warmup 5
  b bench_240 --steps 240 --warmup 16 --no-cpu-baseline --no-traffic
  b bench_8m --steps 20 --warmup 5 --bitrate 8000000
  b bench_s8 --steps 20 --warmup 5 --streams 8 --no-cpu-baseline --no-traffic
fi
if [ "$part" = C ]; then
  for c in 2 3 4 5; do b config$c --config $c; done
  b config2_8m --config 2 --bitrate 8000000 --no-traffic
fi
if [ "$part" = B ]; then
  timeout -k 10 200 python3 tools/capi_latency.py 1920 1080 1000000 12 > $out/capi_1m.log 2>&1 && j $out/capi_1m.log > $out/capi_1m.json
  timeout -k 10 200 python3 tools/capi_latency.py 1920 1080 8000000 12 > $out/capi_8m.log 2>&1 && j $out/capi_8m.log > $out/capi_8m.json
  timeout -k 10 300 python3 tools/parse_mix.py > $out/parse_mix.txt 2>&1
  timeout -k 10 200 python3 tools/parse_prof.py 1920 1080 8000000 1 10 > $out/parse_prof_8m.txt 2>&1
  timeout -k 10 200 python3 tools/parse_prof.py 1920 1080 1000000 1 10 > $out/parse_prof_1m.txt 2>&1
  timeout -k 10 300 python3 tools/enc_prof.py 1920 1080 1000000 8 6 > $out/enc_sections.txt 2>&1
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $root/$out/stats -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --no-traffic --steps 20 --warmup 5 > $root/$out/stats.log 2>&1
  echo "profiled bench exit status $?"; grep -c "SIGSEGV\|Segmentation" $root/$out/stats.log
  cd $root && python3 tools/prof_summary.py $out/stats > $out/kernel_stats_summary.txt
  python3 tools/drain.py $(ls $out/stats/*kernel_trace.csv | head -1) 20 > $out/timeline_20steps.txt
  bash tools/pmc_sq.sh $name/sq > $out/sq_states.txt 2>&1 || echo "sq pass failed"
  head -5 $out/kernel_stats_summary.txt
fi
