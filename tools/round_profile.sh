#!/bin/bash
# Round evidence set (GPU box, repo root) -> gpurun_out/<round>/:
#   bench_default.json/.log  default bench.py run (with the CPU baseline leg)
#   stats/                   rocprofv3 --kernel-trace --stats of the default bench (kernel_stats_summary.txt,
#                            timeline.txt = overlap of the codec kernels in the last 400 ms)
#   fetch/, write/           separate --pmc FETCH_SIZE / WRITE_SIZE passes (no trace domains)
#   pmc_enc_mb.json          HBM bytes per enc_mb_kernel launch (tools/pmc_enc.py; gfx950 x2 FETCH correction)
#   pmc_fetch_write.txt      the same per kernel for every codec kernel
set -e
round=${1:-round1}; shift || true
root=$(pwd)
out=$root/gpurun_out/$round
mkdir -p $out
timeout -k 10 600 python3 bench.py "$@" > $out/bench_default.log 2>&1
grep '^{' $out/bench_default.log | tail -1 > $out/bench_default.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline "$@" > $out/stats.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --steps 32 --warmup 16 "$@" > $out/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --steps 32 --warmup 16 "$@" > $out/write.log 2>&1
cd $root
python3 tools/pmc_enc.py $out/fetch $out/write $out/pmc_enc_mb.json 1920 1080 8
python3 tools/pmc_enc.py $out/fetch $out/write /dev/null 1920 1080 8 --all > $out/pmc_fetch_write.txt
python3 tools/prof_summary.py $out/stats > $out/kernel_stats_summary.txt
python3 tools/timeline.py $(ls $out/stats/*/run_kernel_trace.csv $out/stats/run_kernel_trace.csv 2>/dev/null | head -1) 400 > $out/timeline.txt
cat $out/kernel_stats_summary.txt $out/timeline.txt $out/pmc_fetch_write.txt
