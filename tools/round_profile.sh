#!/bin/bash
# Round profile set (run on the GPU box from the repo root): kernel-trace stats of the default bench,
# then the FETCH_SIZE and WRITE_SIZE PMC passes (separate passes, no trace domains) -> profiles/<round>/
set -e
round=${1:-round1}; shift || true
root=$(pwd)
out=$root/gpurun_out/$round
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline "$@" > $out/stats.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --steps 32 --warmup 16 "$@" > $out/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --steps 32 --warmup 16 "$@" > $out/write.log 2>&1
cd $root
python3 tools/pmc_enc.py $out/fetch $out/write $out/pmc_enc_mb.json 1920 1080 8
python3 tools/prof_summary.py $out/stats > $out/kernel_stats_summary.txt
cat $out/kernel_stats_summary.txt
