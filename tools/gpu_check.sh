#!/bin/bash
# one GPU iteration: selected gpu tests, a profiled default bench (exit status checked), the parse
# section profile and the C-ABI latency at 8 Mbps.   usage: tools/gpu_check.sh <outdir> "<pytest -k expr|ALL|NONE>"
set -o pipefail
out=gpurun_out/$1; mkdir -p $out; k="$2"; root=$(pwd)
if [ "$k" = "ALL" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest FAILED"; tail -40 $out/pytest.log; exit 1; }
elif [ "$k" != "NONE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$k" > $out/pytest.log 2>&1 || { echo "pytest FAILED"; tail -40 $out/pytest.log; exit 1; }
fi
tail -3 $out/pytest.log 2>/dev/null
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $root/$out/stats -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --no-traffic --steps 20 --warmup 5 > $root/$out/stats.log 2>&1
echo "profiled bench exit status $?"
grep -c "SIGSEGV\|Segmentation\|Aborted" $root/$out/stats.log || true
cd $root
python3 tools/prof_summary.py $out/stats > $out/kernel_stats_summary.txt && head -12 $out/kernel_stats_summary.txt
timeout -k 10 200 python3 tools/parse_prof.py 1920 1080 8000000 1 10 > $out/parse_prof_8m.txt 2>&1 && tail -4 $out/parse_prof_8m.txt
timeout -k 10 200 python3 tools/parse_prof.py 1920 1080 1000000 1 10 > $out/parse_prof_1m.txt 2>&1 && tail -2 $out/parse_prof_1m.txt
timeout -k 10 200 python3 tools/capi_latency.py 1920 1080 8000000 12 > $out/capi_8m.log 2>&1 && grep '^{' $out/capi_8m.log | tail -1 | cut -c1-400
