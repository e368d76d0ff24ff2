#!/bin/bash
# rocprofv3 kernel trace of one bench run -> gpurun_out/<name>/ + timeline of the last K steps
# usage: tools/trace_bench.sh <name> <K> [bench args...]
set -o pipefail
name=$1; K=$2; shift 2
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/$name -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --no-traffic "$@" > $root/gpurun_out/$name.log 2>&1 || { echo "trace run failed"; tail -5 $root/gpurun_out/$name.log; exit 1; }
cd $root && grep '^{' gpurun_out/$name.log | tail -1 | cut -c1-200
python3 tools/drain.py gpurun_out/$name/run_kernel_trace.csv $K > gpurun_out/$name/timeline.txt && head -60 gpurun_out/$name/timeline.txt
