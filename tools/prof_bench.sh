#!/bin/bash
# usage: tools/prof_bench.sh <outdir-name> [bench args...]  -- rocprofv3 kernel-trace stats of bench.py
set -e
name=$1; shift
root=$GRAFT_REPO_ROOT; [ -z "$root" ] && root=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/$name -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline "$@" > $root/gpurun_out/$name.log 2>&1
cd $root && python3 tools/prof_summary.py gpurun_out/$name
