#!/bin/bash
# SQ wave-state counters of the default bench (one PMC pass, no trace domains) -> gpurun_out/<name>/
# usage: tools/pmc_sq.sh <name> [bench args...]
set -e
name=$1; shift
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM \
  -d $root/gpurun_out/$name -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --no-traffic --steps 16 --warmup 8 "$@" > $root/gpurun_out/$name.log 2>&1
cd $root && python3 tools/pmc_sq_summary.py gpurun_out/$name
