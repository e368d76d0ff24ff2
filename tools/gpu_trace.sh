#!/bin/bash
# rocprofv3 kernel trace + stats of the driver's bench invocation (no CPU leg, no PMC) -> gpurun_out/<name>/
cd "$(dirname "$0")/.."
name=${1:-r5trace}; shift
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/$name -o run --output-format csv -- python3 $root/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic "$@" > $root/gpurun_out/$name.json 2> $root/gpurun_out/$name.err || exit $?
cd $root
f=$(find gpurun_out/$name -name '*kernel_trace.csv' | head -1)
python3 tools/drain.py $f 20 > gpurun_out/${name}_drain.txt
python3 tools/timeline.py $f 20 > gpurun_out/${name}_timeline.txt
head -3 gpurun_out/${name}_drain.txt; tail -12 gpurun_out/${name}_drain.txt
