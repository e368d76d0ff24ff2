#!/bin/bash
# round 6, job G: the driver's bench invocation at the new default (128 streams per GPU) with the parse SQ pass,
# then rocprofv3 --kernel-trace --stats of the same bench (no CPU leg / PMC) for the kernel averages
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6g; mkdir -p $d
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $d/bench_default.json 2> $d/bench_default.err || { tail -5 $d/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$d/bench_default.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['traffic_x_alg'], d['cpu_baseline']['value'], json.dumps(d['kernels']))"
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $root/$d/prof -o run --output-format csv -- python3 $root/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $root/$d/bench_prof.json 2> $root/$d/bench_prof.err || { tail -5 $root/$d/bench_prof.err; exit 1; }
cd $root && f=$(find $d/prof -name '*kernel_stats.csv' | head -1) && head -12 "$f"
