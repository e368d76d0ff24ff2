#!/bin/bash
# same-box A/B of library builds at the driver's invocation (no CPU leg / PMC), interleaved rounds
# usage: tools/ab_bench_libs.sh <tag> <rounds> "<extra bench args>" lib...
cd "$(dirname "$0")/../../.."
tag=$1; n=$2; extra=$3; shift 3
out=gpurun_out/abb_${tag}.txt; : > $out
for r in $(seq 1 $n); do
  for lib in "$@"; do
    b=$(basename $lib .so)
    H264MI_LIB=$lib timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic $extra > gpurun_out/abb_${tag}_${b}_$r.json 2> gpurun_out/abb_${tag}_${b}_$r.err || { echo "$b $r failed" >> $out; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/abb_${tag}_${b}_$r.json')); print('$r $b', round(d['value'],1), round(d['ms_per_step'],3), round(d['kernels']['enc_mb_kernel']['avg_ms'],3), round(d['kernels']['dec_recon_kernel']['avg_ms'],3), d['parity']['vs_oracle'][-4:])" >> $out
  done
done
cat $out
