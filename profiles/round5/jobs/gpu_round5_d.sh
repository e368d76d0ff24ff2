#!/bin/bash
# round-5 GPU call: encoder timeline at 8 and 16 streams (contention), bench at 32 / 48 / 64 streams per GPU
cd "$(dirname "$0")/../../.."
out=gpurun_out/r5_capacity.txt; : > $out
for S in 8 16; do
  echo "== timeline S=$S" >> $out
  timeout -k 10 120 python -u tools/enc_timeline.py 1920 1080 1000000 $S 6 2>&1 | grep -A3 "^frame [45]" >> $out || exit $?
done
for S in 32 48 64; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --streams $S --no-cpu-baseline --no-traffic > gpurun_out/r5_bench_s$S.json 2> gpurun_out/r5_bench_s$S.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r5_bench_s$S.json')); print('S=$S', round(d['value'],1), round(d['ms_per_step'],3), d['kernels']['enc_mb_kernel'], d['kernels']['dec_recon_kernel'])" >> $out
done
cat $out | cut -c1-250
