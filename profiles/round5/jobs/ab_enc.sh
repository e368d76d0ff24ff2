#!/bin/bash
# same-box A/B of two library builds: the encoder timeline at 32 streams (frame spans, row 0 / row 67 lives)
# and the driver's bench line without the CPU leg or PMC passes, alternating A B A B ...
# usage: tools/ab_enc.sh <tag> <libA> <libB> [rounds=2]
cd "$(dirname "$0")/../../.."
tag=$1; A=$2; B=$3; n=${4:-2}
out=gpurun_out/ab_${tag}.txt; : > $out
for r in $(seq 1 $n); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    H264MI_LIB=$lib timeout -k 10 150 python -u tools/enc_timeline.py 1920 1080 1000000 32 6 > gpurun_out/ab_${tag}_tl_$v$r.txt 2>&1 || { echo "timeline $v$r failed" >> $out; exit 1; }
    echo "$v$r timeline: $(grep '^frame [345]' gpurun_out/ab_${tag}_tl_$v$r.txt | sed -e 's/ | enc rows.*row 0 / row0 /' -e 's/).*//' | tr '\n' ' ')" >> $out
    H264MI_LIB=$lib timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/ab_${tag}_b_$v$r.json 2> gpurun_out/ab_${tag}_b_$v$r.err || { echo "bench $v$r failed" >> $out; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_${tag}_b_$v$r.json')); print('$v$r bench', round(d['value'],1), round(d['ms_per_step'],3), round(d['kernels']['enc_mb_kernel']['avg_ms'],3), round(d['kernels']['dec_recon_kernel']['avg_ms'],3), d['parity']['vs_oracle'][-4:])" >> $out
  done
done
cat $out
