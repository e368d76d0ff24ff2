#!/bin/bash
# same-box comparison of several library builds by the encoder timeline alone (32 x 1080p, frames 3..5: span and
# row 0's life), interleaved over rounds.   usage: tools/ab_tl.sh <tag> <rounds> lib...
cd "$(dirname "$0")/../../.."
tag=$1; n=$2; shift 2
out=gpurun_out/abtl_${tag}.txt; : > $out
for r in $(seq 1 $n); do
  for lib in "$@"; do
    b=$(basename $lib .so)
    H264MI_LIB=$lib timeout -k 10 150 python -u tools/enc_timeline.py 1920 1080 1000000 32 6 > gpurun_out/abtl_${tag}_${b}_$r.txt 2>&1 || { echo "$b $r failed" >> $out; exit 1; }
    echo "$r $b: $(grep '^frame [345]' gpurun_out/abtl_${tag}_${b}_$r.txt | sed -e 's/ | enc rows.*row 0 / row0 /' -e 's/).*//' -e 's/frame //' -e 's/span //' | tr '\n' ' ')" >> $out
  done
done
cat $out
