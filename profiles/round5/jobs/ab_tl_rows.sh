#!/bin/bash
# like ab_tl.sh, printing the frame span and the lives of rows 0 / 63 / 67 (encoder timeline, 32 streams, frames 3..5)
cd "$(dirname "$0")/../../.."
tag=$1; n=$2; shift 2
out=gpurun_out/abtr_${tag}.txt; : > $out
for r in $(seq 1 $n); do
  for lib in "$@"; do
    b=$(basename $lib .so)
    H264MI_LIB=$lib timeout -k 10 150 python -u tools/enc_timeline.py 1920 1080 1000000 32 6 > gpurun_out/abtr_${tag}_${b}_$r.txt 2>&1 || { echo "$b $r failed" >> $out; exit 1; }
    python3 - gpurun_out/abtr_${tag}_${b}_$r.txt "$r $b" >> $out <<'PY'
import re, sys
t = open(sys.argv[1]).read().split('\nframe ')
res = []
for blk in t:
    m = re.match(r'(?:frame )?([345]): span (\d+) us', blk)
    if not m: continue
    life = dict(re.findall(r' (\d+):(\d+)', blk.split('enc row life by row (us):')[1].split('\n')[0]))
    res.append(f"f{m.group(1)} span {m.group(2)} r0 {life['0']} r63 {life['63']} r67 {life['67']}")
print(sys.argv[2] + ': ' + ' | '.join(res))
PY
  done
done
cat $out
