#!/bin/bash
# encoder launch scheduling sweep (encoder alone, 32 x 1080p, frames 0..5): wave priority of the encoder rows
# (H264MI_ENC_PRIO) x deblocking ticket lag (H264MI_DBK_LAG); prints each run's frame spans.
# CFGS="prio:dlag ..." overrides the list; TAG names the output file
cd "$(dirname "$0")/.."
out=gpurun_out/r5_sched${TAG}.txt; : > $out
for cfg in ${CFGS:-0:0 2:0 3:0 2:8 2:16 2:32 0:16}; do
  p=${cfg%%:*}; d=${cfg##*:}
  echo "== prio $p dlag $d" >> $out
  H264MI_ENC_PRIO=$p H264MI_DBK_LAG=$d timeout -k 10 120 python -u tools/enc_timeline.py 1920 1080 1000000 32 6 2>&1 | grep "^frame" >> $out || exit $?
done
grep -v "^frame [0-2]" $out | cut -c1-60
