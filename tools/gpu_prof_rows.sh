#!/bin/bash
# encoder section profile at 32 streams: every row, then MB rows 0 and 67 alone -> gpurun_out/r5<tag>_encprof_s32*.txt
cd "$(dirname "$0")/.."
tag=${1:-p}
timeout -k 10 200 python -u tools/enc_prof.py 1920 1080 1000000 32 6 > gpurun_out/r5${tag}_encprof_s32.txt 2>&1 || exit $?
for r in 0 67; do
  H264MI_ENC_PROF_ROW=$r timeout -k 10 200 python -u tools/enc_prof.py 1920 1080 1000000 32 6 > gpurun_out/r5${tag}_encprof_s32_row$r.txt 2>&1 || exit $?
done
grep -h -A3 "^frame 4: [0-9]" gpurun_out/r5${tag}_encprof_s32*.txt | cut -c1-400
