#!/bin/bash
# round 6, job R: enc_mb_kernel section profile (profiling build) at 32 and 128 streams, encoder alone
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6r; mkdir -p $d
for S in 32 128; do
  H264MI_LIB=$(pwd)/openh264-wasm_amd/lib/ab/libh264mi_prof.so timeout -k 10 300 python -u tools/enc_prof.py 1920 1080 1000000 $S 6 > $d/encprof_s$S.txt 2>&1 || { tail -5 $d/encprof_s$S.txt; exit 1; }
  tail -25 $d/encprof_s$S.txt
done
