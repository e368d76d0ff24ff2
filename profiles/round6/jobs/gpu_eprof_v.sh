#!/bin/bash
# round 6: enc_mb_kernel section profile (profiling build) at 128 streams after the granule-poll wait and Intra4x4
# table fixes: all rows, then MB row 40 alone (compare encprof_s128_h*.txt)
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6eprofv; mkdir -p $d
P=$(pwd)/openh264-wasm_amd/lib/ab/libh264mi_prof.so
H264MI_LIB=$P timeout -k 10 300 python -u tools/enc_prof.py 1920 1080 1000000 128 6 > $d/encprof_s128_v.txt 2>&1 || { tail -5 $d/encprof_s128_v.txt; exit 1; }
H264MI_ENC_PROF_ROW=40 H264MI_LIB=$P timeout -k 10 300 python -u tools/enc_prof.py 1920 1080 1000000 128 6 > $d/encprof_s128_v_row40.txt 2>&1 || { tail -5 $d/encprof_s128_v_row40.txt; exit 1; }
grep "frame 4:" $d/encprof_s128_v.txt $d/encprof_s128_v_row40.txt | cut -c1-400
