#!/bin/bash
# a reconstruction variant library ($1): section profile vs the previous build, GPU tests on it, bench A/B
cd "$(dirname "$0")/../../.."
v=$1; tag=${TAG:-var}
./tools/ab_recon_prof.sh $tag openh264-wasm_amd/lib/libh264mi_pre.so $v > /dev/null || exit 1
grep "frame 4\|dec_recon\|==" gpurun_out/rprof_$tag.txt
H264MI_LIB=$v timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5l_tests.txt 2>&1 || { tail -30 gpurun_out/r5l_tests.txt; exit 1; }
tail -1 gpurun_out/r5l_tests.txt
./tools/ab_bench_libs.sh $tag 3 '' openh264-wasm_amd/lib/libh264mi_pre.so $v
