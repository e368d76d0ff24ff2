#!/bin/bash
# I slices in the asm macroblock run: GPU tests, then the IDR / scene-change slice parse times of the
# previous library ($1) and this one, then a same-box bench A/B
cd "$(dirname "$0")/../../.."
base=${1:-openh264-wasm_amd/lib/libh264mi_base.so}
new=openh264-wasm_amd/lib/libh264mi.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5i_tests.txt 2>&1 || { tail -30 gpurun_out/r5i_tests.txt; exit 1; }
tail -2 gpurun_out/r5i_tests.txt
out=gpurun_out/r5i_parse.txt; : > $out
for lib in $base $new; do
  for br in 1000000 8000000; do
    echo "== $(basename $lib) br $br" >> $out
    H264MI_LIB=$lib timeout -k 10 180 python -u tools/parse_prof.py 1920 1080 $br 4 2 2>&1 | grep "^frame" | cut -c1-120 >> $out || exit 1
  done
done
cat $out
./tools/ab_bench_libs.sh iasm 2 '' $base $new
