#!/bin/bash
# recon chroma (both planes per lane): GPU tests, then a same-box bench A/B against the previous build
cd "$(dirname "$0")/../../.."
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5k_tests.txt 2>&1 || { tail -30 gpurun_out/r5k_tests.txt; exit 1; }
tail -1 gpurun_out/r5k_tests.txt
./tools/ab_bench_libs.sh ${TAG:-rchroma} 3 '' openh264-wasm_amd/lib/libh264mi_pre.so openh264-wasm_amd/lib/libh264mi.so
