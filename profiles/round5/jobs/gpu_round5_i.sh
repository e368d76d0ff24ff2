#!/bin/bash
# the whole GPU suite, then a same-box A/B (encoder timeline + the driver's bench line) against the last commit's build
cd "$(dirname "$0")/../../.."
tag=${1:-i}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5${tag}_gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5${tag}_gpu_tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
./tools/ab_enc.sh ${tag} openh264-wasm_amd/lib/libh264mi_base.so openh264-wasm_amd/lib/libh264mi.so 2
