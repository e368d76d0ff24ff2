#!/bin/bash
# encoder parity tests, then a same-box timeline A/B (frame span, rows 0 / 63 / 67) against the last commit's build
cd "$(dirname "$0")/../../.."
tag=${1:-j}
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_configs.py tests/test_gpu_batch.py -q --timeout 120 --timeout-method thread > gpurun_out/r5${tag}_enc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5${tag}_enc_tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
L=openh264-wasm_amd/lib
./tools/ab_tl_rows.sh ${tag} 3 $L/libh264mi_base.so $L/libh264mi.so
