#!/bin/bash
# round-5 GPU call: encoder parity tests, row profiles, then a same-box A/B against the session's base build
cd "$(dirname "$0")/../../.."
tag=${1:-g}
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_configs.py tests/test_gpu_batch.py -q --timeout 120 --timeout-method thread > gpurun_out/r5${tag}_enc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5${tag}_enc_tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
./tools/gpu_prof_rows.sh ${tag} || exit $?
./tools/ab_enc.sh ${tag} openh264-wasm_amd/lib/libh264mi_base.so openh264-wasm_amd/lib/libh264mi.so 2
