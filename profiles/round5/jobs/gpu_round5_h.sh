#!/bin/bash
# encoder parity tests, detail section profiles, same-box timeline A/B against the last commit's build
cd "$(dirname "$0")/../../.."
tag=${1:-h}
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_configs.py tests/test_gpu_batch.py -q --timeout 120 --timeout-method thread > gpurun_out/r5${tag}_enc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5${tag}_enc_tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
H264MI_LIB=openh264-wasm_amd/lib/libh264mi_detail.so ./tools/gpu_prof_rows.sh ${tag} > /dev/null || exit $?
grep -h -A2 "^frame 4: [0-9]" gpurun_out/r5${tag}_encprof_s32_row0.txt | cut -c1-300
L=openh264-wasm_amd/lib
./tools/ab_tl.sh ${tag} 3 $L/libh264mi_base.so $L/libh264mi.so
