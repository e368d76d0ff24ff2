#!/bin/bash
# round-5 GPU call: encoder parity tests, section profiles (all rows, rows 0 and 67), the driver's bench line
cd "$(dirname "$0")/../../.."
tag=${1:-f}
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_configs.py tests/test_gpu_batch.py -q --timeout 120 --timeout-method thread > gpurun_out/r5${tag}_enc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5${tag}_enc_tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
./tools/gpu_prof_rows.sh ${tag} || exit $?
timeout -k 10 200 python -u tools/enc_timeline.py 1920 1080 1000000 32 6 > gpurun_out/r5${tag}_timeline_s32.txt 2>&1 || exit $?
grep "frame [45]" -A3 gpurun_out/r5${tag}_timeline_s32.txt | cut -c1-250
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5${tag}_bench.json 2> gpurun_out/r5${tag}_bench.err
rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/r5${tag}_bench.json')); print(d['value'], d['ms_per_step'], d['kernels']['enc_mb_kernel'], d['roofline'].get('traffic_x_alg'), d['parity']['vs_oracle'][-60:])"; exit $rc
