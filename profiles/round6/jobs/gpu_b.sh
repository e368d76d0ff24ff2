#!/bin/bash
# round 6, job B: exact GOM rate control on the device vs the oracle (first run: the new tests only)
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6b; mkdir -p $d
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread -k "exact_gom or rc_state" > $d/gpu_tests.txt 2>&1
rc=$?; tail -12 $d/gpu_tests.txt; exit $rc
