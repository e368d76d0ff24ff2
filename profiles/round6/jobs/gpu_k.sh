#!/bin/bash
# round 6, job K: the new GPU tests (grouped tickets) + the exact-GOM tests
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6k; mkdir -p $d
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 180 --timeout-method thread -k "grouped or exact_gom" > $d/gpu_tests.txt 2>&1
rc=$?; tail -8 $d/gpu_tests.txt; exit $rc
