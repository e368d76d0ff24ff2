export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests/test_gpu_encoder.py tests/test_content_extremes.py tests/test_gpu_batch.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2/gpu3.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/r2/gpu3.log | head -60
exit $rc
