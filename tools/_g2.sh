export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests/test_gpu_syntax.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2/gpusyntax.log 2>&1; rc=$?
tail -40 gpurun_out/r2/gpusyntax.log
exit $rc
