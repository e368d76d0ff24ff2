export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/gputest.log 2>&1 || { tail -30 gpurun_out/r2/gputest.log; exit 1; }
tail -3 gpurun_out/r2/gputest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2/bench_20.json 2> gpurun_out/r2/bench_20.err || { tail -20 gpurun_out/r2/bench_20.err; exit 1; }
cat gpurun_out/r2/bench_20.json
