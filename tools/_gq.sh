# quick GPU check: gpu tests, default bench (no CPU leg), kernel-trace per-stream stats
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bq.log 2>&1 && grep -o '"value": [0-9.]*\|"avg_launch_ms": [0-9.]*\|parity_selfcheck[^,]*' gpurun_out/bq.log
rm -rf gpurun_out/pq
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pq -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $GRAFT_REPO_ROOT/gpurun_out/pq.log 2>&1
cd $GRAFT_REPO_ROOT && python tools/kstats_by_stream.py $(find gpurun_out/pq -name '*kernel_trace.csv' | head -1)
