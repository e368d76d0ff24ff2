# GPU: full -m gpu suite, then the parse section profile (1080p, 1 Mbps, P frames)
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/gputest.log 2>&1 || { tail -40 gpurun_out/r2/gputest.log; exit 1; }
tail -2 gpurun_out/r2/gputest.log
timeout -k 10 200 python -u tools/parse_prof.py 1920 1080 1000000 4 10 > gpurun_out/r2/parse_prof.log 2>&1 || { tail -20 gpurun_out/r2/parse_prof.log; exit 1; }
cat gpurun_out/r2/parse_prof.log
