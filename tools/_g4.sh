export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 200 python -u tools/parse_prof.py 1920 1080 1000000 4 6 > gpurun_out/r2/parse_prof.log 2>&1 || { tail -20 gpurun_out/r2/parse_prof.log; exit 1; }
cat gpurun_out/r2/parse_prof.log
timeout -k 10 200 python -u tools/capi_latency.py 1920 1080 1000000 12 > gpurun_out/r2/capi_lat.log 2>&1 || { tail -20 gpurun_out/r2/capi_lat.log; exit 1; }
cat gpurun_out/r2/capi_lat.log
