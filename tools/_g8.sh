# kernel trace of the default bench at the driver's settings -> timeline
export TMPDIR=/tmp
root=$GRAFT_REPO_ROOT
rm -rf $root/gpurun_out/tl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $root/gpurun_out/tl -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --steps 20 --warmup 5 "$@" > $root/gpurun_out/tl.log 2>&1
cd $root && python3 tools/timeline.py $(find gpurun_out/tl -name '*kernel_trace.csv' | head -1) 20 > gpurun_out/timeline.txt && head -5 gpurun_out/timeline.txt && grep -c . gpurun_out/timeline.txt
