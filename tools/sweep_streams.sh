# Per-GPU capacity sweep: streams per GPU x encoder lanes (bench.py without the CPU leg).
# usage: bash tools/sweep_streams.sh "--streams 8" "--streams 32 --lanes 2" ...
set -e
mkdir -p gpurun_out/sweep
for cfg in "$@"; do
  n=$(echo $cfg | tr -d ' -')
  echo "== $cfg"
  timeout -k 10 150 python -u bench.py --steps 160 --warmup 32 --no-cpu-baseline $cfg > gpurun_out/sweep/$n.log 2>&1
  tail -1 gpurun_out/sweep/$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
