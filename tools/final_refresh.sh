#!/bin/bash
# refresh of the headline lines after late changes -> gpurun_out/final2/
set -o pipefail
out=gpurun_out/final2; mkdir -p $out
j() { grep '^{' $1 | tail -1; }
b() { tag=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $out/$tag.log 2>&1 || { echo "$tag failed"; tail $out/$tag.log; exit 1; }
      j $out/$tag.log > $out/$tag.json; echo "$tag: $(grep -o '"value": [0-9.]*' $out/$tag.json | head -1) $(grep -o '"ms_per_step": [0-9.]*' $out/$tag.json)"; }
b bench_default --gpus 1 --steps 20 --warmup 5
b bench_240 --steps 240 --warmup 16 --no-cpu-baseline --no-traffic
b bench_8m --steps 20 --warmup 5 --bitrate 8000000
timeout -k 10 200 python3 tools/capi_latency.py 1920 1080 8000000 12 > $out/capi_8m.log 2>&1 && j $out/capi_8m.log > $out/capi_8m.json && cut -c 150-330 $out/capi_8m.json
