#!/bin/bash
# A/B kernel variants on the GPU box: runs the bench (and enc-only rocprof) with each .so variant
# swapped in for openh264-wasm_amd/lib/libh264mi.so.  usage: tools/variant_bench.sh <name>=<so> ...
set -e
root=$(pwd)
cp openh264-wasm_amd/lib/libh264mi.so /tmp/base.so
for kv in "$@"; do
  name=${kv%%=*}; so=${kv#*=}
  cp $so openh264-wasm_amd/lib/libh264mi.so
  timeout -k 10 300 python bench.py --steps 96 --warmup 32 --no-cpu-baseline > gpurun_out/vb_$name.log 2>&1
  python -c "import json; d=json.loads(open('gpurun_out/vb_$name.log').read().strip().splitlines()[-1]); print('$name', round(d['value'],1), 'enc_mb avg ms', round(d['roofline']['avg_launch_ms'],3), d['parity_selfcheck'][-4:])"
done
cp /tmp/base.so openh264-wasm_amd/lib/libh264mi.so
