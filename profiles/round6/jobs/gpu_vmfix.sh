#!/bin/bash
# round 6: explicit vmcnt(0) at the granule poll's exits (no false pending registers at the P path's start):
# same-box A/B of the bench against the library without it (interleaved), then the encoder parity tests on it
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6vmfix; mkdir -p $d; out=$d/ab.txt; : > $out
for r in 1 2; do
  for lib in openh264-wasm_amd/lib/ab/libh264mi_base.so openh264-wasm_amd/lib/ab/libh264mi_vmfix.so; do
    b=$(basename $lib .so)
    H264MI_LIB=$lib timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $d/${b}_$r.json 2> $d/${b}_$r.err || { echo "$b $r failed" >> $out; tail -5 $d/${b}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$d/${b}_$r.json')); print('$r $b', round(d['value'],1), round(d['ms_per_step'],3), round(d['kernels']['enc_mb_kernel']['avg_ms'],3), d['parity']['vs_oracle'][-4:] if isinstance(d['parity']['vs_oracle'], str) else d['parity'])" >> $out
  done
done
cat $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_batch.py -m gpu -x -q --timeout 180 --timeout-method thread > $d/gpu_tests.txt 2>&1
rc=$?; tail -3 $d/gpu_tests.txt; exit $rc
