#!/bin/bash
# round 6: same-box A/B (interleaved) of the granule-poll wait fixes: base (before), vmfix (explicit vmcnt(0) at the
# poll's exits), vmfix2 (+ first test outside the poll loop), st2 (+ the row above's pixel granules preloaded with
# the previous MB's outputs and taken at step 1, H264MI_ENC_ST2PF=1); then the encoder parity tests on st2
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6st2; mkdir -p $d; out=$d/ab.txt; : > $out
L=openh264-wasm_amd/lib/ab
for r in 1 2; do
  for lib in $L/libh264mi_base.so $L/libh264mi_vmfix.so $L/libh264mi_vmfix2.so $L/libh264mi_st2.so; do
    b=$(basename $lib .so)
    H264MI_LIB=$lib timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $d/${b}_$r.json 2> $d/${b}_$r.err || { echo "$b $r failed" >> $out; tail -5 $d/${b}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$d/${b}_$r.json')); print('$r $b', round(d['value'],1), round(d['ms_per_step'],3), round(d['kernels']['enc_mb_kernel']['avg_ms'],3), d['parity']['selfcheck'][-4:])" >> $out
  done
done
cat $out
H264MI_LIB=$L/libh264mi_st2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_batch.py -m gpu -x -q --timeout 180 --timeout-method thread > $d/gpu_tests_st2.txt 2>&1
rc=$?; tail -3 $d/gpu_tests_st2.txt; exit $rc
