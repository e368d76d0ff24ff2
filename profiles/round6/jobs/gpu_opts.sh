#!/bin/bash
# round 6, end: same-box A/B (interleaved) of encoder build options re-checked after the MB-loop wait fixes: default,
# H264MI_ENC_XF_LDS=0 (transform constants in registers), H264MI_ENC_LATE_COMMIT=1, H264MI_ENC_PH1=0
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6opt; mkdir -p $d; out=$d/ab.txt; : > $out
L=openh264-wasm_amd/lib/ab
for r in 1 2; do
  for lib in $L/libh264mi_def.so $L/libh264mi_xfreg.so $L/libh264mi_lcommit.so $L/libh264mi_ph0.so; do
    b=$(basename $lib .so)
    H264MI_LIB=$lib timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $d/${b}_$r.json 2> $d/${b}_$r.err || { echo "$b $r failed" >> $out; tail -5 $d/${b}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$d/${b}_$r.json')); print('$r $b', round(d['value'],1), round(d['ms_per_step'],3), round(d['kernels']['enc_mb_kernel']['avg_ms'],3), d['parity']['selfcheck'][-4:])" >> $out
  done
done
cat $out
