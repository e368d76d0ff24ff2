#!/bin/bash
# round 6: the Intra4x4 search without vector-load waits (tap table in LDS, decision tables nibble-packed for scalar
# loads): the whole GPU suite on the default library, same-box bench A/B against the library before it (vmfix2),
# and single-call C-ABI latencies (the IDR encode is all Intra4x4 searches) with both
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6i4; mkdir -p $d; out=$d/ab.txt; : > $out
L=openh264-wasm_amd/lib/ab
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $d/gpu_tests.txt 2>&1
rc=$?; tail -3 $d/gpu_tests.txt; [ $rc -ne 0 ] && { echo "tests rc=$rc"; exit $rc; }
for r in 1 2; do
  for lib in $L/libh264mi_vmfix2.so $L/libh264mi_i4lds.so; do
    b=$(basename $lib .so)
    H264MI_LIB=$lib timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $d/${b}_$r.json 2> $d/${b}_$r.err || { echo "$b $r failed" >> $out; tail -5 $d/${b}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$d/${b}_$r.json')); print('$r $b', round(d['value'],1), round(d['ms_per_step'],3), round(d['kernels']['enc_mb_kernel']['avg_ms'],3), d['parity']['selfcheck'][-4:])" >> $out
  done
done
for lib in $L/libh264mi_vmfix2.so $L/libh264mi_i4lds.so; do
  b=$(basename $lib .so)
  H264MI_LIB=$lib timeout -k 10 300 python -u tools/capi_latency.py 1920 1080 8000000 24 > $d/capi_8m_$b.json 2> $d/capi_$b.err || { tail -3 $d/capi_$b.err; exit 1; }
  python3 -c "import json; print('$b', json.load(open('$d/capi_8m_$b.json')))" | cut -c1-600 >> $out
done
cat $out
