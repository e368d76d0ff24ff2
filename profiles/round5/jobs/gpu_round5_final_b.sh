#!/bin/bash
# round-5 final evidence, part B: rocprofv3 kernel trace + stats of the bench, SQ wave states, encoder section
# profiles (all rows, rows 0 / 67, detail build), the encoder timeline at 32 streams
cd "$(dirname "$0")/../../.."
d=gpurun_out/final5; mkdir -p $d
./tools/gpu_trace.sh final5/trace > /dev/null || exit $?
f=$(find $d/trace -name '*kernel_stats.csv' | head -1); cp $f $d/kernel_stats.csv
python3 - <<PY > $d/kernel_stats_summary.txt
import csv
rows = list(csv.DictReader(open('$d/kernel_stats.csv')))
for r in rows[:12]:
    print(r['Name'][:60], r['Calls'], 'avg %.3f ms' % (float(r['AverageNs']) / 1e6), 'total %.1f ms' % (float(r['TotalDurationNs']) / 1e6), r['Percentage'])
PY
cat $d/kernel_stats_summary.txt | head -5
./tools/pmc_sq.sh final5/sq > $d/sq_states.txt 2>&1 || exit $?
head -3 $d/sq_states.txt
H264MI_LIB=openh264-wasm_amd/lib/libh264mi_detail.so ./tools/gpu_prof_rows.sh final5_detail > /dev/null || exit $?
mv gpurun_out/r5final5_detail_encprof_s32*.txt $d/ 2>/dev/null
timeout -k 10 200 python -u tools/enc_timeline.py 1920 1080 1000000 32 6 > $d/timeline_s32.txt 2>&1 || exit $?
grep "frame 4" -A3 $d/timeline_s32.txt | cut -c1-200
for br in 1000000 8000000; do
  timeout -k 10 240 python -u tools/capi_latency.py 1920 1080 $br 12 > $d/capi_$br.json 2> $d/capi_$br.err || { tail -5 $d/capi_$br.err; exit 1; }
  tail -c 300 $d/capi_$br.json
done
