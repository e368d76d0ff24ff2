#!/bin/bash
# round-5 final evidence, part E (after the reconstruction changes): rocprofv3 kernel trace + stats of the
# bench and the SQ wave states (part B without the encoder-only profiles, which the decoder does not change)
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
cat $d/kernel_stats_summary.txt | head -4
head -1 $d/trace_drain.txt; tail -3 $d/trace_drain.txt
./tools/pmc_sq.sh final5/sq > $d/sq_states.txt 2>&1 || exit $?
head -3 $d/sq_states.txt
