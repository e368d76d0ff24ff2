#!/bin/bash
# SQ / SQC counters of dec_parse_kernel on one synthetic slice kind of tools/parse_mix.py (one pass per
# counter set, no trace domains) -> gpurun_out/pmc_mix/<kind>_<pass>/   usage: tools/pmc_mix.sh <kind>
set -e
kind=$1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_SALU" \
           "SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $root/gpurun_out/pmc_mix/${kind}_$i -o run --output-format csv -- \
    python3 $root/tools/parse_mix.py --kind $kind > $root/gpurun_out/pmc_mix/${kind}_$i.log 2>&1
done
cd $root && python3 - "$kind" <<'PY'
import csv, glob, sys, collections
kind = sys.argv[1]
for i in (1, 2):
    fs = glob.glob(f'gpurun_out/pmc_mix/{kind}_{i}/**/*counter_collection.csv', recursive=True)
    d = collections.defaultdict(list)
    for f in fs:
        for row in csv.DictReader(open(f)):
            if 'dec_parse_kernel' in row['Kernel_Name']:
                d[(int(row['Dispatch_Id']), row['Counter_Name'])].append(float(row['Counter_Value']))
    disp = sorted({k[0] for k in d})
    for di in disp:
        print(kind, 'dispatch', di, ' '.join(f'{c}={sum(v):.0f}' for (dd, c), v in sorted(d.items()) if dd == di))
PY
