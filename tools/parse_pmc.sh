#!/bin/bash
# SQ counters of dec_parse_kernel, one dispatch per frame (1 stream, 1080p): instructions and wave
# cycles per slice. usage: tools/parse_pmc.sh <outdir-name> [bitrate] [counters...]
set -e
name=${1:-parse_pmc}; br=${2:-1000000}; shift 2 || true
ctr=${@:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM}
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $ctr \
  -d $root/gpurun_out/$name -o run --output-format csv -- python3 $root/tools/parse_prof.py 1920 1080 $br 1 10 --pmc > $root/gpurun_out/$name.log 2>&1
cd $root && python3 - gpurun_out/$name <<'PY'
import csv, glob, sys
f = glob.glob(f'{sys.argv[1]}/**/*counter_collection.csv', recursive=True)[0]
rows = {}
for r in csv.DictReader(open(f)):
    if 'dec_parse' not in r['Kernel_Name']: continue
    rows.setdefault(int(r['Dispatch_Id']), {})[r['Counter_Name']] = float(r['Counter_Value'])
for d in sorted(rows):
    print(f"dispatch {d}: " + ' '.join(f'{k} {v:.0f}' for k, v in sorted(rows[d].items())))
PY
