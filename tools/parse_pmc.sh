#!/bin/bash
# SQ counters of dec_parse_kernel, one dispatch per frame (1 stream, 1080p, 1 Mbps): instructions
# and wave cycles per slice. usage: tools/parse_pmc.sh <outdir-name>
set -e
name=${1:-parse_pmc}
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM \
  -d $root/gpurun_out/$name -o run --output-format csv -- python3 $root/tools/parse_prof.py 1920 1080 1000000 1 10 --pmc > $root/gpurun_out/$name.log 2>&1
cd $root && python3 - gpurun_out/$name <<'PY'
import csv, glob, sys
f = glob.glob(f'{sys.argv[1]}/**/*counter_collection.csv', recursive=True)[0]
rows = {}
for r in csv.DictReader(open(f)):
    if 'dec_parse' not in r['Kernel_Name']: continue
    rows.setdefault(int(r['Dispatch_Id']), {})[r['Counter_Name']] = float(r['Counter_Value'])
for d in sorted(rows):
    c = rows[d]
    print(f"dispatch {d}: wave-cycles {c.get('SQ_WAVE_CYCLES',0):.0f} salu {c.get('SQ_INSTS_SALU',0):.0f} valu {c.get('SQ_INSTS_VALU',0):.0f} "
          f"lds {c.get('SQ_INSTS_LDS',0):.0f} smem {c.get('SQ_INSTS_SMEM',0):.0f} parked {c.get('SQ_WAIT_ANY',0):.0f} stall {c.get('SQ_WAIT_INST_ANY',0):.0f} active {c.get('SQ_ACTIVE_INST_ANY',0):.0f}")
PY
