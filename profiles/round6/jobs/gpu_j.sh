#!/bin/bash
# round 6, job J: A/B of the encoder's stream-grouped tickets (H264MI_ENC_SGRP = streams per group of a queue, 0 = all):
# enc_mb_kernel FETCH_SIZE (encoder alone) and the pipeline
cd "$(dirname "$0")/../../.."
root=$(pwd); d=$root/gpurun_out/r6j; mkdir -p $d
cd /tmp && export TMPDIR=/tmp
for G in ${GROUPS_:-0 2 4 8}; do
  H264MI_ENC_SGRP=$G timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $d/fetch_$G -o run --output-format csv -- python3 $root/bench.py --traffic-probe --streams ${S:-128} > $d/fetch_$G.log 2>&1 || { echo "pass $G failed"; tail -3 $d/fetch_$G.log; exit 1; }
done
cd $root && python3 - <<'PY'
import csv, glob, collections, os
for v in os.environ.get('GROUPS_', '0 2 4 8').split():
    per = collections.defaultdict(float)
    for f in glob.glob(f'gpurun_out/r6j/fetch_{v}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'enc_mb_kernel' in r['Kernel_Name']: per[int(r['Dispatch_Id'])] += float(r['Counter_Value'])
    ks = sorted(per)[2:]
    print('sgrp', v, 'FETCH_SIZE KiB per launch', sum(per[k] for k in ks) / len(ks))
PY
for rep in 1 2; do for G in ${GROUPS_:-0 2 4 8}; do
  H264MI_ENC_SGRP=$G timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-traffic --no-cpu-baseline --clip 30 --streams ${S:-128} > $d/b_$G_$rep.json 2> $d/b_$G.err || { tail -3 $d/b_$G.err; exit 1; }
  python3 -c "import json; d=json.load(open('$d/b_$G_$rep.json')); k=d['kernels']; print('sgrp $G rep $rep', round(d['value']), round(d['ms_per_step'],2), {a: round(b['avg_ms'],2) for a, b in k.items()}, d['parity']['vs_oracle'][:40])"
done; done
