#!/bin/bash
# round 6, job I: A/B of the granule poll backoff (H264MI_POLL_BACKOFF 1 = lib/libh264mi.so, 0 = lib/ab/libh264mi_nobackoff.so):
# enc_mb_kernel FETCH_SIZE at 128 streams (encoder alone), then the pipeline at 128 and 32 streams, alternating builds
cd "$(dirname "$0")/../../.."
root=$(pwd); d=$root/gpurun_out/r6i; mkdir -p $d
NB=$root/openh264-wasm_amd/lib/ab/libh264mi_nobackoff.so
cd /tmp && export TMPDIR=/tmp
for v in on off; do
  L=""; [ $v = off ] && L=$NB
  H264MI_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $d/fetch_$v -o run --output-format csv -- python3 $root/bench.py --traffic-probe --streams 128 > $d/fetch_$v.log 2>&1 || { echo "pass $v failed"; tail -3 $d/fetch_$v.log; exit 1; }
done
cd $root && python3 - <<'PY'
import csv, glob, collections
for v in ('on', 'off'):
    per = collections.defaultdict(float)
    for f in glob.glob(f'gpurun_out/r6i/fetch_{v}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'enc_mb_kernel' in r['Kernel_Name']: per[int(r['Dispatch_Id'])] += float(r['Counter_Value'])
    ks = sorted(per)[2:]
    print('backoff', v, 'FETCH_SIZE KiB per launch', sum(per[k] for k in ks) / len(ks))
PY
for rep in 1 2; do for v in on off; do for S in 128 32; do
  L=""; [ $v = off ] && L=$NB
  H264MI_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-traffic --no-cpu-baseline --clip 30 --streams $S > $d/b_${v}_s${S}_$rep.json 2> $d/b_${v}_s${S}_$rep.err || { tail -3 $d/b_${v}_s${S}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$d/b_${v}_s${S}_$rep.json')); k=d['kernels']; print('backoff $v S $S rep $rep', round(d['value']), round(d['ms_per_step'],2), {a: round(b['avg_ms'],2) for a, b in k.items()})"
done; done; done
