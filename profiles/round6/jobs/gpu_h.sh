#!/bin/bash
# round 6, job H: enc_mb_kernel HBM traffic vs streams per GPU (the bench's traffic probe, encoder alone)
cd "$(dirname "$0")/../../.."
root=$(pwd); d=$root/gpurun_out/r6h; mkdir -p $d
cd /tmp && export TMPDIR=/tmp
for S in ${STREAMS:-32 128}; do
  for ctr in FETCH_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    n=$(echo $ctr | tr ' ' '_')
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d $d/s${S}_$n -o run --output-format csv -- python3 $root/bench.py --traffic-probe --streams $S > $d/s${S}_$n.log 2>&1 || { echo "pass $S $ctr failed"; tail -3 $d/s${S}_$n.log; exit 1; }
  done
done
cd $root && python3 - <<'PY'
import csv, glob, collections, os
d = 'gpurun_out/r6h'
for sub in sorted(os.listdir(d)):
    p = os.path.join(d, sub)
    if not os.path.isdir(p): continue
    per = collections.defaultdict(dict)
    for f in glob.glob(p + '/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'enc_mb_kernel' in r['Kernel_Name']:
                k = r['Counter_Name']; per[int(r['Dispatch_Id'])][k] = per[int(r['Dispatch_Id'])].get(k, 0.0) + float(r['Counter_Value'])
    ks = sorted(per)[2:]
    tot = collections.Counter()
    for k in ks: tot.update(per[k])
    print(sub, {c: v / len(ks) for c, v in tot.items()})
PY
