#!/bin/bash
# round 6, job M: encoder scheduling knobs at the 128-stream default (pipeline, no CPU leg / PMC), two passes
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6m; mkdir -p $d
run() {  # name, env assignments...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-traffic --no-cpu-baseline --clip 30 > $d/$n.json 2> $d/$n.err || { tail -3 $d/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('$d/$n.json')); k=d['kernels']; print('$n', round(d['value']), round(d['ms_per_step'],2), {a: round(b['avg_ms'],2) for a, b in k.items() if 'avg_ms' in b})"
}
for rep in 1 2; do
  run base_$rep X=0 && run xq0_$rep H264MI_ENC_XQ=0 && run lag4_$rep H264MI_DBK_LAG=4 && run lag16_$rep H264MI_DBK_LAG=16 && \
  run prio2_$rep H264MI_ENC_PRIO=2 && run prio4_$rep H264MI_ENC_PRIO=4 || exit 1
done
