#!/bin/bash
# round 6, job D: the metric pipeline (encode+decode, parity vs the oracle) with OpenH264's exact GOM rate control,
# at the metric's 32 streams and at 256 streams, and the row plan at 256 streams for comparison
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6d; mkdir -p $d
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --gom-exact --no-traffic > $d/bench_exact_s32.json 2> $d/bench_exact_s32.err || { tail -5 $d/bench_exact_s32.err; exit 1; }
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --gom-exact --no-traffic --streams 256 --clip 8 > $d/bench_exact_s256.json 2> $d/bench_exact_s256.err || { tail -5 $d/bench_exact_s256.err; exit 1; }
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-traffic --streams 256 --clip 8 > $d/bench_rowplan_s256.json 2> $d/bench_rowplan_s256.err || { tail -5 $d/bench_rowplan_s256.err; exit 1; }
for f in bench_exact_s32 bench_exact_s256 bench_rowplan_s256; do
python3 -c "import json; d=json.load(open('$d/$f.json')); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['config']['p_frame_qp'], str(d['parity'])[:300])"
done
