#!/bin/bash
cd "$GRAFT_REPO_ROOT"
d=gpurun_out/pskip; mkdir -p $d
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $d/bench_default.json 2> $d/bench_default.err || { tail -5 $d/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$d/bench_default.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r.get('traffic_x_alg'), d['cpu_baseline']['value'], str(d['parity'])[:200])"
timeout -k 10 600 python -u bench.py --gpus 1 > $d/bench_240.json 2> $d/bench_240.err || { tail -5 $d/bench_240.err; exit 1; }
python3 -c "import json; d=json.load(open('$d/bench_240.json')); print('240 steps', d['value'], d['ms_per_step'], str(d['parity']['vs_oracle'])[:160])"
