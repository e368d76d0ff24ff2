#!/bin/bash
# round 6, end: single-call C-ABI latencies and the 8 Mbps bench line with the pinned P-slice decisions
cd "$GRAFT_REPO_ROOT"
d=gpurun_out/capi_final; mkdir -p $d
timeout -k 10 300 python -u tools/capi_latency.py 1920 1080 1000000 24 > $d/capi_1m.json 2> $d/e1.err || { tail -3 $d/e1.err; exit 1; }
timeout -k 10 300 python -u tools/capi_latency.py 1920 1080 8000000 24 > $d/capi_8m.json 2> $d/e2.err || { tail -3 $d/e2.err; exit 1; }
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --bitrate 8000000 --no-cpu-baseline --no-traffic > $d/bench_8m.json 2> $d/b8.err || { tail -3 $d/b8.err; exit 1; }
python3 -c "import json; [print(f, json.load(open('$d/'+f))) for f in ('capi_1m.json','capi_8m.json')]" | cut -c1-400
python3 -c "import json; d=json.load(open('$d/bench_8m.json')); print('8 Mbps', d['value'], d['ms_per_step'], str(d['parity']['vs_oracle'])[-30:])"
