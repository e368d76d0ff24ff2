#!/bin/bash
# round-5 final evidence, part D: C-ABI latency over 24 frames at 8 Mbps (the frame-22 scene change
# included, round 4's 87 ms maximum), the 8 Mbps bench line, and the default 240-step bench (drain amortised)
cd "$(dirname "$0")/../../.."
d=gpurun_out/final5; mkdir -p $d
timeout -k 10 240 python -u tools/capi_latency.py 1920 1080 8000000 24 > $d/capi_8m_24.json 2> $d/capi_8m_24.err || { tail -5 $d/capi_8m_24.err; exit 1; }
tail -c 330 $d/capi_8m_24.json
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --bitrate 8000000 --no-cpu-baseline --no-traffic > $d/bench_8m.json 2> $d/bench_8m.err || { tail -5 $d/bench_8m.err; exit 1; }
python3 -c "import json; d=json.load(open('$d/bench_8m.json')); print('8m', d['value'], d['ms_per_step'], d['parity']['vs_oracle'][-30:])"
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-traffic > $d/bench_240.json 2> $d/bench_240.err || { tail -5 $d/bench_240.err; exit 1; }
python3 -c "import json; d=json.load(open('$d/bench_240.json')); print('240', d['value'], d['ms_per_step'], d['steps'], d['parity']['vs_oracle'][-30:])"
