#!/bin/bash
# round 6, job S: single-call C-ABI latency (the wrapper's call pattern), 1080p 1 / 8 Mbps, row plan and exact GOM
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6s; mkdir -p $d
timeout -k 10 300 python -u tools/capi_latency.py 1920 1080 1000000 24 > $d/capi_1m.json 2> $d/e1.err || { tail -3 $d/e1.err; exit 1; }
timeout -k 10 300 python -u tools/capi_latency.py 1920 1080 8000000 24 > $d/capi_8m.json 2> $d/e2.err || { tail -3 $d/e2.err; exit 1; }
H264MI_GOM_EXACT=1 timeout -k 10 300 python -u tools/capi_latency.py 1920 1080 8000000 24 > $d/capi_8m_exact.json 2> $d/e3.err || { tail -3 $d/e3.err; exit 1; }
for f in capi_1m capi_8m capi_8m_exact; do echo $f; cut -c1-600 $d/$f.json; done
