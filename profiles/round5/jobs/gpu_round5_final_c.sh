#!/bin/bash
# round-5 final evidence, part C: single-call C-ABI latency at 1 and 8 Mbps (the IDR's I slice in the asm
# macroblock run), and the parse profile of the bench's 25 frames (IDR and frame-22 scene-change slices)
cd "$(dirname "$0")/../../.."
d=gpurun_out/final5; mkdir -p $d
for br in 1000000 8000000; do
  timeout -k 10 240 python -u tools/capi_latency.py 1920 1080 $br 12 > $d/capi_$br.json 2> $d/capi_$br.err || { tail -5 $d/capi_$br.err; exit 1; }
  tail -c 400 $d/capi_$br.json
done
timeout -k 10 400 python -u tools/parse_prof.py 1920 1080 1000000 4 25 2>&1 | grep "^frame" | cut -c1-110 > $d/parse_prof_25.txt || exit 1
sed -n '1p;22,25p' $d/parse_prof_25.txt
