#!/bin/bash
# reconstruction section profiles (tools/recon_prof.py, 32 x 1080p, 8 frames) of library builds, same box
# usage: tools/ab_recon_prof.sh <tag> lib...
cd "$(dirname "$0")/../../.."
tag=$1; shift
out=gpurun_out/rprof_${tag}.txt; : > $out
for lib in "$@"; do
  echo "== $(basename $lib)" >> $out
  H264MI_LIB=$lib timeout -k 10 200 python -u tools/recon_prof.py 1920 1080 1000000 32 8 2>&1 | grep -v amdgpu.ids >> $out || exit 1
done
cat $out
