#!/bin/bash
# encoder-alone kernel time for variant libraries (lib/var_<name>.so) beside the base library
set -o pipefail
root=$(pwd); out=gpurun_out/encvar; mkdir -p $out
for v in base "$@"; do
  lib=$root/openh264-wasm_amd/lib/libh264mi.so; [ $v != base ] && lib=$root/openh264-wasm_amd/lib/var_$v.so
  cd /tmp && export TMPDIR=/tmp
  H264MI_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $root/$out/$v -o run --output-format csv -- python3 $root/tools/enc_only.py 32 8 > $root/$out/$v.log 2>&1 || { echo "$v failed"; tail -5 $root/$out/$v.log; exit 1; }
  cd $root && echo "$v: $(python3 tools/prof_summary.py $out/$v 2>/dev/null | grep enc_mb_kernel)"
done

