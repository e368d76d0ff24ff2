#!/bin/bash
# round-5 GPU call: the -m gpu suite, then (if the suite ended normally: pass or test failures) the
# encoder's section profile at 32 streams
cd "$(dirname "$0")/../../.."
timeout -k 10 840 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5_gputest.log 2>&1
rc=$?
tail -3 gpurun_out/r5_gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stopping"; exit $rc; fi
timeout -k 10 240 python -u tools/enc_prof.py 1920 1080 1000000 32 6 > gpurun_out/r5_encprof_s32.txt 2>&1
rc2=$?
tail -4 gpurun_out/r5_encprof_s32.txt
exit $rc2
