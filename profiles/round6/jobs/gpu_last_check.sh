#!/bin/bash
# round 6, last: the GPU suite and smoke() on the in-tree library the driver will load
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6last; mkdir -p $d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $d/gpu_tests.txt 2>&1
rc=$?; tail -2 $d/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $d/smoke.txt 2>&1 || { tail -5 $d/smoke.txt; exit 1; }
tail -1 $d/smoke.txt
