#!/bin/bash
# round 6, job C: exact GOM rate control vs the row plan at high stream counts (tools/gom_ab.py)
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6c; mkdir -p $d
timeout -k 10 500 python -u tools/gom_ab.py --streams ${GOM_AB_STREAMS:-32,128,256} > $d/gom_ab.jsonl 2> $d/gom_ab.err; rc=$?
cat $d/gom_ab.jsonl; tail -3 $d/gom_ab.err; exit $rc
