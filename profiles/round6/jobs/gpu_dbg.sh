#!/bin/bash
cd "$(dirname "$0")/../../.."
d=gpurun_out/r6dbg; mkdir -p $d
timeout -k 10 300 python -u tools/debug/gom_diff.py 352 288 500000 4 6 > $d/gom_diff.txt 2>&1; rc=$?; cat $d/gom_diff.txt | tail -30; exit $rc
