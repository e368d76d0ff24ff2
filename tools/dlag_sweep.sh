#!/bin/bash
# encoder launch time at 32 streams for deblocking-ticket lags (env H264MI_DBK_LAG), encoder alone
set -o pipefail
cd /tmp && export TMPDIR=/tmp
for d in "$@"; do
  H264MI_DBK_LAG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/dlag_$d -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/enc_only.py 32 8 > $GRAFT_REPO_ROOT/gpurun_out/dlag_$d.log 2>&1 || { echo "lag $d failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/dlag_$d.log; exit 1; }
  echo "lag $d: $(grep enc_mb_kernel $GRAFT_REPO_ROOT/gpurun_out/dlag_$d/run_kernel_stats.csv | head -1 | cut -d, -f1-6)"
done
