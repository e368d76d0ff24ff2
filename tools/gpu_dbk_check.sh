set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "encoder or decoder or configs or content or batch" > gpurun_out/dbk_pytest.log 2>&1 || { echo "pytest FAILED"; grep -B5 "Error\|assert" gpurun_out/dbk_pytest.log | head -60; exit 1; }
tail -1 gpurun_out/dbk_pytest.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/enc_only2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/enc_only.py 32 8 > $GRAFT_REPO_ROOT/gpurun_out/enc_only2.log 2>&1
cd $GRAFT_REPO_ROOT && python3 tools/prof_summary.py gpurun_out/enc_only2 | head -5
bash tools/sweep_pcus.sh 24
timeout -k 10 300 python3 tools/enc_prof.py 1920 1080 1000000 32 4 2>&1 | grep -v amdgpu | tail -2
