set -o pipefail
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_pytest.log 2>&1 || { echo "pytest FAILED"; grep -B5 "Error\|assert\|FAILED" gpurun_out/full_pytest.log | head -60; exit 1; }
tail -1 gpurun_out/full_pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -2
