set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "decoder or configs or napi or capi or smoke or batch" > gpurun_out/capi_pytest.log 2>&1 || { echo "pytest FAILED"; grep -B5 "Error\|assert" gpurun_out/capi_pytest.log | head -60; exit 1; }
tail -1 gpurun_out/capi_pytest.log
timeout -k 10 200 python3 tools/capi_latency.py 1920 1080 8000000 12 2>&1 | grep '^{' | cut -c1-420
