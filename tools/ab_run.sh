set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "syntax or decoder or configs or content" > gpurun_out/ab14_pytest.log 2>&1 || { echo "pytest FAILED"; grep -B5 "Error\|assert" gpurun_out/ab14_pytest.log | head -60; exit 1; }
tail -1 gpurun_out/ab14_pytest.log
PARSE_AB_BR=8000000 timeout -k 10 300 python3 tools/parse_ab.py gpurun_out/ab14/m8 v12 v13 --frames 16 2>&1 | grep -v amdgpu.ids
PARSE_AB_BR=1000000 timeout -k 10 300 python3 tools/parse_ab.py gpurun_out/ab14/m1 v12 v13 --frames 16 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python3 tools/parse_mix.py 2>&1 | grep -v amdgpu.ids
