set -o pipefail
H264MI_LIB=$GRAFT_REPO_ROOT/openh264-wasm_amd/lib/variants/ew3.so timeout -k 10 400 python3 bench.py --no-traffic --no-cpu-baseline > gpurun_out/ew3.log 2>&1 || { tail -5 gpurun_out/ew3.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/ew3.log').read().strip().splitlines()[-1]); k=d['kernels']; print('ew3', round(d['value'],1), round(d['ms_per_step'],2), 'enc', round(k['enc_mb_kernel']['avg_ms'],2), 'recon', round(k['dec_recon_kernel']['avg_ms'],2))"
