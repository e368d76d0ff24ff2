set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3c_pytest.log 2>&1 || { echo "pytest FAILED"; grep -B3 "Error\|assert" gpurun_out/r3c_pytest.log | head -40; exit 1; }
tail -1 gpurun_out/r3c_pytest.log
mkdir -p gpurun_out/cap4
run() { tag=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/cap4/$tag.log 2>&1 || { echo FAIL $tag; tail -5 gpurun_out/cap4/$tag.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/cap4/$tag.log') if l.startswith('{')][-1])
r=d['roofline']
print('$tag', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v['avg_ms'],3) for k,v in d['kernels'].items()}, d['parity']['selfcheck'][-4:], 'traffic', r['traffic'] and round(r['traffic']/1e6,1), r['traffic_range'] and [round(x/1e6,1) for x in r['traffic_range']], r['traffic_note'][-60:])"; }
run s8_20_traffic --streams 8 --steps 20 --warmup 5
run s32_20 --no-traffic --streams 32 --steps 20 --warmup 5
run s32_20_notail --no-traffic --streams 32 --steps 20 --warmup 5 --no-tail-frames
run s32_20_pc48 --no-traffic --streams 32 --steps 20 --warmup 5 --parse-cus 48
run s32_120 --no-traffic --streams 32 --steps 120 --warmup 16
