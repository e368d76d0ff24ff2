set -o pipefail
mkdir -p gpurun_out/r2l
for cfg in "4 3 0" "4 3 8" "4 3 16" "4 3 24" "2 6 16" "1 8 16" "4 3 32"; do
  set -- $cfg
  st=$(( $1 == 1 ? 10 : ($1 == 2 ? 6 : 4) ))
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --group $1 --parse-streams $2 --parse-cus $3 --stages $st > gpurun_out/r2l/g$1p$2c$3.log 2>&1 || { echo "FAIL $cfg"; tail -5 gpurun_out/r2l/g$1p$2c$3.log; exit 1; }
  echo "G=$1 P=$2 cus=$3: $(grep -o '"value": [0-9.]*' gpurun_out/r2l/g$1p$2c$3.log | head -1) $(grep -o '"kernels": .*}}' gpurun_out/r2l/g$1p$2c$3.log | cut -c1-200)"
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --parse-cus 16 > gpurun_out/r2l/c16_240.log 2>&1 && echo "240 steps cus 16: $(grep -o '"value": [0-9.]*' gpurun_out/r2l/c16_240.log | head -1)"
timeout -k 10 200 python -u bench.py --no-cpu-baseline --config 4 --parse-cus 32 > gpurun_out/r2l/cfg4.log 2>&1 && echo "config4 cus 32: $(grep -o '"value": [0-9.]*' gpurun_out/r2l/cfg4.log | head -1)"
