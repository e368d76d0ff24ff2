set -o pipefail
mkdir -p gpurun_out/r2r
for cfg in "4 3 16 4" "4 3 24 4" "1 16 24 20" "1 16 32 20" "2 8 24 10"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-traffic --steps 20 --warmup 5 --group $1 --parse-streams $2 --parse-cus $3 --stages $4 > gpurun_out/r2r/g$1p$2c$3.log 2>&1 || { echo "FAIL $cfg"; tail -5 gpurun_out/r2r/g$1p$2c$3.log; exit 1; }
  echo "G=$1 P=$2 cus=$3: $(grep -o '"value": [0-9.]*' gpurun_out/r2r/g$1p$2c$3.log | head -1) $(grep -o '"kernels": .*}}' gpurun_out/r2r/g$1p$2c$3.log | cut -c1-160)"
done
