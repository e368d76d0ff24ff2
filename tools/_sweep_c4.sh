set -o pipefail
mkdir -p gpurun_out/r2s
for cfg in "4 3 0" "4 6 0" "8 6 0" "4 6 64" "8 4 64" "16 3 0"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --config 4 --no-cpu-baseline --no-traffic --group $1 --parse-streams $2 --parse-cus $3 > gpurun_out/r2s/g$1p$2c$3.log 2>&1 || { echo "FAIL $cfg"; tail -5 gpurun_out/r2s/g$1p$2c$3.log; exit 1; }
  echo "G=$1 P=$2 cus=$3: $(grep -o '"value": [0-9.]*' gpurun_out/r2s/g$1p$2c$3.log | head -1) $(grep -o '"kernels": .*}}' gpurun_out/r2s/g$1p$2c$3.log | cut -c1-170)"
done
