set -o pipefail
mkdir -p gpurun_out/r2j
timeout -k 10 300 python -u tools/parse_prof.py 1920 1080 1000000 2 12 2>&1 | grep -v amdgpu.ids | tail -4
for cfg in "4 3 4" "1 8 10" "2 6 6" "1 12 14" "2 8 8"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --group $1 --parse-streams $2 --stages $3 > gpurun_out/r2j/g$1p$2.log 2>&1 || { echo "FAIL $cfg"; tail -5 gpurun_out/r2j/g$1p$2.log; exit 1; }
  echo "G=$1 P=$2 stages=$3: $(grep -o '"value": [0-9.]*' gpurun_out/r2j/g$1p$2.log | head -1) $(grep -o '"dec_parse_kernel": {"avg_ms": [0-9.]*' gpurun_out/r2j/g$1p$2.log)"
done
