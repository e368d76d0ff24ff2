set -o pipefail
mkdir -p gpurun_out/aba
v() { grep -o '"value": [0-9.]*' $1 | head -1; }
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/aba/1.log 2>&1; echo "plain: $(v gpurun_out/aba/1.log)"
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-traffic --parity-frames 0 > gpurun_out/aba/2.log 2>&1; echo "cpu baseline, new order: $(v gpurun_out/aba/2.log)"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/aba/3.log 2>&1; echo "traffic only: $(v gpurun_out/aba/3.log)"
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/aba/4.log 2>&1; echo "plain: $(v gpurun_out/aba/4.log)"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/aba/5.log 2>&1; echo "both: $(v gpurun_out/aba/5.log)"
