# GPU: full -m gpu suite, parse profile, bench at the driver's settings
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/gputest.log 2>&1 || { tail -40 gpurun_out/r2/gputest.log; exit 1; }
tail -2 gpurun_out/r2/gputest.log
timeout -k 10 200 python -u tools/parse_prof.py 1920 1080 1000000 4 10 > gpurun_out/r2/parse_prof.log 2>&1 || { tail -20 gpurun_out/r2/parse_prof.log; exit 1; }
tail -3 gpurun_out/r2/parse_prof.log
for g in 4; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --group $g --no-cpu-baseline > gpurun_out/r2/bench_g$g.json 2> gpurun_out/r2/bench_g$g.err || { tail -20 gpurun_out/r2/bench_g$g.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r2/bench_g$g.json'));print('group $g', d['value'], d['ms_per_step'], d['kernels'])"
done
