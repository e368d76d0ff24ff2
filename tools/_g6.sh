# bench at the driver's settings, group 4 and group 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
for g in 4 1; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --group $g --no-cpu-baseline > gpurun_out/r2/bench_g$g.json 2> gpurun_out/r2/bench_g$g.err || { tail -20 gpurun_out/r2/bench_g$g.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r2/bench_g$g.json'));print('group $g', d['value'], d['ms_per_step'], d['kernels'])"
done
