set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_nstep_running.py tests/test_gpu_parity.py -k "running or nstep" > gpurun_out/r06b_pytest_running.txt 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r06b_pytest_running.txt; exit 1; }
tail -3 gpurun_out/r06b_pytest_running.txt
for pop in exact running; do
timeout -k 10 300 python -u bench.py --nstep 20 --nstep-pop $pop --steps 20 --warmup 5 --fuse 20 --no-cpu-baseline --no-k-sweep > gpurun_out/r06b_bench_n20_$pop.json 2> gpurun_out/r06b_bench_n20_$pop.err || { echo BENCH_FAIL $pop; tail -20 gpurun_out/r06b_bench_n20_$pop.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06b_bench_n20_$pop.json'));print('$pop', d['value'], d['kernel_us_per_step'], d['timed_region_us_per_launch'])"
done
