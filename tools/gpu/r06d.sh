set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_nstep_running.py tests/test_gpu_parity.py -k "running or nstep" > $O/pytest_running.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_running.txt; exit 1; }
tail -1 $O/pytest_running.txt
MADIGAN_LIB_PATH=tools/_var/nstamps/libmadigan_hip.so NSTEP=20 NSTEP_POP=running FUSE=20 timeout -k 10 200 python tools/stamps_trio.py > $O/stamps_running.json 2> $O/stamps_running.err || { echo stamps fail; tail -5 $O/stamps_running.err; exit 1; }
echo "stamps: $(tail -1 $O/stamps_running.json)"
for pop in exact running; do
timeout -k 10 300 python -u bench.py --nstep 20 --nstep-pop $pop --steps 20 --warmup 5 --fuse 20 --no-cpu-baseline --no-k-sweep > $O/bench_n20_$pop.json 2> $O/bench_n20_$pop.err || { echo BENCH_FAIL $pop; tail -20 $O/bench_n20_$pop.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_n20_$pop.json'));print('$pop', d['value'], d['kernel_us_per_step'], d['timed_region_us_per_launch'])"
done
