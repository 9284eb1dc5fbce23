set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_nstep_running.py tests/test_gpu_reference_shape.py tests/test_gpu_bench_shapes.py tests/test_gpu_window_view.py tests/test_gpu_replay.py tests/test_gpu_configs.py > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
MADIGAN_LIB_PATH=tools/_var/nstamps/libmadigan_hip.so NSTEP=20 NSTEP_POP=running FUSE=20 timeout -k 10 200 python tools/stamps_trio.py > $O/stamps_running.json 2> $O/stamps_running.err || { echo stamps fail; tail -5 $O/stamps_running.err; exit 1; }
echo "stamps: $(tail -1 $O/stamps_running.json)"
for pop in exact running; do
timeout -k 10 300 python -u bench.py --nstep 20 --nstep-pop $pop --steps 20 --warmup 5 --fuse 20 --no-cpu-baseline --no-k-sweep > $O/bench_n20_$pop.json 2> $O/bench_n20_$pop.err || { echo BENCH_FAIL $pop; tail -20 $O/bench_n20_$pop.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_n20_$pop.json'));print('n20 $pop', d['value'], d['kernel_us_per_step'], d['timed_region_us_per_launch'])"
done
for wl in "R1 8192" "R1 65536" "C2 4096" "C4 8192" "C5 8192"; do
set -- $wl
timeout -k 10 300 python -u bench.py --workload $1 --n-envs $2 --steps 256 --warmup 64 --no-cpu-baseline > $O/bench_$1_$2.json 2> $O/bench_$1_$2.err || { echo BENCH_FAIL $wl; tail -20 $O/bench_$1_$2.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_$1_$2.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$1 $2', '%.4g'%d['value'], 'gather_us %.1f frac %.3f'%(r['avg_launch_us'], r['frac']), 'step_us', d.get('step_launch_avg_us'))"
done
