set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_shapes.py tests/test_gpu_nstep_running.py > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
export PLAN="k1_8192||--fuse 1 --steps 64 --warmup 16 --no-k-sweep --no-cpu-baseline
k1_65536||--fuse 1 --n-envs 65536 --steps 64 --warmup 16 --no-k-sweep --no-cpu-baseline
k1_262144||--fuse 1 --n-envs 262144 --steps 32 --warmup 8 --no-k-sweep --no-cpu-baseline
drv||--steps 20 --warmup 5 --no-k-sweep --no-cpu-baseline"
TAG=r06s/ab bash tools/ab_bench.sh || exit 1
