set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06o; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_reference_shape.py tests/test_gpu_bench_shapes.py tests/test_gpu_window_view.py tests/test_gpu_replay.py tests/test_gpu_configs.py tests/test_gpu_nstep_running.py > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
W="--steps 256 --warmup 64 --no-cpu-baseline"
export PLAN="R1_65536||--workload R1 --n-envs 65536 $W
R1_65536_running||--workload R1 --n-envs 65536 --nstep-pop running $W
R1_8192||--workload R1 --n-envs 8192 $W
R1_8192_running||--workload R1 --n-envs 8192 --nstep-pop running $W
R1_8192_sortinoB||--workload R1 --n-envs 8192 --shaper sortino_shaperB $W
C2||--workload C2 $W
C4||--workload C4 $W
C5||--workload C5 $W"
TAG=r06o/ab bash tools/ab_bench.sh || exit 1
