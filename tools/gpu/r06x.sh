set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_nstep_running.py tests/test_gpu_reference_shape.py tests/test_gpu_parity.py -k "nstep or running or reference" > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest.txt | head; tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
W="--steps 256 --warmup 64 --no-cpu-baseline"
export PLAN="R1_8k_sortinoB||--workload R1 --n-envs 8192 --shaper sortino_shaperB $W
R1_8k_sortinoB_running||--workload R1 --n-envs 8192 --shaper sortino_shaperB --nstep-pop running $W
R1_64k_sortinoB_running||--workload R1 --n-envs 65536 --shaper sortino_shaperB --nstep-pop running --steps 128 --warmup 64 --no-cpu-baseline
R1_8k_running||--workload R1 --n-envs 8192 --nstep-pop running $W
n20r||--nstep 20 --nstep-pop running --steps 20 --warmup 5 --fuse 20 --no-k-sweep --no-cpu-baseline"
TAG=r06x/ab bash tools/ab_bench.sh || exit 1
