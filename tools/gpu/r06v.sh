set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_reference_shape.py tests/test_gpu_bench_shapes.py tests/test_gpu_window_view.py tests/test_gpu_replay.py tests/test_gpu_configs.py > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
H="MADIGAN_LIB_PATH=tools/_var/head/libmadigan_hip.so"
W="--steps 256 --warmup 64 --no-cpu-baseline"
PLAN=""
for r in 1 2; do
for wl in "R1_64k|--workload R1 --n-envs 65536 --steps 128 --warmup 64 --no-cpu-baseline" "R1_8k|--workload R1 --n-envs 8192 $W" "C2|--workload C2 $W" "C4|--workload C4 $W" "C5|--workload C5 $W"; do
  n=${wl%%|*}; a=${wl#*|}
  PLAN="$PLAN
${n}_head_$r|$H|$a
${n}_new_$r||$a"
done; done
export TAG=r06v/ab PLAN
bash tools/ab_bench.sh
