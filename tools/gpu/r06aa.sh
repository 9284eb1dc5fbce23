set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_variants.py tests/test_gpu_configs.py tests/test_gpu_env_kats.py > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
H="MADIGAN_LIB_PATH=tools/_var/head/libmadigan_hip.so"
PLAN=""
for r in 1 2; do
for wl in "R1_8k|--workload R1 --n-envs 8192 --win-fuse 1 --steps 64 --warmup 16 --no-cpu-baseline" "R1_64k|--workload R1 --n-envs 65536 --win-fuse 1 --steps 32 --warmup 8 --no-cpu-baseline" "C2|--workload C2 --win-fuse 1 --steps 64 --warmup 16 --no-cpu-baseline"; do
  n=${wl%%|*}; a=${wl#*|}
  PLAN="$PLAN
${n}_head_$r|$H|$a
${n}_new_$r||$a"
done; done
export TAG=r06aa/ab PLAN
bash tools/ab_bench.sh
