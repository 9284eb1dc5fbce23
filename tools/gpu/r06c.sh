# running-pop n = 20 DDR anatomy: stamps (running / exact) and the row-store ablation
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06c; mkdir -p $O
for pop in running exact; do
  MADIGAN_LIB_PATH=tools/_var/nstamps/libmadigan_hip.so NSTEP=20 NSTEP_POP=$pop FUSE=20 timeout -k 10 200 python tools/stamps_trio.py > $O/stamps_$pop.json 2> $O/stamps_$pop.err || { echo stamps fail; tail -5 $O/stamps_$pop.err; exit 1; }
  echo "stamps $pop: $(tail -1 $O/stamps_$pop.json)"
done
TAG=r06c/probe ARGS="--nstep 20 --nstep-pop running --steps 400 --warmup 40 --fuse 20" VARS="nrow=tools/_var/nrow/libmadigan_hip.so" ROUNDS=2 bash tools/nst_probe.sh
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_reference_shape.py -k "bitwise" > $O/pytest_one_bitwise.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_one_bitwise.txt; exit 1; }
tail -2 $O/pytest_one_bitwise.txt
