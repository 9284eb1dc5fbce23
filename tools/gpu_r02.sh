#!/bin/bash
# Round-2 GPU pass (run on the GPU box from the repo root):
#   1. pytest -m gpu (new test files first), smoke
#   2. bench at the driver's shape (--steps 20 --warmup 5) and at 256-step launches
#   3. rocprofv3 kernel trace + PMC passes of the driver-shape bench (20-step
#      launches) and of 1-step launches
# Each GPU step has its own time limit; a fault, abort or timeout ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r02
mkdir -p $O
stop_if_fatal() {  # exit codes other than 0 / 1 (test failures) end the GPU work
  rc=$1; what=$2
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "$what: fatal rc=$rc"; exit $rc; fi
  if grep -q "Timeout" $O/$3 2>/dev/null; then echo "$what: timeout"; exit 124; fi
}
PT="python -u -m pytest -x -v --timeout 180 --timeout-method thread -p no:cacheprovider"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 $PT tests/test_gpu_env_kats.py tests/test_gpu_configs.py > $O/pytest_new.log 2>&1
  stop_if_fatal $? "new tests" pytest_new.log
  tail -5 $O/pytest_new.log
  timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1
  stop_if_fatal $? "gpu tests" pytest_gpu.log
  tail -3 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $O/smoke.log; exit 1; }
  cat $O/smoke.log
fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { echo "bench failed"; tail -30 $O/bench20.err; exit 1; }
cat $O/bench20.json
timeout -k 10 300 python bench.py --steps 2048 --warmup 256 --no-cpu-baseline --sweep > $O/bench256.json 2> $O/bench256.err || { echo "bench256 failed"; tail -30 $O/bench256.err; exit 1; }
cat $O/bench256.json
B20="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-probe"
B1="python bench.py --steps 64 --warmup 8 --fuse 1 --no-cpu-baseline --no-probe"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt20 -o kt -- $B20 > $O/kt20.log 2>&1 || { echo "kt20 failed"; tail -20 $O/kt20.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt1 -o kt -- $B1 > $O/kt1.log 2>&1 || { echo "kt1 failed"; tail -20 $O/kt1.log; exit 1; }
for tag in 20 1; do
  B=$B20; [ $tag = 1 ] && B=$B1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc$tag/fetch -o p -- $B > $O/pmc${tag}_fetch.log 2>&1 || { echo "pmc fetch $tag failed"; tail -20 $O/pmc${tag}_fetch.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc$tag/write -o p -- $B > $O/pmc${tag}_write.log 2>&1 || { echo "pmc write $tag failed"; tail -20 $O/pmc${tag}_write.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAVES --output-format csv -d $O/pmc$tag/sq -o p -- $B > $O/pmc${tag}_sq.log 2>&1 || { echo "pmc sq $tag failed"; tail -20 $O/pmc${tag}_sq.log; exit 1; }
done
find $O -name "*.csv" | head -50
