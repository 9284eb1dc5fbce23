#!/bin/bash
# Round-2 closing GPU pass (run on the GPU box from the repo root):
#   1. pytest -m gpu (every GPU test), smoke
#   2. bench at the driver's shape (--steps 20 --warmup 5, with the CPU
#      baseline), the 256-step sweep, the C1 latency line
#   3. rocprofv3 kernel traces + separate FETCH_SIZE / WRITE_SIZE / SQ PMC
#      passes of 20-, 1- and 256-step launches
# Each GPU step has its own time limit; a failure, abort or timeout ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r02
mkdir -p $O
PT="python -u -m pytest -v --timeout 180 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { echo "bench failed"; tail -30 $O/bench20.err; exit 1; }
cat $O/bench20.json
timeout -k 10 300 python bench.py --steps 2048 --warmup 256 --no-cpu-baseline --sweep > $O/bench256.json 2> $O/bench256.err || { echo "bench256 failed"; tail -30 $O/bench256.err; exit 1; }
timeout -k 10 300 python bench.py --workload C1 > $O/c1.json 2> $O/c1.err || { echo "c1 failed"; tail -30 $O/c1.err; exit 1; }
B20="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-probe"
B1="python bench.py --steps 64 --warmup 8 --fuse 1 --no-cpu-baseline --no-probe"
B256="python bench.py --steps 512 --warmup 256 --no-cpu-baseline --no-probe"
for tag in 20 1 256; do
  B=$B20; [ $tag = 1 ] && B=$B1; [ $tag = 256 ] && B=$B256
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$tag -o kt -- $B > $O/kt$tag.log 2>&1 || { echo "kt$tag failed"; tail -20 $O/kt$tag.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc$tag/fetch -o p -- $B > $O/pmc${tag}_fetch.log 2>&1 || { echo "pmc fetch $tag failed"; tail -20 $O/pmc${tag}_fetch.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc$tag/write -o p -- $B > $O/pmc${tag}_write.log 2>&1 || { echo "pmc write $tag failed"; tail -20 $O/pmc${tag}_write.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAVES --output-format csv -d $O/pmc$tag/sq -o p -- $B > $O/pmc${tag}_sq.log 2>&1 || { echo "pmc sq $tag failed"; tail -20 $O/pmc${tag}_sq.log; exit 1; }
done
echo r02b done
