#!/bin/bash
# Round-4 evidence pass (run on the GPU box from the repo root):
#   1. pytest -m gpu (every GPU test) and smoke()
#   2. bench lines: the driver shape (with the CPU baseline), 256-step launches
#      with the launch-length sweep, C1, the windowed C2 / C4 / C5, n-step 20
#   3. rocprofv3 kernel traces of the same commands, and separate FETCH_SIZE /
#      WRITE_SIZE / SQ PMC passes of the driver shape, 1- and 256-step launches
#      and of C4 / C5 (gather + step kernels)
# Every GPU step has its own time limit; a failure, abort or timeout ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04final
mkdir -p $O
PT="python -u -m pytest -v --timeout 180 --timeout-method thread -p no:cacheprovider"
# PART=a: tests, smoke and bench lines; PART=b: the rocprof traces and PMC passes (gpurun's 1200 s limit)
if [ "${PART:-a}" = a ]; then
timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $O/smoke.log; exit 1; }
cat $O/smoke.log
run() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));r=d.get('roofline',{});print('$n', '%.4g'%d['value'], d['unit'], 'frac', r.get('frac'), 'launch_us', r.get('avg_launch_us'))"
}
run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
run bench_fuse256 300 python bench.py --steps 2048 --warmup 256 --no-cpu-baseline --sweep
run bench_C1 300 python bench.py --workload C1
run bench_nstep20 300 python bench.py --steps 512 --warmup 64 --fuse 64 --nstep 20 --no-cpu-baseline --no-probe --no-k-sweep
run bench_a16 300 python bench.py --steps 512 --warmup 64 --fuse 64 --assets 16 --no-cpu-baseline --no-probe --no-k-sweep
for w in C2 C4 C5; do
  run bench_$w 600 python bench.py --workload $w --steps 256 --warmup 64 --no-cpu-baseline --no-k-sweep
done
fi
if [ "${PART:-a}" = b ]; then
B20="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-probe --no-k-sweep"
B1="python bench.py --steps 64 --warmup 8 --fuse 1 --no-cpu-baseline --no-probe --no-k-sweep"
B256="python bench.py --steps 512 --warmup 256 --no-cpu-baseline --no-probe --no-k-sweep"
BC4="python bench.py --workload C4 --steps 128 --warmup 64 --no-cpu-baseline --no-probe --no-k-sweep"
BC5="python bench.py --workload C5 --steps 128 --warmup 64 --no-cpu-baseline --no-probe --no-k-sweep"
BC2="python bench.py --workload C2 --steps 128 --warmup 64 --no-cpu-baseline --no-probe --no-k-sweep"
BA16="python bench.py --assets 16 --steps 128 --warmup 64 --fuse 64 --no-cpu-baseline --no-probe --no-k-sweep"
for tag in 20 1 256 C2 C4 C5 a16; do
  case $tag in 20) B=$B20;; 1) B=$B1;; 256) B=$B256;; C2) B=$BC2;; C4) B=$BC4;; C5) B=$BC5;; a16) B=$BA16;; esac
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$tag -o kt -- $B > $O/kt$tag.log 2>&1 || { echo "kt$tag failed"; tail -20 $O/kt$tag.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc$tag/fetch -o p -- $B > $O/pmc${tag}_fetch.log 2>&1 || { echo "pmc fetch $tag failed"; tail -20 $O/pmc${tag}_fetch.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc$tag/write -o p -- $B > $O/pmc${tag}_write.log 2>&1 || { echo "pmc write $tag failed"; tail -20 $O/pmc${tag}_write.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAVES --output-format csv -d $O/pmc$tag/sq -o p -- $B > $O/pmc${tag}_sq.log 2>&1 || { echo "pmc sq $tag failed"; tail -20 $O/pmc${tag}_sq.log; exit 1; }
done
fi
echo r04final ${PART:-a} done
