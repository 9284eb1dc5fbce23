#!/bin/bash
# per-launch fixed cost of the step kernel: wall stamps at several launch
# lengths, instruction-fetch / wait counters of 1- and 20-step launches
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/fixed
rm -rf $O; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || echo "list failed"
for F in 1 4 20 64; do
  FUSE=$F MADIGAN_LIB_PATH=tools/_var/stamps/libmadigan_hip.so timeout -k 10 120 python tools/stamps.py > $O/stamps_$F.json 2>> $O/stamps.err || { echo "stamps failed"; tail -20 $O/stamps.err; exit 1; }
  cat $O/stamps_$F.json
done
B20="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-probe"
B1="python bench.py --steps 64 --warmup 8 --fuse 1 --no-cpu-baseline --no-probe"
for tag in 20 1; do
  B=$B20; [ $tag = 1 ] && B=$B1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_IFETCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/pmc$tag/sq -o p -- $B > $O/pmc${tag}_sq.log 2>&1 || { echo "pmc sq $tag failed"; tail -5 $O/pmc${tag}_sq.log; }
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d $O/pmc$tag/sqc -o p -- $B > $O/pmc${tag}_sqc.log 2>&1 || { echo "pmc sqc $tag failed"; tail -5 $O/pmc${tag}_sqc.log; }
done
echo fixed done
