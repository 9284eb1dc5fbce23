#!/bin/bash
# profiling recipe (run on the GPU box from the repo root)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo; cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
B="python bench.py --steps 512 --warmup 256 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $B > $OUT/kt.log 2>&1 || { echo "kt failed"; tail -20 $OUT/kt.log; exit 1; }
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM --output-format csv -d $OUT/pmc1 -o pmc1 -- $B > $OUT/pmc1.log 2>&1 || { echo "pmc1 failed"; tail -20 $OUT/pmc1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/pmc2 -o pmc2 -- $B > $OUT/pmc2.log 2>&1 || { echo "pmc2 failed"; tail -20 $OUT/pmc2.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d $OUT/pmc3 -o pmc3 -- $B > $OUT/pmc3.log 2>&1 || { echo "pmc3 failed"; tail -20 $OUT/pmc3.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc4 -o pmc4 -- $B > $OUT/pmc4.log 2>&1 || { echo "pmc4 failed"; tail -20 $OUT/pmc4.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc5 -o pmc5 -- $B > $OUT/pmc5.log 2>&1 || { echo "pmc5 failed"; tail -20 $OUT/pmc5.log; exit 1; }
find $OUT -name "*.csv"
