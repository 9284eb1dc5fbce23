#!/bin/bash
# windowed workloads: kernel-trace stats and HBM traffic (FETCH_SIZE, WRITE_SIZE
# in separate passes) of the launch-history gather; run on the GPU box
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
for w in C4 C5; do
  OUT=gpurun_out/profw/$w
  mkdir -p $OUT
  B="python bench.py --workload $w --no-cpu-baseline --steps 256 --warmup 64"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $B > $OUT/kt.log 2>&1 || { echo "kt $w failed"; tail -20 $OUT/kt.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc4 -o pmc4 -- $B > $OUT/pmc4.log 2>&1 || { echo "pmc4 $w failed"; tail -20 $OUT/pmc4.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc5 -o pmc5 -- $B > $OUT/pmc5.log 2>&1 || { echo "pmc5 $w failed"; tail -20 $OUT/pmc5.log; exit 1; }
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench $w failed"; tail -20 $OUT/bench.err; exit 1; }
done
timeout -k 10 300 python bench.py --workload C2 --no-cpu-baseline > gpurun_out/profw/bench_C2.json 2> gpurun_out/profw/bench_C2.err || { echo "bench C2 failed"; exit 1; }
find gpurun_out/profw -name "*stats.csv" -o -name "*counter_collection.csv" | head
