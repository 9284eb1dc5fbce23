#!/bin/bash
# HBM-bound C3-family lines: the step kernel at N envs
# large enough that the SoA state (1.4 KB / env) exceeds the 256 MB Infinity
# Cache, with a kernel trace and FETCH / WRITE PMC passes of the same command.
#   N_LIST="262144 524288" bash tools/gpu_hbm.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/hbm
mkdir -p $O
for N in ${N_LIST:-262144 524288}; do
  B="python bench.py --n-envs $N --steps 512 --warmup 64 --fuse 64 --no-cpu-baseline --no-probe"
  timeout -k 10 300 $B > $O/bench_$N.json 2> $O/bench_$N.err || { echo "bench $N failed"; tail -20 $O/bench_$N.err; exit 1; }
  cat $O/bench_$N.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$N -o kt -- $B > $O/kt_$N.log 2>&1 || { echo "kt $N failed"; tail -20 $O/kt_$N.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$N/fetch -o p -- $B > $O/pmc_${N}_fetch.log 2>&1 || { echo "pmc fetch $N failed"; tail -20 $O/pmc_${N}_fetch.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_$N/write -o p -- $B > $O/pmc_${N}_write.log 2>&1 || { echo "pmc write $N failed"; tail -20 $O/pmc_${N}_write.log; exit 1; }
done
echo hbm done
