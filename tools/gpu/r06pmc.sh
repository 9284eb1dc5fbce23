set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for spec in "C3_trendou_8192x8_fuse20|FUSE=20 REPS=8" "C3_trendou_8192x8_fuse1|FUSE=1 REPS=32 AGE=2048"; do
  n=${spec%%|*}; pr=${spec#*|}
  TAG=r06f_$n LIBS="$n=madigan_amd/libmadigan_hip.so" PROBE="WORKLOAD=C3 $pr" SQ=1 EXTRA_GROUPS="FETCH_SIZE WRITE_SIZE" bash tools/pmc_pass.sh > gpurun_out/pmc_r06f_$n.txt 2>&1 || { echo PMC_FAIL $n; tail -10 gpurun_out/pmc_r06f_$n.txt; exit 1; }
  tail -1 gpurun_out/pmc_r06f_$n.txt
done
