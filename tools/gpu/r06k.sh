# R1 driven one step at a time (ring path); gather counters at R1 / C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06k; mkdir -p $O
export PLAN="R1_agent_ring_8192||--workload R1 --n-envs 8192 --win-fuse 1 --steps 64 --warmup 16
R1_agent_ring_65536||--workload R1 --n-envs 65536 --win-fuse 1 --steps 32 --warmup 8
C2_agent_ring_4096||--workload C2 --win-fuse 1 --steps 64 --warmup 16"
TAG=r06k/ab bash tools/ab_bench.sh || exit 1
export PMC_KERNEL=k_hist_gather
for spec in "R1_gather_65536x1_W64|WORKLOAD=R1 ASSETS=1 N=65536 FUSE=64 REPS=3 GATHER=1" "R1_gather_8192x1_W64|WORKLOAD=R1 ASSETS=1 N=8192 FUSE=64 REPS=4 GATHER=1" "C2_gather_4096x4_W64|WORKLOAD=C2 ASSETS=4 N=4096 FUSE=64 REPS=4 GATHER=1"; do
  name=${spec%%|*}; probe=${spec#*|}
  TAG=r06k_$name LIBS="$name=madigan_amd/libmadigan_hip.so" PROBE="$probe" SQ=1 EXTRA_GROUPS="FETCH_SIZE WRITE_SIZE" bash tools/pmc_pass.sh > $O/pmc_$name.txt 2>&1 || { echo PMC_FAIL $name; tail -10 $O/pmc_$name.txt; exit 1; }
  tail -1 $O/pmc_$name.txt
done
echo r06k done
