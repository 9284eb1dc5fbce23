W="--steps 128 --warmup 64 --no-cpu-baseline"
export PLAN="R1_64k_wf64||--workload R1 --n-envs 65536 $W
R1_64k_wf32||--workload R1 --n-envs 65536 --win-fuse 32 $W
R1_64k_wf16||--workload R1 --n-envs 65536 --win-fuse 16 $W
R1_64k_wf16_kmaj|MGN_GATHER_KMAJOR=1|--workload R1 --n-envs 65536 --win-fuse 16 $W
R1_32k_wf64||--workload R1 --n-envs 32768 $W
R1_16k_wf64||--workload R1 --n-envs 16384 $W
R1_16k_wf64_kmaj|MGN_GATHER_KMAJOR=1|--workload R1 --n-envs 16384 $W"
export TAG=r06m
bash tools/ab_bench.sh
# R1 at 65536 envs: the three-role ONE layout vs the single-role kernel, SQ counters per step launch
cd $GRAFT_REPO_ROOT
for sc in trio single; do
  TAG=r06m_R1_64k_$sc LIBS="R1_step_65536x1_$sc=madigan_amd/libmadigan_hip.so" PROBE="WORKLOAD=R1 ASSETS=1 N=65536 FUSE=64 REPS=3 SCHED=$sc" SQ=1 EXTRA_GROUPS="FETCH_SIZE WRITE_SIZE" bash tools/pmc_pass.sh > gpurun_out/r06m/pmc_R1_64k_$sc.txt 2>&1 || { echo PMC_FAIL $sc; tail -10 gpurun_out/r06m/pmc_R1_64k_$sc.txt; exit 1; }
  tail -1 gpurun_out/r06m/pmc_R1_64k_$sc.txt
done
