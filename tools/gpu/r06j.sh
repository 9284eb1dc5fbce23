# round 6 evidence part A: GPU suite, the driver line, n-step lines, K = 1 lines
# at the C3 shape and beyond the Infinity Cache, the reference-driven R1 line,
# one-asset handles without a window on both schedules, and PMC traffic passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 600 python -u bench.py > $O/bench_driver.json 2> $O/bench_driver.err || { echo DRIVER_FAIL; tail -20 $O/bench_driver.err; exit 1; }
python tools/bench_brief.py $O/bench_driver.json 2>/dev/null || tail -c 600 $O/bench_driver.json
export PLAN="n20_exact||--nstep 20 --nstep-pop exact --steps 20 --warmup 5 --fuse 20 --no-k-sweep --no-cpu-baseline
n20_running||--nstep 20 --nstep-pop running --steps 20 --warmup 5 --fuse 20 --no-k-sweep
k1_8192||--fuse 1 --steps 64 --warmup 16 --no-k-sweep
k1_65536||--fuse 1 --n-envs 65536 --steps 64 --warmup 16 --no-k-sweep
k1_262144||--fuse 1 --n-envs 262144 --steps 32 --warmup 8 --no-k-sweep
R1_agent_8192||--workload R1 --n-envs 8192 --win-fuse 1 --steps 64 --warmup 16
R1_agent_65536||--workload R1 --n-envs 65536 --win-fuse 1 --steps 32 --warmup 8
one_trio_65536||--assets 1 --n-envs 65536 --schedule trio --fuse 20 --steps 40 --warmup 20 --no-k-sweep
one_single_65536||--assets 1 --n-envs 65536 --schedule single --fuse 20 --steps 40 --warmup 20 --no-k-sweep"
TAG=r06j/ab bash tools/ab_bench.sh || exit 1
for spec in "C3_trendou_65536x8_fuse1|N=65536 FUSE=1 REPS=16" "C3_trendou_262144x8_fuse1|N=262144 FUSE=1 REPS=8" "C3_trendou_8192x8_n20_running_fuse20|NSTEP=20 NSTEP_POP=running FUSE=20 REPS=8"; do
  name=${spec%%|*}; probe=${spec#*|}
  TAG=r06j_$name LIBS="$name=madigan_amd/libmadigan_hip.so" PROBE="$probe" SQ=0 EXTRA_GROUPS="FETCH_SIZE WRITE_SIZE" bash tools/pmc_pass.sh > $O/pmc_$name.txt 2>&1 || { echo PMC_FAIL $name; tail -10 $O/pmc_$name.txt; exit 1; }
  tail -2 $O/pmc_$name.txt
done
echo r06j done
