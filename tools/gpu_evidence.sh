#!/bin/bash
# The round's evidence on one GPU box, in parts that each fit one gpurun call
# (TAG names gpurun_out/<TAG>*; copy what is judged into profiles/):
#   PART=A  GPU suite + smoke; the driver line and its kernel trace
#           (reconciled); 256-step launches, n = 20 DDR, 16 assets (traced)
#   PART=B  the windowed configs C2 / C4 / C5 and the reference's own shape R1
#           (8192 DDR / sortinoB, 65536 DDR), each with its kernel trace
#   PART=C  PMC: per-role VALU (ablation builds tools/_var/abl{G,L,F}), HBM
#           traffic and VALU per launch of the C3 shapes; the randomised
#           three-role fuzz against the two-role kernel and the oracle
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
T=${TAG:-ev}
case "$PART" in
A)
  TAG=$T SUITE=1 DRV=1 TRACE=1 \
    EXTRA="fuse256|--steps 2048 --warmup 256 --fuse 256 --no-k-sweep;n20|--steps 20 --warmup 5 --fuse 20 --nstep 20 --no-k-sweep --no-cpu-baseline;n20r|--steps 20 --warmup 5 --fuse 20 --nstep 20 --nstep-pop running --no-k-sweep --no-cpu-baseline;k1_65536|--fuse 1 --n-envs 65536 --steps 64 --warmup 16 --no-k-sweep --no-cpu-baseline;a16|--assets 16 --steps 512 --warmup 64 --fuse 64 --no-k-sweep" \
    bash tools/gpu_pass.sh
  ;;
B)
  TAG=$T TRACE=1 \
    EXTRA="c2|--workload C2 --steps 256 --warmup 64;c4|--workload C4 --steps 256 --warmup 64;c5|--workload C5 --steps 256 --warmup 64;r1_8k|--workload R1 --n-envs 8192 --steps 256 --warmup 64;r1_8k_sortino|--workload R1 --n-envs 8192 --steps 256 --warmup 64 --shaper sortino_shaperB;r1_64k|--workload R1 --n-envs 65536 --steps 128 --warmup 64;r1_64k_running|--workload R1 --n-envs 65536 --steps 128 --warmup 64 --nstep-pop running;r1_8k_running|--workload R1 --n-envs 8192 --steps 256 --warmup 64 --nstep-pop running" \
    bash tools/gpu_pass.sh
  ;;
C)
  TAG=${T}_roles LIBS="base=madigan_amd/libmadigan_hip.so ablG=tools/_var/ablG/libmadigan_hip.so ablL=tools/_var/ablL/libmadigan_hip.so ablF=tools/_var/ablF/libmadigan_hip.so" \
    PROBE="WORKLOAD=C3 FUSE=20 REPS=8" bash tools/pmc_pass.sh || exit 1
  for spec in "C3_trendou_8192x8_fuse20|FUSE=20 REPS=8" "C3_trendou_8192x8_fuse1|FUSE=1 REPS=32 AGE=2048" \
              "C3_trendou_8192x8_fuse256|FUSE=256 REPS=4" "C3_trendou_8192x16_fuse64|ASSETS=16 FUSE=64 REPS=6"; do
    n=${spec%%|*}; pr=${spec#*|}
    TAG=${T}_$n LIBS="$n=madigan_amd/libmadigan_hip.so" PROBE="WORKLOAD=C3 $pr" EXTRA_GROUPS="FETCH_SIZE WRITE_SIZE" \
      bash tools/pmc_pass.sh || exit 1
  done
  mkdir -p gpurun_out/$T
  timeout -k 10 600 python -u tools/fuzz_trio.py ${FUZZ_CASES:-120} 29 > gpurun_out/$T/fuzz_trio.txt 2>&1 \
    || { echo "fuzz failed"; tail -20 gpurun_out/$T/fuzz_trio.txt; exit 1; }
  tail -3 gpurun_out/$T/fuzz_trio.txt
  ;;
*)
  echo "PART=A|B|C"; exit 2
  ;;
esac
