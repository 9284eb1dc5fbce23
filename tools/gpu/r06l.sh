W="--steps 128 --warmup 64"
PLAN=""
for r in 1 2; do
for wl in "R1_64k|--workload R1 --n-envs 65536" "R1_8k|--workload R1 --n-envs 8192" "C2|--workload C2" "C4|--workload C4" "C5|--workload C5"; do
  n=${wl%%|*}; a=${wl#*|}
  PLAN="$PLAN
${n}_env_$r||$a $W --no-cpu-baseline
${n}_kmaj_$r|MGN_GATHER_KMAJOR=1|$a $W --no-cpu-baseline"
done; done
export TAG=r06l PLAN
bash tools/ab_bench.sh
