W="--steps 128 --warmup 64 --no-cpu-baseline"
PLAN=""
for wl in "R1_64k|--workload R1 --n-envs 65536" "R1_8k|--workload R1 --n-envs 8192" "C2|--workload C2" "C4|--workload C4" "C5|--workload C5"; do
  n=${wl%%|*}; a=${wl#*|}
  for ks in 16 32 64; do
    PLAN="$PLAN
${n}_ks$ks|MGN_GATHER_KS=$ks|$a $W
${n}_ks${ks}_kmaj|MGN_GATHER_KS=$ks MGN_GATHER_KMAJOR=1|$a $W"
  done
done
export TAG=r06n PLAN
bash tools/ab_bench.sh
