PLAN=""
for r in 1 2 3; do
for v in base gprio2 gprio3; do
  if [ $v = base ]; then E=""; else E="MADIGAN_LIB_PATH=tools/_var/$v/libmadigan_hip.so"; fi
  PLAN="$PLAN
${v}_k1_$r|$E|--fuse 1 --steps 64 --warmup 16 --no-k-sweep --no-cpu-baseline --no-probe"
done; done
export TAG=r06t PLAN
bash tools/ab_bench.sh
