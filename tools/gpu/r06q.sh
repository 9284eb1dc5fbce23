PLAN=""
for r in 1 2; do
for v in base k1tw64 k1tw64lb5; do
  if [ $v = base ]; then E=""; else E="MADIGAN_LIB_PATH=tools/_var/$v/libmadigan_hip.so"; fi
  for N in 8192 65536 262144; do
    PLAN="$PLAN
${v}_${N}_$r|$E|--fuse 1 --n-envs $N --steps 64 --warmup 16 --no-k-sweep --no-cpu-baseline --no-probe"
  done
done; done
export TAG=r06q PLAN
bash tools/ab_bench.sh
