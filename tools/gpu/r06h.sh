N20="--nstep 20 --nstep-pop running --steps 20 --warmup 5 --fuse 20 --no-k-sweep --no-probe"
PLAN=""
for r in 1 2 3; do
for v in head base line earlyz cheap all; do
  if [ $v = base ]; then E=""; else E="MADIGAN_LIB_PATH=tools/_var/$v/libmadigan_hip.so"; fi
  PLAN="$PLAN
${v}_$r|$E|$N20"
done; done
export TAG=r06h PLAN
bash tools/ab_bench.sh
