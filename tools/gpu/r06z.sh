N20="--nstep 20 --nstep-pop running --steps 20 --warmup 5 --fuse 20 --no-k-sweep --no-probe --no-cpu-baseline"
PLAN=""
for r in 1 2 3; do
for v in head pairs; do
  PLAN="$PLAN
${v}_$r|MADIGAN_LIB_PATH=tools/_var/$v/libmadigan_hip.so|$N20"
done; done
export TAG=r06z PLAN
bash tools/ab_bench.sh
