#!/bin/bash
# A/B of library variants over named bench shapes.
#   VARIANTS="base=base head=tools/_var/head/libmadigan_hip.so" SHAPES="C3_20 a16 C5" R=2 bash tools/gpu_r04_ab_gen.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abgen}
rm -rf $O; mkdir -p $O
args_of() {
  case $1 in
    C3_20) echo "--fuse 20 --steps 2000 --warmup 200" ;;
    k1) echo "--fuse 1 --steps 512 --warmup 64" ;;
    k16) echo "--fuse 16 --steps 1024 --warmup 64" ;;
    C3_256) echo "--fuse 256 --steps 2048 --warmup 256" ;;
    a16) echo "--assets 16 --fuse 64 --steps 512 --warmup 64" ;;
    a16_20) echo "--assets 16 --fuse 20 --steps 500 --warmup 60" ;;
    C5) echo "--workload C5 --steps 256 --warmup 64" ;;
    C4) echo "--workload C4 --steps 256 --warmup 64" ;;
    C2) echo "--workload C2 --steps 256 --warmup 64" ;;
    n20) echo "--nstep 20 --fuse 64 --steps 512 --warmup 64" ;;
    *) echo "unknown shape $1" >&2; return 1 ;;
  esac
}
for r in $(seq 1 ${R:-2}); do
  for sh in $SHAPES; do
    a=$(args_of $sh) || exit 1
    for v in $VARIANTS; do
      name=${v%%=*}; path=${v#*=}
      [ "$path" = base ] && path=madigan_amd/libmadigan_hip.so
      MADIGAN_LIB_PATH=$path timeout -k 10 300 python bench.py $a --no-cpu-baseline --no-probe --no-k-sweep > $O/$name.$r.$sh.json 2>> $O/err.log || { echo "fail $name $sh"; tail -5 $O/err.log; exit 1; }
      python -c "
import json;d=json.load(open('$O/$name.$r.$sh.json'))
print('$sh', '$name', $r, 'us/step', round(d.get('kernel_us_per_step') or 0, 3), 'launch_us', round(d.get('step_launch_avg_us') or 0, 1), 'value %.4g' % d['value'])"
    done
  done
done
