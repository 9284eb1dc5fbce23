#!/bin/bash
# A/B of library variants on the two-role kernel's shapes: 16 TrendOU assets
# (64-step launches) and C5 (16-asset replay, W = 64).  VARIANTS="name=path ..."
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/abd
rm -rf $O; mkdir -p $O
run() {  # name path tag args...
  local name=$1 path=$2 tag=$3; shift 3
  [ "$path" = base ] && path=madigan_amd/libmadigan_hip.so
  MADIGAN_LIB_PATH=$path timeout -k 10 200 python bench.py "$@" --no-cpu-baseline --no-probe > $O/$name.$tag.json 2>> $O/err.log || { echo "fail $name $tag"; tail -5 $O/err.log; exit 1; }
  python -c "import json;d=json.load(open('$O/$name.$tag.json'));print('$name','$tag',d['config'].get('schedule'),round(d.get('kernel_us_per_step', d.get('step_launch_avg_us', 0)),3),'%.4g'%d['value'])"
}
for r in $(seq 1 ${R:-2}); do
  for v in $VARIANTS; do
    name=${v%%=*}; path=${v#*=}
    run $name $path a16.$r --steps 512 --warmup 64 --fuse 64 --assets 16 || exit 1
    run $name $path c5.$r --workload C5 --steps 128 --warmup 64 || exit 1
  done
done
