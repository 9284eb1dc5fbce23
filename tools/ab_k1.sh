#!/bin/bash
# K = 1 launch time (avg_launch_us, launch events) per library variant.
# VARIANTS="name=path ..."; R rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/abk1
rm -rf $O; mkdir -p $O
for r in $(seq 1 ${R:-2}); do
  for v in $VARIANTS; do
    name=${v%%=*}; path=${v#*=}
    [ "$path" = base ] && path=madigan_amd/libmadigan_hip.so
    MADIGAN_LIB_PATH=$path timeout -k 10 120 python bench.py --steps 64 --warmup 8 --fuse 1 --no-cpu-baseline --no-probe > $O/$name.$r.json 2>> $O/err.log || { echo "fail $name"; tail -5 $O/err.log; exit 1; }
    python -c "import json;d=json.load(open('$O/$name.$r.json'));print('k1','$name',$r,round(d['roofline']['avg_launch_us'],2))"
  done
done
