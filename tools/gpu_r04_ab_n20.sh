#!/bin/bash
# A/B of library variants on the n = 20 DDR C3 shape (64-step launches)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abn20}
rm -rf $O; mkdir -p $O
for r in $(seq 1 ${R:-2}); do
  for v in $VARIANTS; do
    name=${v%%=*}; path=${v#*=}
    [ "$path" = base ] && path=madigan_amd/libmadigan_hip.so
    MADIGAN_LIB_PATH=$path timeout -k 10 200 python bench.py --steps 512 --warmup 64 --fuse 64 --nstep 20 --no-cpu-baseline --no-probe --no-k-sweep > $O/$name.$r.json 2>> $O/err.log || { echo "fail $name"; tail -5 $O/err.log; exit 1; }
    python -c "import json;d=json.load(open('$O/$name.$r.json'));print('$name', $r, 'n20 us/step', round(d['kernel_us_per_step'],3))"
  done
done
