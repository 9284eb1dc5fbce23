#!/bin/bash
# A/B timing of library variants on one box: VARIANTS="name=path ..." (path
# to a libmadigan_hip.so; "base" = the product library), R rounds alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/ab
rm -rf $O; mkdir -p $O
for r in $(seq 1 ${R:-3}); do
  for v in $VARIANTS; do
    name=${v%%=*}; path=${v#*=}
    [ "$path" = base ] && path=madigan_amd/libmadigan_hip.so
    MADIGAN_LIB_PATH=$path timeout -k 10 200 python bench.py --steps 2048 --warmup 256 --no-cpu-baseline --no-probe > $O/$name.$r.256.json 2>> $O/err.log || { echo "fail $name"; tail -5 $O/err.log; exit 1; }
    MADIGAN_LIB_PATH=$path timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe > $O/$name.$r.20.json 2>> $O/err.log || { echo "fail $name"; tail -5 $O/err.log; exit 1; }
    MADIGAN_LIB_PATH=$path timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --fuse 20 --no-cpu-baseline --no-probe > $O/$name.$r.f20.json 2>> $O/err.log || { echo "fail $name"; tail -5 $O/err.log; exit 1; }
    python -c "import json;a=json.load(open('$O/$name.$r.256.json'));b=json.load(open('$O/$name.$r.20.json'));c=json.load(open('$O/$name.$r.f20.json'));print('$name', $r, 'k256', round(a['kernel_us_per_step'],3), 'drv', round(b['value']/1e9,3), round(b['kernel_us_per_step'],3), 'f20x100', round(c['kernel_us_per_step'],3))"
  done
done
