#!/bin/bash
# A/B of library variants on C4 (Composite, window) and C2 step launches
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abc4}
rm -rf $O; mkdir -p $O
for r in $(seq 1 ${R:-2}); do
  for v in $VARIANTS; do
    name=${v%%=*}; path=${v#*=}
    [ "$path" = base ] && path=madigan_amd/libmadigan_hip.so
    for w in ${WLS:-C4}; do
      MADIGAN_LIB_PATH=$path timeout -k 10 300 python bench.py --workload $w --steps 256 --warmup 64 --no-cpu-baseline --no-probe --no-k-sweep > $O/$name.$r.$w.json 2>> $O/err.log || { echo "fail $name $w"; tail -5 $O/err.log; exit 1; }
      python -c "import json;d=json.load(open('$O/$name.$r.$w.json'));print('$name', $r, '$w', 'step_launch_us', round(d['step_launch_avg_us'],1), 'value %.4g' % d['value'])"
    done
  done
done
