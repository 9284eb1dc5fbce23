#!/bin/bash
# A/B timing of library variants on a windowed workload: WL=C4 VARIANTS="name=path ..."
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/abw
mkdir -p $O
for r in $(seq 1 ${R:-3}); do
  for wl in ${WL:-C4}; do
  for v in $VARIANTS; do
    name=${v%%=*}; path=${v#*=}
    [ "$path" = base ] && path=madigan_amd/libmadigan_hip.so
    extra=""; case "$name" in duo|trio|single) extra="--schedule $name";; esac
    MADIGAN_LIB_PATH=$path timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline $extra > $O/$wl.$name.$r.json 2>> $O/err.log || { echo "fail $name"; tail -5 $O/err.log; exit 1; }
    python -c "import json;a=json.load(open('$O/$wl.$name.$r.json'));print('$wl', '$name', $r, 'value', round(a['value']/1e6,1), 'step_us', round(a['step_launch_avg_us'],1), 'gather_us', round(a['roofline']['avg_launch_us'],1), 'episodes', a['episodes_completed'])"
  done
  done
done
