#!/bin/bash
# the secondary shapes on the product build: n = 20 DDR, 16 TrendOU assets,
# C2 / C4 / C5 (windowed; 64-step launches), C1
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-shapes}
rm -rf $O; mkdir -p $O
run() {  # tag seconds args...
  local tag=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" --no-cpu-baseline --no-probe --no-k-sweep > $O/$tag.json 2>> $O/err.log || { echo "fail $tag"; tail -5 $O/err.log; exit 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));print('$tag',d['config'].get('schedule'),'kernel_us/step',round(d.get('kernel_us_per_step') or 0,3),'step_launch_us',d.get('step_launch_avg_us'),'value %.4g'%d['value'])"
}
run n20 200 --steps 512 --warmup 64 --fuse 64 --nstep 20
run a16 200 --steps 512 --warmup 64 --fuse 64 --assets 16
run c2 300 --workload C2 --steps 256 --warmup 64
run c4 300 --workload C4 --steps 256 --warmup 64
run c5 400 --workload C5 --steps 256 --warmup 64
