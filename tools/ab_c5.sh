#!/bin/bash
# C5 (16-asset replay, W = 64) on the two- and three-role kernels, and the
# 16-asset replay rollout without window (64-step launches).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/abc5
rm -rf $O; mkdir -p $O
for r in $(seq 1 ${R:-2}); do
  for s in duo trio; do
    timeout -k 10 300 python bench.py --workload C5 --steps 256 --warmup 64 --no-cpu-baseline --no-probe --schedule $s > $O/c5.$s.$r.json 2>> $O/err.log || { echo "fail c5 $s"; tail -5 $O/err.log; exit 1; }
    python -c "import json;d=json.load(open('$O/c5.$s.$r.json'));print('c5','$s',$r,d['config']['schedule'],round(d['step_launch_avg_us'],1),round(d['roofline']['avg_launch_us'],1),'%.4g'%d['value'],'view','%.4g'%d.get('view_mode',{}).get('value',0),'eps',d['episodes_completed'])"
  done
done
