#!/bin/bash
# Round-3: host overhead of the driver's timed region (ctypes vs the CPython
# binding, timing modes, interrupt vs polled completion waits), then the
# driver line itself.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 300 python tools/host_overhead.py > $O/host_default.log 2>&1 || { echo "probe failed"; tail -20 $O/host_default.log; exit 1; }
grep -v "^{" $O/host_default.log | grep -v amdgpu.ids
HSA_ENABLE_INTERRUPT=0 timeout -k 10 300 python tools/host_overhead.py > $O/host_poll.log 2>&1 || { echo "probe (poll) failed"; tail -20 $O/host_poll.log; exit 1; }
grep -v "^{" $O/host_poll.log | grep -v amdgpu.ids
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv.$r.json 2> $O/drv.$r.err || { echo "bench failed"; tail -20 $O/drv.$r.err; exit 1; }
  python -c "import json;d=json.load(open('$O/drv.$r.json'));print('drv',$r,'%.4g'%d['value'],round(d['ms_per_step']*20e3,2),round(d['roofline']['avg_launch_us'],2))"
done
echo r03i done
