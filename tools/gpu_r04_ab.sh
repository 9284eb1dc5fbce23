#!/bin/bash
# GPU suite (unless SKIP_TESTS) then an A/B of library variants: 20-step and
# 64-step launches and the one-step launch, R rounds alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab4}
rm -rf $O; mkdir -p $O
PT="python -u -m pytest -v --timeout 180 --timeout-method thread -p no:cacheprovider"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
X=${EXTRA:-}
for r in $(seq 1 ${R:-2}); do
  for v in $VARIANTS; do
    name=${v%%=*}; path=${v#*=}
    [ "$path" = base ] && path=madigan_amd/libmadigan_hip.so
    MADIGAN_LIB_PATH=$path timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe --no-k-sweep $X > $O/$name.$r.20.json 2>> $O/err.log || { echo "fail $name"; tail -5 $O/err.log; exit 1; }
    MADIGAN_LIB_PATH=$path timeout -k 10 120 python bench.py --steps 1024 --warmup 128 --fuse 64 --no-cpu-baseline --no-probe --no-k-sweep $X > $O/$name.$r.64.json 2>> $O/err.log || { echo "fail $name"; tail -5 $O/err.log; exit 1; }
    MADIGAN_LIB_PATH=$path timeout -k 10 120 python bench.py --steps 64 --warmup 8 --fuse 1 --no-cpu-baseline --no-probe --no-k-sweep $X > $O/$name.$r.1.json 2>> $O/err.log || { echo "fail $name"; tail -5 $O/err.log; exit 1; }
    python -c "import json;a=json.load(open('$O/$name.$r.20.json'));b=json.load(open('$O/$name.$r.64.json'));c=json.load(open('$O/$name.$r.1.json'));print('$name', $r, 'k20_us', round(a['roofline']['avg_launch_us'],2), 'k64_us/step', round(b['kernel_us_per_step'],3), 'k1_us', round(c['roofline']['avg_launch_us'],3))"
  done
done
