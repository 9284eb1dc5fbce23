#!/bin/bash
# Round-4 first pass: the GPU suite on the current build, then the baseline
# figures this box gives for the one-, 20- and 256-step launches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
PT="python -u -m pytest -v --timeout 180 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
run() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));r=d.get('roofline',{});print('$n', '%.4g'%d['value'], 'frac', r.get('frac'), 'launch_us', r.get('avg_launch_us'), 'us/step', d.get('kernel_us_per_step'))"
}
run drv 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
run k1 300 python bench.py --steps 64 --warmup 8 --fuse 1 --no-cpu-baseline --no-probe
run k256 300 python bench.py --steps 2048 --warmup 256 --no-cpu-baseline --no-probe --sweep
python -c "import json;d=json.load(open('$O/k256.json'));print({k:round(v['us_per_step'],3) for k,v in d['fusion_sweep'].items()})"
echo r04a done
