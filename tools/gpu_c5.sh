#!/bin/bash
# replay parity tests + the C5 bench line (GPU box)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/c5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c5/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/c5/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/c5/pytest_gpu.log
timeout -k 10 300 python bench.py --workload C5 --no-cpu-baseline > gpurun_out/c5/bench.json 2> gpurun_out/c5/bench.err || { tail -20 gpurun_out/c5/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c5/bench.json')); print('C5 %.3e'%d['value'], d['roofline']['avg_launch_us'], d['step_launch_avg_us'])"
