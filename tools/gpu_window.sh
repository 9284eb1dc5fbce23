#!/bin/bash
# windowed workloads on the GPU box: parity tests, then the C2/C4/C5 bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/win
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/win/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/win/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/win/pytest_gpu.log
for w in C2 C4 C5; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/win/bench_$w.json 2> gpurun_out/win/bench_$w.err || { echo "bench $w failed"; tail -20 gpurun_out/win/bench_$w.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/win/bench_$w.json')); print('$w', '%.3e'%d['value'], d['roofline']['kernel'], '%.1f us'%d['roofline']['avg_launch_us'], '%.0f GB/s'%d['roofline']['achieved'], 'frac %.3f'%d['roofline']['frac'], 'step launch %.1f us'%d.get('step_launch_avg_us',0), 'K', d['config']['steps_per_launch'], 'eps', d['episodes_completed'])"
done
