#!/bin/bash
# round-end pass on the GPU box: parity + smoke + headline bench, the windowed
# profiles, the fusion sweep and the C1 latency line; stops at the first failure
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
bash tools/gpu_check.sh || exit 1
bash tools/prof_window.sh || exit 1
mkdir -p gpurun_out/extra
timeout -k 10 300 python bench.py --sweep --no-cpu-baseline > gpurun_out/extra/sweep.json 2> gpurun_out/extra/sweep.err || { tail -20 gpurun_out/extra/sweep.err; exit 1; }
timeout -k 10 300 python bench.py --workload C1 > gpurun_out/extra/c1.json 2> gpurun_out/extra/c1.err || { tail -20 gpurun_out/extra/c1.err; exit 1; }
cat gpurun_out/extra/c1.json
