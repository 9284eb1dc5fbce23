#!/bin/bash
# K = 1 diagnostic (tools/k1_diag.py), then the driver line and the 256-step
# line with the launch-length sweep (fresh actions per launch)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04final
mkdir -p $O
timeout -k 10 200 python tools/k1_diag.py > gpurun_out/k1_diag.json 2> gpurun_out/k1_diag.err || { tail -5 gpurun_out/k1_diag.err; exit 1; }
cat gpurun_out/k1_diag.json
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -5 $O/bench_driver.err; exit 1; }
timeout -k 10 300 python bench.py --steps 2048 --warmup 256 --no-cpu-baseline --sweep > $O/bench_fuse256.json 2> $O/bench_fuse256.err || { tail -5 $O/bench_fuse256.err; exit 1; }
python - <<'EOF'
import json
for f in ("bench_driver", "bench_fuse256"):
    d = json.load(open("gpurun_out/r04final/%s.json" % f))
    print(f, "%.4g" % d["value"], round(d["roofline"]["frac"], 4),
          {k: (round(v["kernel_us_per_launch"], 2), round(v["back_to_back_us_per_step"], 3))
           for k, v in d.get("launch_lengths", {}).items()})
EOF
