#!/bin/bash
# host-overhead matrix around the driver-shape launch (tools/host_overhead2.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/host
timeout -k 10 120 python tools/host_overhead2.py > gpurun_out/host/default.json 2> gpurun_out/host/default.err || exit $?
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python tools/host_overhead2.py > gpurun_out/host/devka1.json 2> gpurun_out/host/devka1.err || exit $?
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 python tools/host_overhead2.py > gpurun_out/host/devka0.json 2> gpurun_out/host/devka0.err || exit $?
python - <<'PY'
import json
for t in ("default", "devka1", "devka0"):
    d = json.load(open(f"gpurun_out/host/{t}.json"))
    print(t, {k: ({kk: round(vv, 1) for kk, vv in v.items()} if isinstance(v, dict) and k != "env" else v) for k, v in d.items()})
PY
