#!/bin/bash
# A/B bench lines on one box: each line of $PLAN is "name|ENV=... ENV2=...|bench args";
# writes gpurun_out/$TAG/<name>.json and prints a summary line per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}; mkdir -p $O
while IFS='|' read -r name envs args; do
  [ -z "$name" ] && continue
  env $envs timeout -k 10 300 python -u bench.py $args --no-cpu-baseline > $O/$name.json 2> $O/$name.err \
    || { echo "$name failed"; tail -20 $O/$name.err; exit 1; }
  python - "$O/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "value %.4g" % d["value"], "kern_us %.2f" % r.get("avg_launch_us", 0), "frac %.3f" % r["frac"],
      "us/step %.4f" % d.get("kernel_us_per_step", 0), "step_us %s" % d.get("step_launch_avg_us"))
PY
done <<< "$PLAN"
echo "$O done"
