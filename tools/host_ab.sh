#!/bin/bash
# The driver's timed region (one 20-step launch, --steps 20 --warmup 5) under
# runtime settings, alternated ROUNDS times on one box: ms_per_step x 20 is the
# region, roofline.avg_launch_us the kernel by its launch events.
#   TAG=x VARIANTS="base|;devkarg|HIP_FORCE_DEV_KERNARG=1;marker|--timing marker" bash tools/host_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-hostab}
mkdir -p $O
IFS=';' read -ra VS <<< "$VARIANTS"
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in "${VS[@]}"; do
    n=${v%%|*}; a=${v#*|}
    envs=""; args=""
    for w in $a; do case $w in *=*) envs="$envs $w";; *) args="$args $w";; esac; done
    env $envs timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-probe --no-k-sweep $args \
      > $O/${n}_$r.json 2> $O/${n}_$r.err || { echo "$n $r failed"; tail -5 $O/${n}_$r.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/${n}_$r.json').read().strip().splitlines()[-1]);print('$n $r region_us %.2f kernel_us %.2f' % (d['ms_per_step']*1e3*d['steps'], d['roofline']['avg_launch_us']))"
  done
done
