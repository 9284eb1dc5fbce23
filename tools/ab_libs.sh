#!/bin/bash
# A/B of two library builds on one box: bench lines alternated between the
# product library and LIB_B (MADIGAN_LIB_PATH), ROUNDS times each.
#   TAG=... LIB_B=tools/_var/base/libmadigan_hip.so ARGS="--steps ..." bash tools/ab_libs.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in new base; do
    if [ $v = base ]; then L="MADIGAN_LIB_PATH=$LIB_B"; else L=""; fi
    env $L timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline --no-probe --no-k-sweep > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v $r failed"; tail -20 $O/${v}_$r.err; exit 1; }
    python -c "import json,sys;d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$v $r', 'kernel_us_per_step %.4f'%d.get('kernel_us_per_step', 0), 'launch_us %.2f'%r.get('avg_launch_us', 0), 'value %.4g'%d['value'])"
  done
done
