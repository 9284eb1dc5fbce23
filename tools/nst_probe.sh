#!/bin/bash
# n-step (n = 20 DDR, C3 8192 x 8, 64-step launches) diagnostics on one box:
# per-role stamps of the diagnostic build, then bench lines alternated between
# the product library and the ablation / candidate builds named in VARS
# ("name=path;name=path").  TAG names gpurun_out/<TAG>.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-nstprobe}
mkdir -p $O
ARGS=${ARGS:-"--nstep 20 --steps 512 --warmup 64 --fuse 64"}
if [ -n "$STAMPS" ]; then
  for s in $STAMPS; do
    n=${s%%=*}; lib=${s#*=}
    MADIGAN_LIB_PATH=$lib NSTEP=${NSTEP:-20} FUSE=64 timeout -k 10 200 python tools/stamps_trio.py > $O/stamps_$n.json 2> $O/stamps_$n.err \
      || { echo "stamps $n failed"; tail -5 $O/stamps_$n.err; exit 1; }
    echo "stamps $n: $(tail -1 $O/stamps_$n.json)"
  done
fi
IFS=';' read -ra VS <<< "$VARS"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "base=" "${VS[@]}"; do
    n=${v%%=*}; lib=${v#*=}
    if [ -n "$lib" ]; then L="MADIGAN_LIB_PATH=$lib"; else L=""; fi
    env $L timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline --no-probe --no-k-sweep > $O/${n}_$r.json 2> $O/${n}_$r.err \
      || { echo "$n $r failed"; tail -20 $O/${n}_$r.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/${n}_$r.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$n $r', 'us/step %.4f'%d.get('kernel_us_per_step', 0), 'launch_us %.2f'%r.get('avg_launch_us', 0), 'step_launch_us %.2f'%d.get('step_launch_avg_us', 0), 'value %.4g'%d['value'])"
  done
done
echo "$O done"
