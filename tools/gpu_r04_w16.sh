#!/bin/bash
# 16 OU assets with a W = 64 window (bench.py --workload C2 --win-assets 16,
# 8192 envs, 64-step launches): the two-role kernel, the automatic schedule
# (the two-slot three-role kernel) and the one-slot three-role kernel
# (m1_16 variant); then the K = 1 / 20 iteration timelines (MGN_ITERSTAMP build)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/w16
mkdir -p $O
for r in 1 2; do
  for v in "duo base" "auto base" "trio tools/_var/m1_16/libmadigan_hip.so"; do
    set -- $v
    L=$2; [ "$L" = base ] && L=madigan_amd/libmadigan_hip.so
    MADIGAN_LIB_PATH=$L timeout -k 10 300 python bench.py --workload C2 --win-assets 16 --steps 256 --warmup 64 \
      --no-cpu-baseline --no-probe --no-k-sweep --schedule $1 > $O/w16_$1_$r.json 2>> $O/w16.err || { tail -5 $O/w16.err; exit 1; }
    python -c "import json;d=json.load(open('$O/w16_$1_$r.json'));print('w16', '$1', '${2: -16}', $r, d['config']['schedule'], 'step_launch_us', round(d['step_launch_avg_us'],1), 'value %.4g' % d['value'])"
  done
done
FUSES="${FUSES:-1 20}" bash tools/gpu_r04_iter.sh
