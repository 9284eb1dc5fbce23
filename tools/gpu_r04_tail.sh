#!/bin/bash
# the tail-reset build: GPU suite, the K = 1 diagnostic, then A/B against the
# build without it (MGN_TRIO_TAILRST=0) at 1-, 16-, 20- and 256-step launches
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests > gpurun_out/pt_tail.log 2>&1
rc=$?; tail -3 gpurun_out/pt_tail.log; [ $rc -le 1 ] || exit 1
[ $rc -eq 0 ] || grep -E "^FAILED|Error" gpurun_out/pt_tail.log | head -5
for v in base notail; do
  L=madigan_amd/libmadigan_hip.so; [ $v = notail ] && L=tools/_var/notail/libmadigan_hip.so
  MADIGAN_LIB_PATH=$L timeout -k 10 200 python tools/k1_diag.py > gpurun_out/k1_diag_$v.json 2> gpurun_out/k1_diag.err || { tail -5 gpurun_out/k1_diag.err; exit 1; }
  echo "k1_diag $v $(cat gpurun_out/k1_diag_$v.json)"
done
VARIANTS="base=base notail=tools/_var/notail/libmadigan_hip.so" SHAPES="k1 k16 C3_20 C3_256" R=2 TAG=abtail bash tools/gpu_r04_ab_gen.sh
