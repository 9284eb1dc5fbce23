#!/bin/bash
# masked-term cash chain (MGN_SPEC_CHMASK): GPU suite, then A/B at 1-, 20- and 256-step launches
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests > gpurun_out/pt_chm.log 2>&1
rc=$?; tail -3 gpurun_out/pt_chm.log; [ $rc -eq 0 ] || exit 1
VARIANTS="base=base nochmask=tools/_var/nochmask/libmadigan_hip.so" SHAPES="C3_20 C3_256 k1" R=3 TAG=abchm bash tools/gpu_r04_ab_gen.sh
