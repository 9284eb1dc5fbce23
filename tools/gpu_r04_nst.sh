#!/bin/bash
# GPU suite on the current build, per-role stamps of the secondary shapes,
# then the n = 20 DDR step against the finish role's n-step ablation builds
# (MGN_NST_ABL_{TERM,SUM,ROW}: no summand arithmetic / no ordered sum / no
# zero row entries; outputs wrong, timing only)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests > gpurun_out/pt_full.log 2>&1
rc=$?; tail -3 gpurun_out/pt_full.log; [ $rc -le 1 ] || exit 1
SHAPES=1 FUSES=64 bash tools/gpu_r04_stamps.sh || exit 1
VARIANTS="base=base term=tools/_var/nst_TERM/libmadigan_hip.so sum=tools/_var/nst_SUM/libmadigan_hip.so row=tools/_var/nst_ROW/libmadigan_hip.so" SHAPES="n20" R=2 TAG=abnst bash tools/gpu_r04_ab_gen.sh
