#!/bin/bash
# n-step prefix from the generator role (MGN_NST_GPFX): the n-step / schedule /
# tail GPU tests, then A/B against the build without it
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests -k "nstep or n_step or schedules or tail or nst or Nstep" > gpurun_out/pt_gpfx.log 2>&1
rc=$?; tail -3 gpurun_out/pt_gpfx.log; [ $rc -eq 0 ] || exit 1
VARIANTS="base=base nogpfx=tools/_var/nogpfx/libmadigan_hip.so" SHAPES="n20 C3_20" R=2 TAG=abgpfx bash tools/gpu_r04_ab_gen.sh
