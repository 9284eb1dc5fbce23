#!/bin/bash
# plain cash chain (MGN_SPEC_PLAIN): GPU suite, equivalence fuzz, A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests > gpurun_out/pt_plain.log 2>&1
rc=$?; tail -3 gpurun_out/pt_plain.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/fuzz_trio.py 120 31 > gpurun_out/fuzz_plain.log 2>&1 || { tail -5 gpurun_out/fuzz_plain.log; exit 1; }
tail -1 gpurun_out/fuzz_plain.log
VARIANTS="base=base noplain=tools/_var/noplain/libmadigan_hip.so" SHAPES="C3_20 C3_256 a16 C5 k1" R=2 TAG=abplain bash tools/gpu_r04_ab_gen.sh
