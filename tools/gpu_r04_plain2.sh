#!/bin/bash
# plain cash chain, single walk (MGN_SPEC_PLAIN=1 variant) against the default build
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
MADIGAN_LIB_PATH=tools/_var/plain1/libmadigan_hip.so timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests -k "parity or configs or bench_shapes or replay" > gpurun_out/pt_plain2.log 2>&1
rc=$?; tail -3 gpurun_out/pt_plain2.log; [ $rc -eq 0 ] || exit 1
VARIANTS="base=base plain1=tools/_var/plain1/libmadigan_hip.so" SHAPES="C3_20 C3_256 a16 C5 k1" R=2 TAG=abplain2 bash tools/gpu_r04_ab_gen.sh
