#!/bin/bash
# plain cash chain only in the two-slot (16-asset) unit against the default build
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
MADIGAN_LIB_PATH=tools/_var/plainm2/libmadigan_hip.so timeout -k 10 300 python -u tools/fuzz_trio.py 120 37 > gpurun_out/fuzz_plainm2.log 2>&1 || { tail -5 gpurun_out/fuzz_plainm2.log; exit 1; }
tail -1 gpurun_out/fuzz_plainm2.log
VARIANTS="base=base plainm2=tools/_var/plainm2/libmadigan_hip.so" SHAPES="a16 a16_20 a16 a16_20" R=2 TAG=abplainm2 bash tools/gpu_r04_ab_gen.sh
