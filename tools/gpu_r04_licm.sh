#!/bin/bash
# machine LICM off in the APAD 4 / 8 units against the default build
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
VARIANTS="base=base licm=tools/_var/licm/libmadigan_hip.so" SHAPES="C3_20 C3_256 k1 C4 n20" R=2 TAG=ablicm bash tools/gpu_r04_ab_gen.sh
