#!/bin/bash
# n-step unit A/B only (against the previous build)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
VARIANTS="prev=tools/_var/prev/libmadigan_hip.so new=base" SHAPES="n20 C3_20 C3_256 k1" R=2 TAG=abnstunit bash tools/gpu_r04_ab_gen.sh
