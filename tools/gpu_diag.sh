#!/bin/bash
# diagnostics of the C3 step kernel: phase stamps (diagnostic build) + ablations
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/diag
mkdir -p $O
for f in 20 64 256; do
  FUSE=$f MADIGAN_LIB_PATH=tools/_var/stamps/libmadigan_hip.so timeout -k 10 120 python tools/stamps.py >> $O/stamps.json 2>> $O/stamps.err || { echo "stamps failed"; tail -20 $O/stamps.err; exit 1; }
done
cat $O/stamps.json
timeout -k 10 200 python tools/ablate.py > $O/ablate.json 2> $O/ablate.err || { echo "ablate failed"; tail -20 $O/ablate.err; exit 1; }
cat $O/ablate.json
