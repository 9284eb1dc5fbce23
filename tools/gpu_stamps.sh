#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/stamps
rm -rf $O; mkdir -p $O
for f in ${FUSES:-1 20 256}; do
  FUSE=$f MADIGAN_LIB_PATH=tools/_var/stamps/libmadigan_hip.so timeout -k 10 120 python tools/stamps.py >> $O/stamps.json 2>> $O/stamps.err || { echo "stamps failed"; tail -20 $O/stamps.err; exit 1; }
done
cat $O/stamps.json
