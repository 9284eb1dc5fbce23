#!/bin/bash
# per-block wall stamps (raw, with HW_ID / XCC_ID) of the diagnostic build
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/strag
rm -rf $O; mkdir -p $O
for F in ${FUSES:-1 20 64}; do
  STAMPS_RAW=$O/raw_$F.npy FUSE=$F MADIGAN_LIB_PATH=tools/_var/stamps/libmadigan_hip.so timeout -k 10 120 python tools/stamps.py > $O/stamps_$F.json 2>> $O/stamps.err || { echo "stamps failed"; tail -20 $O/stamps.err; exit 1; }
  cat $O/stamps_$F.json
done
echo strag done
