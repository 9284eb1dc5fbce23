#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/strag3
rm -rf $O; mkdir -p $O
for v in stamps stampsnt stamps stampsnt; do
  STAMPS_RAW=$O/raw_$v.$RANDOM.npy FUSE=20 MADIGAN_LIB_PATH=tools/_var/$v/libmadigan_hip.so timeout -k 10 120 python tools/stamps.py >> $O/stamps_$v.json 2>> $O/stamps.err || { echo "stamps $v failed"; tail -20 $O/stamps.err; exit 1; }
done
VARIANTS="base=base nt=tools/_var/nt/libmadigan_hip.so" R=3 bash tools/ab.sh
