#!/bin/bash
# per-role cycles of the three-role kernel (diagnostic build -DMGN_STAMPS)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/stamps
mkdir -p $O
for f in ${FUSES:-64}; do
  FUSE=$f MADIGAN_LIB_PATH=tools/_var/stamps/libmadigan_hip.so timeout -k 10 120 python tools/stamps_trio.py > $O/st_$f.json 2>> $O/st.err || { echo "stamps failed"; tail -20 $O/st.err; exit 1; }
  cat $O/st_$f.json
done
