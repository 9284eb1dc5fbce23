#!/bin/bash
# s_memtime timeline of the three-role kernel (diagnostic build -DMGN_ITERSTAMP)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/iter
mkdir -p $O
for f in ${FUSES:-1 20}; do
  MADIGAN_LIB_PATH=${LIB:-tools/_var/iter/libmadigan_hip.so} timeout -k 10 120 python tools/iterstamps.py $f 20 > $O/iter_$f.json 2>> $O/iter.err || { echo "iter $f failed"; tail -20 $O/iter.err; exit 1; }
  cat $O/iter_$f.json
done
