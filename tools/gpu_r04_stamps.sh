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
# the secondary shapes (64-step launches): 16 TrendOU assets, n = 20 DDR, C4, C5
if [ -n "$SHAPES" ]; then
  for spec in "C3 16 1" "C3 8 20" "C4 8 1" "C5 16 1"; do
    set -- $spec
    WORKLOAD=$1 ASSETS=$2 NSTEP=$3 FUSE=64 MADIGAN_LIB_PATH=tools/_var/stamps/libmadigan_hip.so timeout -k 10 200 python tools/stamps_trio.py > $O/st_$1_$2_$3.json 2>> $O/st.err || { echo "stamps $spec failed"; tail -20 $O/st.err; exit 1; }
    cat $O/st_$1_$2_$3.json
  done
fi
