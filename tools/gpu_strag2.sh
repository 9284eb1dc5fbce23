#!/bin/bash
# straggler blocks vs the output set
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/strag2
rm -rf $O; mkdir -p $O
run() {  # tag fields
  STAMPS_FIELDS=$2 STAMPS_RAW=$O/raw_$1.npy FUSE=20 MADIGAN_LIB_PATH=tools/_var/stamps/libmadigan_hip.so timeout -k 10 120 python tools/stamps.py > $O/stamps_$1.json 2>> $O/stamps.err || { echo "stamps $1 failed"; tail -20 $O/stamps.err; exit 1; }
}
run all_a "reward,shaped,done,obs_price,obs_port,timestamp,tprice,tunits,tcost,risk,margin_call"
run reward "reward"
run none ","
run f64 "reward,shaped,obs_price,obs_port,timestamp,tprice,tunits,tcost"
run bytes "done,risk,margin_call"
run all_b "reward,shaped,done,obs_price,obs_port,timestamp,tprice,tunits,tcost,risk,margin_call"
echo strag2 done
