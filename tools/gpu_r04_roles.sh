#!/bin/bash
# PMC instruction counts of the three-role kernel: product build and the
# role-ablation builds (64-step launches at 8192 x 8)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/roles
rm -rf $O; mkdir -p $O
B="python bench.py --steps 256 --warmup 64 --fuse 64 --no-cpu-baseline --no-probe --no-k-sweep"
for v in base ablG ablL ablF; do
  lib=tools/_var/$v/libmadigan_hip.so
  [ $v = base ] && lib=madigan_amd/libmadigan_hip.so
  MADIGAN_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/$v -o p -- $B > $O/$v.log 2>&1 || { echo "pmc $v failed"; tail -20 $O/$v.log; exit 1; }
done
for v in base ablG ablL ablF; do mv $O/$v/*/p_counter_collection.csv $O/$v/ 2>/dev/null; done
python tools/pmc_roles.py $O 64
