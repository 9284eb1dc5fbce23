#!/bin/bash
# PMC passes of tools/pmc_probe.py, one rocprofv3 run per counter group and
# per library (each within the per-block counter limits; no trace domains):
#   TAG=x LIBS="base=madigan_amd/libmadigan_hip.so ablL=tools/_var/ablL/libmadigan_hip.so" \
#   PROBE="WORKLOAD=C3 FUSE=20 REPS=8" bash tools/pmc_pass.sh
# then: python tools/pmc_brief.py gpurun_out/pmc_x
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/pmc_${TAG:-pass}
mkdir -p $O
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT"
# SQ=0: only the EXTRA_GROUPS passes (e.g. EXTRA_GROUPS="FETCH_SIZE WRITE_SIZE",
# one counter per pass: HBM traffic, MI355X_MICROARCH.md's HBM section)
GS=()
if [ "${SQ:-1}" = 1 ]; then GS+=("$G1" "$G2"); fi
for x in ${EXTRA_GROUPS}; do GS+=("$x"); done
for lv in ${LIBS:-base=madigan_amd/libmadigan_hip.so}; do
  n=${lv%%=*}; lib=${lv#*=}
  gi=0
  for grp in "${GS[@]}"; do
    gi=$((gi + 1))
    env $PROBE MADIGAN_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv \
      -d $O/$n/g$gi -o p -- python3 tools/pmc_probe.py > $O/${n}_g$gi.log 2>&1 \
      || { echo "pmc $n g$gi failed"; tail -20 $O/${n}_g$gi.log; exit 1; }
  done
done
python tools/pmc_brief.py $O ${UPDATE:+--update} --json $O/brief.json
