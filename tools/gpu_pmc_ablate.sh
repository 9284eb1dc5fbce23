#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/abl
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d $O/p1 -o p -- python tools/ablate_pmc.py > $O/p1.log 2>&1 || { echo "pmc failed"; tail -20 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p2 -o p -- python tools/ablate_pmc.py > $O/p2.log 2>&1 || { echo "pmc2 failed"; tail -20 $O/p2.log; exit 1; }
tail -2 $O/p1.log
