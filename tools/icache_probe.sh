set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05s_icache; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -i "icache\|IFETCH" $O/avail.txt | head -20
for spec in "n20|NSTEP=20 FUSE=64 REPS=6" "c3f20|FUSE=20 REPS=8"; do
  n=${spec%%|*}; pr=${spec#*|}
  env WORKLOAD=C3 $pr timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAVES --output-format csv -d $O/$n -o p -- python3 tools/pmc_probe.py > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
done
echo done
