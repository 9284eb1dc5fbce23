#!/bin/bash
# instruction-cache behaviour of the step kernel at 1- and 64-step launches
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/icache
rm -rf $O; mkdir -p $O
for f in 1 64; do
  B="python bench.py --steps 128 --warmup 64 --fuse $f --no-cpu-baseline --no-probe --no-k-sweep"
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES SQ_INSTS_VALU --output-format csv -d $O/f$f -o p -- $B > $O/f$f.log 2>&1 || { echo "pmc $f failed"; tail -20 $O/f$f.log; exit 1; }
done
python - <<'PY'
import csv, glob
for f in (1, 64):
    d = {}
    for r in csv.DictReader(open(glob.glob(f"gpurun_out/icache/f{f}/p_counter_collection.csv")[0])):
        if "k_step_trio" not in r["Kernel_Name"]:
            continue
        c = d.setdefault(int(r["Dispatch_Id"]), {})
        c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(d)[-8:]
    avg = {k: sum(d[i].get(k, 0) for i in ids) / len(ids) for k in d[ids[0]]}
    w = avg.get("SQ_WAVES", 1)
    print(f, {k: round(v / w, 2) for k, v in avg.items()}, "per wave; steps", f)
PY
