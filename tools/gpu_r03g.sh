#!/bin/bash
# Round-3: per-iteration timeline of the three-role kernel (diagnostic build),
# early write-back A/B (five alternating rounds).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
MADIGAN_LIB_PATH=tools/_var/iter/libmadigan_hip.so timeout -k 10 120 python tools/iterstamps.py 20 10 > $O/iter20.json 2> $O/iter.err || { echo "iter20 failed"; tail -20 $O/iter.err; exit 1; }
cat $O/iter20.json
MADIGAN_LIB_PATH=tools/_var/iter/libmadigan_hip.so timeout -k 10 120 python tools/iterstamps.py 1 20 > $O/iter1.json 2>> $O/iter.err || { echo "iter1 failed"; tail -20 $O/iter.err; exit 1; }
cat $O/iter1.json
B="timeout -k 10 120 python bench.py --no-cpu-baseline --no-probe"
for r in 1 2 3 4 5; do
  for v in base early0; do
    path=tools/_var/$v/libmadigan_hip.so; [ $v = base ] && path=madigan_amd/libmadigan_hip.so
    MADIGAN_LIB_PATH=$path $B --steps 20 --warmup 5 > $O/$v.$r.20.json 2>> $O/err.log || { echo "fail $v"; tail -5 $O/err.log; exit 1; }
    python -c "import json;b=json.load(open('$O/$v.$r.20.json'));print('$v', $r, 'drv', round(b['value']/1e9,3), round(b['roofline']['avg_launch_us'],2), round(b['roofline']['frac'],4))"
  done
done
echo r03g done
