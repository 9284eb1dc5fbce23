#!/bin/bash
# Round-3: 16-asset three-role kernel -- parity (schedules bit-identical incl.
# A = 16 / 13 on the trio) and duo vs trio at 8192 x 16, 64-step launches;
# the C5 refill probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03h
mkdir -p $O
PT="python -u -m pytest -v --timeout 180 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT -m gpu tests/test_gpu_parity.py -k "schedules_bit_identical" > $O/pytest.log 2>&1 || { echo "tests FAILED"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="python bench.py --steps 512 --warmup 64 --fuse 64 --assets 16 --no-cpu-baseline --no-probe"
for r in 1 2; do
  for s in duo trio; do
    timeout -k 10 300 $B --schedule $s > $O/a16_$s.$r.json 2> $O/a16_$s.$r.err || { echo "bench $s failed"; tail -20 $O/a16_$s.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/a16_$s.$r.json'));print('$s',$r,d['config']['schedule'],round(d['kernel_us_per_step'],3))"
  done
done
timeout -k 10 400 python tools/c5_probe.py > $O/c5_probe.log 2>&1 || { echo "probe failed"; tail -20 $O/c5_probe.log; exit 1; }
grep -v "^{" $O/c5_probe.log
echo r03h done
