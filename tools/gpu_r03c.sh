#!/bin/bash
# Round-3: schedules by launch length (K = 1 single / duo / trio), n-step on
# the three-role kernel vs the two-role one, 16 assets; GPU tests touched by
# the trio n-step form.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
PT="python -u -m pytest -v --timeout 180 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT -m gpu tests/test_gpu_parity.py tests/test_gpu_variants.py tests/test_gpu_bench_shapes.py tests/test_gpu_configs.py > $O/pytest.log 2>&1 || echo "tests FAILED (see log)"
tail -2 $O/pytest.log
B="timeout -k 10 120 python bench.py --no-cpu-baseline --no-probe"
for r in 1 2 3; do
  for v in base nopack; do
    path=tools/_var/$v/libmadigan_hip.so; [ $v = base ] && path=madigan_amd/libmadigan_hip.so
    MADIGAN_LIB_PATH=$path $B --steps 20 --warmup 5 > $O/$v.$r.20.json 2>> $O/err.log || { echo "fail $v"; tail -5 $O/err.log; exit 1; }
    MADIGAN_LIB_PATH=$path $B --steps 1024 --warmup 256 > $O/$v.$r.256.json 2>> $O/err.log || { echo "fail $v"; tail -5 $O/err.log; exit 1; }
    python -c "import json;a=json.load(open('$O/$v.$r.256.json'));b=json.load(open('$O/$v.$r.20.json'));print('$v', $r, 'k256', round(a['kernel_us_per_step'],3), 'drv', round(b['value']/1e9,3), round(b['roofline']['avg_launch_us'],2), round(b['roofline']['frac'],4))"
  done
done
for s in trio duo single; do
  $B --steps 64 --warmup 8 --fuse 1 --schedule $s > $O/k1_$s.json 2>> $O/err.log || { echo "fail k1 $s"; tail -5 $O/err.log; exit 1; }
  $B --steps 20 --warmup 5 --schedule $s > $O/k20_$s.json 2>> $O/err.log || { echo "fail k20 $s"; tail -5 $O/err.log; exit 1; }
  python -c "import json;a=json.load(open('$O/k1_$s.json'));b=json.load(open('$O/k20_$s.json'));print('$s', 'k1 us', round(a['kernel_us_per_step'],3), 'k20 launch us', round(b['roofline']['avg_launch_us'],2))"
done
for s in trio duo; do
  for n in 20 5; do
    $B --steps 512 --warmup 64 --fuse 64 --nstep $n --schedule $s > $O/nst${n}_$s.json 2>> $O/err.log || { echo "fail nst $n $s"; tail -5 $O/err.log; exit 1; }
    python -c "import json;a=json.load(open('$O/nst${n}_$s.json'));print('nstep $n $s', round(a['kernel_us_per_step'],3), a['config']['schedule'])"
  done
done
$B --steps 512 --warmup 64 --fuse 64 --assets 16 > $O/a16.json 2>> $O/err.log || { echo "fail a16"; tail -5 $O/err.log; exit 1; }
python -c "import json;a=json.load(open('$O/a16.json'));print('a16', round(a['kernel_us_per_step'],3), a['config']['schedule'])"
for s in trio duo; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt1_$s -o kt -- python bench.py --steps 64 --warmup 8 --fuse 1 --schedule $s --no-cpu-baseline --no-probe > $O/kt1_$s.log 2>&1 || { echo "kt1 $s failed"; tail -20 $O/kt1_$s.log; exit 1; }
done
echo r03c done
