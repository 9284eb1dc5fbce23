#!/bin/bash
# Round-3: parity after the unified n-step pops; build-placement and early write-back A/B.
# write-back A/B at the driver shape; n-step (n = 20, 5) timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
PT="python -u -m pytest -v --timeout 180 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_bench_shapes.py tests/test_gpu_variants.py > $O/pytest.log 2>&1 || echo "tests FAILED (see log)"
tail -2 $O/pytest.log
B="timeout -k 10 120 python bench.py --no-cpu-baseline --no-probe"
for r in 1 2 3; do
  for v in base same early0; do
    path=tools/_var/$v/libmadigan_hip.so; [ $v = base ] && path=madigan_amd/libmadigan_hip.so
    MADIGAN_LIB_PATH=$path $B --steps 20 --warmup 5 > $O/$v.$r.20.json 2>> $O/err.log || { echo "fail $v"; tail -5 $O/err.log; exit 1; }
    MADIGAN_LIB_PATH=$path $B --steps 64 --warmup 8 --fuse 1 > $O/$v.$r.1.json 2>> $O/err.log || { echo "fail $v"; tail -5 $O/err.log; exit 1; }
    python -c "import json;a=json.load(open('$O/$v.$r.1.json'));b=json.load(open('$O/$v.$r.20.json'));print('$v', $r, 'k1', round(a['kernel_us_per_step'],3), 'drv', round(b['value']/1e9,3), round(b['roofline']['avg_launch_us'],2), round(b['roofline']['frac'],4))"
  done
done
for v in base; do
  path=tools/_var/$v/libmadigan_hip.so; [ $v = base ] && path=madigan_amd/libmadigan_hip.so
  for n in 20 5; do
    MADIGAN_LIB_PATH=$path $B --steps 512 --warmup 64 --fuse 64 --nstep $n > $O/nst${n}_$v.json 2>> $O/err.log || { echo "fail nst $v"; tail -5 $O/err.log; exit 1; }
    python -c "import json;a=json.load(open('$O/nst${n}_$v.json'));print('nst$n $v', round(a['kernel_us_per_step'],3), a['config']['schedule'])"
  done
done
echo r03e done
