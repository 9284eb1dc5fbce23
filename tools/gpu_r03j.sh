#!/bin/bash
# Round-3 (session 2): dispatch ramp by workgroup shape; K = 1 launch time per
# schedule; the driver line on this build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py -k launcher > $O/launcher_test.txt 2>&1 || { echo "launcher test failed"; tail -30 $O/launcher_test.txt; exit 1; }
tail -2 $O/launcher_test.txt
#timeout -k 10 120 ./tools/_var/dispatch_ramp > $O/ramp.json 2>&1 || { echo "ramp failed"; tail $O/ramp.json; exit 1; }
for s in trio duo single; do
  timeout -k 10 300 python bench.py --gpus 1 --fuse 1 --steps 200 --warmup 20 --schedule $s --no-cpu-baseline --no-probe > $O/k1_$s.json 2> $O/k1_$s.err || { echo "k1 $s failed"; tail -20 $O/k1_$s.err; exit 1; }
  python -c "import json;d=json.load(open('$O/k1_$s.json'));print('k1','$s','%.4g'%d['value'],round(d['ms_per_step']*1e3,2),round(d['roofline']['avg_launch_us'],2))"
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv.json 2> $O/drv.err || { echo "bench failed"; tail -20 $O/drv.err; exit 1; }
python -c "import json;d=json.load(open('$O/drv.json'));print('drv','%.4g'%d['value'],round(d['ms_per_step']*20e3,2),round(d['roofline']['avg_launch_us'],2))"
for f in 1 20; do
  MADIGAN_LIB_PATH=tools/_var/iter/libmadigan_hip.so timeout -k 10 200 python tools/iterstamps.py $f 10 > $O/iter_$f.json 2> $O/iter_$f.err || { echo "iter $f failed"; tail -20 $O/iter_$f.err; exit 1; }
  cat $O/iter_$f.json
done
echo r03j done
