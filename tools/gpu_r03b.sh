#!/bin/bash
# Round-3: the drop-in Broker / Portfolio GPU tests, then fixed-cost
# ablations of the three-role kernel (diagnostic builds) at the driver shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
PT="python -u -m pytest -v --timeout 180 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PT -m gpu tests/test_gpu_broker.py tests/test_abi.py tests/test_gpu_bench_shapes.py tests/test_gpu_window_view.py tests/test_gpu_configs.py::test_stats_allgather_rccl_single_rank > $O/pytest_broker.log 2>&1 || echo "broker tests FAILED (see log)"
tail -2 $O/pytest_broker.log
for r in 1 2; do
  for v in base xnt nostore ablEpi ablPro; do
    path=tools/_var/$v/libmadigan_hip.so; [ $v = base ] && path=madigan_amd/libmadigan_hip.so
    MADIGAN_LIB_PATH=$path timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe > $O/$v.$r.20.json 2>> $O/err.log || { echo "fail $v"; tail -5 $O/err.log; exit 1; }
    MADIGAN_LIB_PATH=$path timeout -k 10 120 python bench.py --steps 1024 --warmup 256 --no-cpu-baseline --no-probe > $O/$v.$r.256.json 2>> $O/err.log || { echo "fail $v"; tail -5 $O/err.log; exit 1; }
    MADIGAN_LIB_PATH=$path timeout -k 10 120 python bench.py --steps 64 --warmup 8 --fuse 1 --no-cpu-baseline --no-probe > $O/$v.$r.1.json 2>> $O/err.log || { echo "fail $v"; tail -5 $O/err.log; exit 1; }
    python -c "import json;a=json.load(open('$O/$v.$r.256.json'));b=json.load(open('$O/$v.$r.20.json'));c=json.load(open('$O/$v.$r.1.json'));print('$v', $r, 'k256', round(a['kernel_us_per_step'],3), 'drv', round(b['value']/1e9,3), round(b['roofline']['avg_launch_us'],2), 'k1', round(c['kernel_us_per_step'],3))"
  done
done
for t in launch marker; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe --timing $t > $O/timing_$t.json 2>> $O/err.log || { echo "fail timing $t"; tail -5 $O/err.log; exit 1; }
  python -c "import json;b=json.load(open('$O/timing_$t.json'));print('timing $t', round(b['value']/1e9,3), round(b['roofline']['avg_launch_us'],2), round(b['roofline']['frac'],4))"
done
for v in base xnt; do
  path=tools/_var/$v/libmadigan_hip.so; [ $v = base ] && path=madigan_amd/libmadigan_hip.so
  MADIGAN_LIB_PATH=$path timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o kt -- python bench.py --steps 64 --warmup 8 --fuse 1 --no-cpu-baseline --no-probe > $O/kt_$v.log 2>&1 || { echo "kt failed"; tail -20 $O/kt_$v.log; exit 1; }
  MADIGAN_LIB_PATH=$path timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt20_$v -o kt -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe > $O/kt20_$v.log 2>&1 || { echo "kt20 failed"; tail -20 $O/kt20_$v.log; exit 1; }
done
echo r03b done
