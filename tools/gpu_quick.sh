#!/bin/bash
# quick GPU iteration: parity subset, driver-shape + long bench, phase stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/quick
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread -p no:cacheprovider ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_configs.py} > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest fatal rc=$rc"; exit $rc; fi
if grep -q "Timeout" $O/pytest.log; then echo "pytest timeout"; exit 124; fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20.json 2> $O/bench20.err || { echo "bench failed"; tail -30 $O/bench20.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench20.json'));print('bench20', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['kernel_us_per_step'])"
timeout -k 10 300 python bench.py --steps 2048 --warmup 256 --no-cpu-baseline --no-probe --sweep > $O/bench256.json 2> $O/bench256.err || { echo "bench256 failed"; tail -30 $O/bench256.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench256.json'));print('bench256', d['value'], d['kernel_us_per_step'], {k:round(v['us_per_step'],3) for k,v in d['fusion_sweep'].items()})"
FUSE=64 MADIGAN_LIB_PATH=tools/_var/stamps/libmadigan_hip.so timeout -k 10 120 python tools/stamps.py > $O/stamps.json 2>> $O/stamps.err || { echo "stamps failed"; tail -20 $O/stamps.err; exit 1; }
cat $O/stamps.json
