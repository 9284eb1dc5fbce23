#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/wallx
rm -rf $O; mkdir -p $O
W="timeout -k 10 120 env MADIGAN_LIB_PATH=tools/_var/wallx/libmadigan_hip.so"
run() { $W "$@" || { echo "wallx failed $*"; exit 1; }; }
run FUSE=20 python tools/wallx.py $O/all20.npz
run FUSE=20 FIELDS=reward python tools/wallx.py $O/rew20.npz
run FUSE=20 N=4096 python tools/wallx.py $O/all20_n4096.npz
run FUSE=20 N=2048 python tools/wallx.py $O/all20_n2048.npz
run FUSE=1 LAUNCHES=50 python tools/wallx.py $O/all1.npz
run FUSE=64 LAUNCHES=10 python tools/wallx.py $O/all64.npz
timeout -k 10 120 python bench.py --steps 2000 --warmup 100 --fuse 20 --no-cpu-baseline --no-probe > $O/prod_f20.json && python -c "import json;print('product f20', json.load(open('$O/prod_f20.json'))['kernel_us_per_step']*20)"
MADIGAN_LIB_PATH=tools/_var/wallx/libmadigan_hip.so timeout -k 10 120 python bench.py --steps 2000 --warmup 100 --fuse 20 --no-cpu-baseline --no-probe > $O/wallx_f20.json && python -c "import json;print('wallx f20', json.load(open('$O/wallx_f20.json'))['kernel_us_per_step']*20)"
