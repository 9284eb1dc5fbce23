#!/bin/bash
# time the C3 bench under the product library and each tools/_var/<name> build
# (run on the GPU box from the repo root): tools/vartime.sh v1 v2 ...
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --steps 2048 --warmup 256 --no-cpu-baseline"
for rep in 1 2; do
  timeout -k 10 120 $B > gpurun_out/var_prod.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/var_prod.json'));print('prod', round(d['value']/1e9,4), round(d['roofline']['avg_launch_us'],1))"
  for v in "$@"; do
    MADIGAN_LIB_PATH=tools/_var/$v/libmadigan_hip.so timeout -k 10 120 $B > gpurun_out/var_$v.json || exit 1
    python -c "import json;d=json.load(open('gpurun_out/var_$v.json'));print('$v', round(d['value']/1e9,4), round(d['roofline']['avg_launch_us'],1))"
  done
done
