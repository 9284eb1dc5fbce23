#!/bin/bash
# layout / batch-size sweep of the fused step (diagnostic): NS / LS override the lists
cd "$(dirname "$0")/.."
for N in ${NS:-8192 65536 262144}; do
  for L in ${LS:-1 2 4 8}; do
    N=$N LAYOUT=$L timeout -k 10 120 python tools/ablate.py || exit 1
  done
done
