#!/bin/bash
# n-step instantiations in their own unit (LICM off): GPU suite, fuzz, A/B against the previous build
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/nstunit
timeout -k 10 800 python -u -m pytest -v --timeout 180 --timeout-method thread -p no:cacheprovider -m gpu tests > gpurun_out/nstunit/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/nstunit/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/nstunit/smoke.log 2>&1 || { tail -20 gpurun_out/nstunit/smoke.log; exit 1; }
tail -1 gpurun_out/nstunit/smoke.log
timeout -k 10 300 python -u tools/fuzz_trio.py 120 41 > gpurun_out/nstunit/fuzz.log 2>&1 || { tail -5 gpurun_out/nstunit/fuzz.log; exit 1; }
tail -1 gpurun_out/nstunit/fuzz.log
VARIANTS="prev=tools/_var/prev/libmadigan_hip.so new=base" SHAPES="n20 C3_20 C3_256 k1" R=2 TAG=abnstunit bash tools/gpu_r04_ab_gen.sh
timeout -k 10 300 python bench.py --steps 512 --warmup 64 --fuse 64 --nstep 20 --no-cpu-baseline --no-probe --no-k-sweep > gpurun_out/nstunit/bench_nstep20.json 2> gpurun_out/nstunit/bench_nstep20.err || { tail -5 gpurun_out/nstunit/bench_nstep20.err; exit 1; }
echo nstunit done
