#!/bin/bash
# One evidence pass on the GPU box (TAG names the output directory):
#   SUITE=1  the GPU test suite (-m gpu; PYK: a -k expression) and smoke()
#   DRV=1    the driver's bench line (--steps 20 --warmup 5) and the same
#            command under rocprofv3 --kernel-trace --stats
#   EXTRA    further bench lines: "name|args;name|args" (each also traced when
#            TRACE=1)
# Every GPU step runs under its own time limit; the first failure ends the pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pass}
mkdir -p $O
if [ -n "$SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYK:+-k "$PYK"} \
    > $O/pytest_gpu.txt 2>&1 || { echo "gpu suite failed"; grep -E "FAILED|Error|error" $O/pytest_gpu.txt | head -20; tail -30 $O/pytest_gpu.txt; exit 1; }
  tail -2 $O/pytest_gpu.txt
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
  tail -1 $O/smoke.txt
fi
line() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -20 $O/$n.err; exit 1; }
  python tools/bench_brief.py $O/$n.json
  if [ -n "$TRACE" ]; then
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$n -o kt -- python3 bench.py "$@" \
      > $O/kt_$n.json 2> $O/kt_$n.log || { echo "$n trace failed"; tail -20 $O/kt_$n.log; exit 1; }
    python tools/kt_brief.py $O/kt_$n
    python tools/bench_brief.py $O/kt_$n.json
    # the un-profiled line against the trace (profiled launch events read longer)
    if grep -q launch_log $O/kt_$n.json; then
      python tools/reconcile.py $O/$n.json $O/kt_$n --trace-line $O/kt_$n.json --out $O/reconcile_$n.json
    fi
  fi
}
if [ -n "$DRV" ]; then
  line drv --gpus 1 --steps 20 --warmup 5
fi
if [ -n "$EXTRA" ]; then
  IFS=';' read -ra XS <<< "$EXTRA"
  for x in "${XS[@]}"; do
    n=${x%%|*}; a=${x#*|}
    line $n $a
  done
fi
echo "$O done"
