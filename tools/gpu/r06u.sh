set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_variants.py tests/test_gpu_reference_shape.py tests/test_gpu_nstep_running.py > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest.txt | head; tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
