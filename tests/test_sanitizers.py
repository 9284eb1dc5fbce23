"""Host sanitizer builds (ASan / UBSan on the host code).

`make -B -C oracle sanitize` (always rebuilt from the current sources) builds, with -fsanitize=address,undefined and
-fno-sanitize-recover=all:
  * oracle/_build/sanitize_oracle: the C oracle under a driver that calls
    every entry point of madigan_oracle.h over the parity tests'
    configurations (oracle/sanitize_oracle.c);
  * oracle/_build/sanitize_hdf: the product's HDF replay reader
    (madigan_amd/csrc/mgn_hdf.cpp) under a driver covering the envTest.cpp
    fixture, a multi-asset file, the cache-walk tape and the error paths
    (oracle/sanitize_hdf.cpp; mgn_hdf_stage needs a GPU and is not run).
Any ASan / UBSan finding (or leak) makes the binary exit non-zero.
The device kernels cannot be sanitized on this pool (no GPU ASan / xnack+).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-s", "-B", "-C", ORACLE, "sanitize"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail(f"sanitizer build failed:\n{r.stdout}\n{r.stderr}")
    return os.path.join(ORACLE, "_build")


def _run(exe, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    return subprocess.run([exe, *args], capture_output=True, text=True, env=env, timeout=300)


def test_oracle_clean_under_asan_ubsan(built):
    r = _run(os.path.join(built, "sanitize_oracle"))
    assert r.returncode == 0, r.stderr[-4000:]
    assert "all cases clean" in r.stdout
    assert "runtime error" not in r.stderr


def test_hdf_reader_clean_under_asan_ubsan(built, tmp_path):
    r = _run(os.path.join(built, "sanitize_hdf"), str(tmp_path))
    assert r.returncode == 0, r.stderr[-4000:]
    assert "all cases clean" in r.stdout
    assert "runtime error" not in r.stderr
