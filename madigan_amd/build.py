"""Build libmadigan_hip.so in-tree for gfx950 (MI355X).

    python -m madigan_amd.build [--force]

Strict IEEE binary64 on the device: -ffp-contract=off, no fast-math, so the
kernels' arithmetic is the same sequence of correctly rounded operations the
oracle evaluates.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "mgn_api.hip")
DEPS = [os.path.join(HERE, "csrc", f) for f in ("mgn_api.hip", "mgn_kernels.h", "mgn_math.h")] + [
    os.path.join(ROOT, "include", "madigan_amd.h")]
OUT = os.path.join(HERE, "libmadigan_hip.so")
ARCH = os.environ.get("MADIGAN_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required)")


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return OUT
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ffp-contract=off", "-fno-fast-math", "-Wall", "-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
