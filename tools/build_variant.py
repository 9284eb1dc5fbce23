"""Build a diagnostic variant of libmadigan_hip.so with extra defines.

    python tools/build_variant.py NAME [-DMGN_STAMPS ...]

Recompiles mgn_api.hip and mgn_launch_a8t.hip (the C3 headline kernels) with the
extra flags, links them with the product objects of the other APAD units into
tools/_var/NAME/libmadigan_hip.so; select it with MADIGAN_LIB_PATH.  Development
tool only: the product library is madigan_amd/libmadigan_hip.so.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from madigan_amd import build as B  # noqa: E402


def main():
    name, extra = sys.argv[1], sys.argv[2:]
    B.build()
    out_dir = os.path.join(ROOT, "tools", "_var", name)
    os.makedirs(out_dir, exist_ok=True)
    cc = B.hipcc()
    # the translation units rebuilt with the extra flags (MGN_VARIANT_UNITS,
    # comma-separated unit suffixes: default 8t, the C3 headline's unit)
    units = os.environ.get("MGN_VARIANT_UNITS", "8t").split(",")
    redo = {"mgn_api.hip"} | {f"mgn_launch_a{u}.hip" for u in units}

    def one(src):
        base = os.path.basename(src)
        if base not in redo:
            return os.path.join(B.OBJ, base.replace(".hip", ".o"))
        obj = os.path.join(out_dir, base.replace(".hip", ".o"))
        # (MGN_VARIANT_NO_UNIT_FLAGS=1: without the unit's own flags, e.g. with
        # machine LICM in a unit the product builds without it)
        uf = [] if os.environ.get("MGN_VARIANT_NO_UNIT_FLAGS") else B.UNIT_FLAGS.get(base, [])
        subprocess.run([cc, *B.FLAGS, *uf, "-DMGN_DIAG", *extra, "-c", "-o", obj, src], check=True)
        return obj

    with ThreadPoolExecutor(4) as ex:
        objs = list(ex.map(one, B.sources()))
    lib = os.path.join(out_dir, "libmadigan_hip.so")
    subprocess.run([cc, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib, *objs], check=True)
    print(lib)


if __name__ == "__main__":
    main()
