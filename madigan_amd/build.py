"""Build libmadigan_hip.so in-tree for gfx950 (MI355X).

    python -m madigan_amd.build [--force]

Translation units: mgn_api.hip (C ABI, window/action kernels) plus one
mgn_launch_a<APAD>.hip per padded asset count with that APAD's (M, S)
instantiations of the step kernels; they compile in parallel and link into
one shared library.  Strict IEEE binary64 on the device: -ffp-contract=off, no
fast-math, so the kernels evaluate the same sequence of correctly rounded
operations as the oracle.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libmadigan_hip.so")
OBJ = os.path.join(HERE, "_obj")
ARCH = os.environ.get("MADIGAN_OFFLOAD_ARCH", "gfx950")
# kernarg preload: a kernel's leading scalar / pointer arguments (up to 16
# SGPRs) arrive in SGPRs with the wave instead of through the kernel-argument
# segment (k_step_trio passes its ledger-role pointers first)
FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-fno-fast-math", "-Wall", "-mllvm", "-amdgpu-kernarg-preload-count=6"]
# per-unit flags: the step-kernel units are built without machine-level
# loop-invariant code motion -- it hoisted the math kernels' 64-bit polynomial
# constants out of the step loop, left them live across it at the register
# budget and spilled them to scratch: 87-195 VGPRs in the 256-lane n-step
# kernels, 24-264 in the single-role kernels, 72-91 in the two-role n-step
# kernels, 48 -> 4 in the two-slot layout; without it every one of them
# keeps its registers (tests/test_build.py; the single-role kernel's 4 and 8
# slots per lane, 32 and 64 assets, still spill 14-75).  The C3 headline's unit
# (mgn_launch_a8t.hip, the agent loop's multi-step instantiations at A = 8)
# keeps it: its 20-step launch measured 1-2 % slower without it
# (profiles/r05e_licm20; the one-step launches, mgn_launch_a8k1.hip, 5 %
# faster without it, r05e_licm1).  The n-step instantiations live in units of
# their own (mgn_launch_a{1t,2,4,8,16}nst.hip).
_NO_LICM = ["-mllvm", "-disable-machine-licm"]
UNIT_FLAGS = {f"mgn_launch_{u}.hip": _NO_LICM
              for u in ("a1", "a1t", "a1tnst", "a2", "a2nst", "a4", "a4nst", "a8", "a8k1", "a8k1w", "a8nst", "a16", "a16m2",
                        "a16nst",
                        "a32", "a64")}


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required)")


HDF_OUT = os.path.join(HERE, "libmadigan_hdf.so")
HDF_SRC = os.path.join(CSRC, "mgn_hdf.cpp")
HDF5_PREFIX = os.environ.get("MADIGAN_HDF5_PREFIX", "/opt/conda")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def build_hdf(force: bool = False, verbose: bool = False) -> str:
    """libmadigan_hdf.so: the HDF replay reader / stager (host C++ over libhdf5
    and the HIP runtime; no device code)."""
    deps_ = [HDF_SRC, os.path.join(ROOT, "include", "madigan_hdf.h"),
             os.path.join(ROOT, "include", "madigan_amd.h")]
    if not force and os.path.exists(HDF_OUT) and all(
            os.path.getmtime(d) <= os.path.getmtime(HDF_OUT) for d in deps_):
        return HDF_OUT
    inc, lib = os.path.join(HDF5_PREFIX, "include"), os.path.join(HDF5_PREFIX, "lib")
    if not os.path.exists(os.path.join(inc, "hdf5.h")):
        raise RuntimeError(f"hdf5.h not found under {inc} (set MADIGAN_HDF5_PREFIX)")
    cmd = [shutil.which("g++") or "g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-Wall",
           "-D__HIP_PLATFORM_AMD__", f"-I{inc}", f"-I{ROCM}/include", "-o", HDF_OUT + ".tmp",
           HDF_SRC, f"-L{lib}", "-lhdf5", f"-Wl,-rpath,{lib}", f"-L{ROCM}/lib", "-lamdhip64",
           f"-Wl,-rpath,{ROCM}/lib"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"g++ failed on {HDF_SRC}:\n{r.stderr}")
    os.replace(HDF_OUT + ".tmp", HDF_OUT)
    return HDF_OUT


PYCALL_SRC = os.path.join(CSRC, "mgn_pycall.c")


def pycall_out() -> str:
    import sysconfig
    return os.path.join(HERE, "_mgn_pycall" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_pycall(force: bool = False, verbose: bool = False) -> str:
    """_mgn_pycall: the CPython binding of mgn_rollout (host C, linked against
    the in-tree libmadigan_hip.so, found next to it through $ORIGIN)."""
    import sysconfig
    out = pycall_out()
    deps_ = [PYCALL_SRC, OUT, os.path.join(ROOT, "include", "madigan_amd.h")]
    if not force and os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps_):
        return out
    cmd = [shutil.which("gcc") or "gcc", "-O2", "-fPIC", "-shared", "-Wall",
           f"-I{sysconfig.get_paths()['include']}", f"-I{os.path.join(ROOT, 'include')}",
           "-o", out + ".tmp", PYCALL_SRC, f"-L{HERE}", "-l:libmadigan_hip.so", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"gcc failed on {PYCALL_SRC}:\n{r.stderr}")
    os.replace(out + ".tmp", out)
    return out


def deps():
    return sources() + glob.glob(os.path.join(CSRC, "*.h")) + [
        os.path.join(ROOT, "include", "madigan_amd.h")]


# the compile configuration the library was built with (flags per unit and
# the compiler): a change of FLAGS / UNIT_FLAGS alone rebuilds, so an A/B of a
# flag never measures a stale library
FLAGS_STAMP = os.path.join(OBJ, "flags.txt")
# per kernel: registers, scratch and occupancy as the compiler reports them
# (-Rpass-analysis=kernel-resource-usage), written by every build and read by
# tests/test_build.py (no step kernel may spill to scratch)
RESOURCE_USAGE = os.path.join(OBJ, "resource_usage.json")


def _flags_key() -> str:
    """The build's configuration and inputs: flags per unit, the target and a
    digest of every source and header (content, not mtime: an edit made while
    a build was compiling must not look built)."""
    import hashlib
    units = {os.path.basename(s): UNIT_FLAGS.get(os.path.basename(s), []) for s in sources()}
    h = hashlib.sha256()
    for d in sorted(deps()):
        with open(d, "rb") as f:
            h.update(d.encode() + b"\0" + f.read())
    return repr((FLAGS, sorted(units.items()), ARCH, h.hexdigest()))


def needs_build() -> bool:
    if not os.path.exists(OUT) or not os.path.exists(FLAGS_STAMP) or not os.path.exists(RESOURCE_USAGE):
        return True
    with open(FLAGS_STAMP) as f:
        return f.read() != _flags_key()


def parse_resource_usage(text: str) -> dict:
    """The compiler's kernel-resource-usage remarks -> {kernel: {field: int}}."""
    import re
    out, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"remark: [^:]*:?\s*Function Name: (\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark: .*?(SGPRs|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                      r"SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).split(" [")[0]] = int(m.group(2))
    return out


def build(force: bool = False, verbose: bool = False, jobs: int = 0) -> str:
    build_hdf(force=force, verbose=verbose)
    if not force and not needs_build():
        _optional_pycall(False, verbose)
        return OUT
    os.makedirs(OBJ, exist_ok=True)
    key = _flags_key()  # the inputs as they are when the compiles start
    cc = hipcc()
    jobs = jobs or min(8, os.cpu_count() or 4)

    def compile_one(src):
        obj = os.path.join(OBJ, os.path.basename(src).replace(".hip", ".o"))
        cmd = [cc, *FLAGS, *UNIT_FLAGS.get(os.path.basename(src), []),
               "-Rpass-analysis=kernel-resource-usage", "-c", "-o", obj, src]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr}")
        usage = parse_resource_usage(r.stderr)
        rest = "\n".join(ln for ln in r.stderr.splitlines() if "warning:" in ln).strip()
        if rest and verbose:
            print(rest, file=sys.stderr)
        return obj, os.path.basename(src), usage

    with ThreadPoolExecutor(jobs) as ex:
        res = list(ex.map(compile_one, sources()))
    objs = [r[0] for r in res]
    import json
    with open(RESOURCE_USAGE, "w") as f:
        json.dump({unit: usage for _, unit, usage in res}, f, indent=0, sort_keys=True)
    with open(FLAGS_STAMP, "w") as f:
        f.write(key)
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT + ".tmp", *objs, "-ldl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    _optional_pycall(True, verbose)
    return OUT


def _optional_pycall(force: bool, verbose: bool) -> None:
    # the CPython binding is optional (_lib.pycall falls back to ctypes): a
    # missing gcc / Python.h costs the faster per-launch call, not the build
    try:
        build_pycall(force=force, verbose=verbose)
    except Exception as exc:  # noqa: BLE001
        print(f"warning: _mgn_pycall not built ({exc}); the ctypes binding is used", file=sys.stderr)


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
