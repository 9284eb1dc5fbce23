"""CPU checks of the product build (madigan_amd/build.py): the library is
rebuilt when only its flags change, and the step kernels keep their registers
-- no spill to scratch -- as the compiler reports them
(-Rpass-analysis=kernel-resource-usage, recorded by every build in
madigan_amd/_obj/resource_usage.json).  The step units other than A = 8 are
built without machine LICM (build.UNIT_FLAGS), which kept their math constants
from being hoisted out of the step loop and spilled (87-264 VGPRs in the n-step,
two-role n-step and single-role kernels); a compiler update that re-spills them
fails here rather than only measuring slower."""
import json
import os
import re

import pytest

from madigan_amd import build as B


def _hipcc_or_skip():
    try:
        return B.hipcc()
    except RuntimeError as e:
        pytest.skip(f"no ROCm toolchain here: {e}")


@pytest.fixture(scope="module")
def usage():
    _hipcc_or_skip()
    if not os.path.exists(B.RESOURCE_USAGE):
        # (a checkout that has not run build(): nothing to check yet; the
        # driver's build step writes the report)
        pytest.skip(f"{B.RESOURCE_USAGE} missing: the library has not been built "
                    "(python -c 'import __graft_entry__ as g; g.build()')")
    with open(B.RESOURCE_USAGE) as f:
        return json.load(f)


def _kernels(usage, unit, pattern):
    rx = re.compile(pattern)
    return {k: v for k, v in usage[unit].items() if rx.search(k)}


# (unit, mangled-name pattern, the most VGPRs the kernels may spill, why)
_NO_LICM_UNITS = sorted(B.UNIT_FLAGS)
CASES = [
    # k_step_trio<S, RQ1, DISC=true, OMC in {O_STD = 4093, O_ALL = 16383}, ...>: the
    # agent loop's instantiations, the C3 headline among them (S = 8, GK = TrendOU)
    # (the multi-step instantiations: ONE = K1 = false, the name's last two flags)
    ("mgn_launch_a8t.hip", r"k_step_trioILi8ELb[01]ELb1ELj(4093|16383)E.*ELb0ELb0EEEv", 0, "C3 headline"),
    # the one-step instantiations (K1), their own unit
    ("mgn_launch_a8k1.hip", r"k_step_trioILi8ELb[01]ELb1ELj(4093|16383)E.*ELb0ELb1EEEv", 0, "C3 one-step launches"),
    # the two-slot layout's window instantiations (C5's): 48 -> 2 in round 4
    ("mgn_launch_a16m2.hip", r"k_step_trio", 2, "two slots per lane"),
    # the one-step launches of large batches at four waves per SIMD (128
    # VGPRs; the measured layout spills 16-20, mgn_launch_a8k1w.hip)
    ("mgn_launch_a8k1w.hip", r"k_step_trio", 24, "one-step launches, four waves per SIMD"),
    # the single-role kernel's 4 and 8 slots per lane (32 / 64 assets)
    ("mgn_launch_a32.hip", r"k_stepILi4E", 32, "single-role, 4 slots per lane"),
    ("mgn_launch_a64.hip", r"k_stepILi[48]E", 80, "single-role, 4 / 8 slots per lane"),
] + [(u, r"k_step(_trio|_duo|ILi[12]E)", 0, "built without machine LICM")
     for u in _NO_LICM_UNITS if u not in ("mgn_launch_a16m2.hip", "mgn_launch_a64.hip", "mgn_launch_a8k1w.hip")]


@pytest.mark.parametrize("unit,pattern,max_spill,what", CASES)
def test_step_kernels_do_not_spill(usage, unit, pattern, max_spill, what):
    ks = _kernels(usage, unit, pattern)
    assert ks, f"{what}: no kernel matching {pattern} in {unit}"
    for name, v in ks.items():
        assert v["VGPRs Spill"] <= max_spill, f"{what}: {name} spills {v['VGPRs Spill']} VGPRs"
        # three waves per SIMD: the three-role kernel's 768-thread workgroup
        # (four in the wide one-step unit)
        if unit == "mgn_launch_a8k1w.hip":
            assert v["Occupancy"] >= 4, f"{what}: {name} occupancy {v['Occupancy']}"
        if "Li256E" in name:
            assert v["Occupancy"] >= 3, f"{what}: {name} occupancy {v['Occupancy']}"


def test_flag_change_rebuilds(monkeypatch):
    _hipcc_or_skip()
    if not os.path.exists(B.FLAGS_STAMP):
        pytest.skip("the library has not been built")
    if B.needs_build():
        pytest.skip("the library is out of date (its inputs changed since the build)")
    monkeypatch.setattr(B, "FLAGS", B.FLAGS + ["-DMGN_UNUSED_FLAG"])
    assert B.needs_build(), "a flag change alone must rebuild"
    monkeypatch.setattr(B, "UNIT_FLAGS", {})
    monkeypatch.setattr(B, "FLAGS", [f for f in B.FLAGS if f != "-DMGN_UNUSED_FLAG"])
    assert B.needs_build(), "a unit-flag change alone must rebuild"


def test_diag_switches_refused_without_diag(tmp_path):
    """Stamp / ablation switches compile only in diagnostic builds (mgn_diag.h)."""
    import subprocess
    cc = _hipcc_or_skip()
    src = tmp_path / "t.hip"
    src.write_text('#include "mgn_diag.h"\n')
    r = subprocess.run([cc, "--offload-arch=gfx950", "-fsyntax-only", "-DMGN_TRIO_ABL_G",
                        f"-I{B.CSRC}", str(src)], capture_output=True, text=True)
    assert r.returncode != 0 and "diagnostic builds" in r.stderr
    r = subprocess.run([cc, "--offload-arch=gfx950", "-fsyntax-only", "-DMGN_TRIO_ABL_G", "-DMGN_DIAG",
                        f"-I{B.CSRC}", str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
